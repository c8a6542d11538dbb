#!/bin/bash
# Round-2 closing records at HEAD: GPU suite, smoke(), the driver's bench command,
# the PRIMAL leg with its CPU baseline and a kernel trace of it.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r02u
mkdir -p $OUT
echo "[$(date +%T)] gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.txt 2>&1
rc=$?; tail -3 $OUT/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
echo "[$(date +%T)] smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || exit $?
tail -1 $OUT/smoke.txt
echo "[$(date +%T)] bench c2"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
echo "[$(date +%T)] bench primal"
timeout -k 10 300 python3 bench.py --env primal > $OUT/bench_primal.json 2> $OUT/bench_primal.err || exit $?
cat $OUT/bench_primal.json
echo "[$(date +%T)] primal kernel trace"
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/primal_trace -o run --output-format csv \
  -- python3 $R/bench.py --env primal --cpu-seconds 0 > $OUT/bench_primal_traced.json 2> $OUT/primal_trace.err || exit $?
echo "[$(date +%T)] done"
