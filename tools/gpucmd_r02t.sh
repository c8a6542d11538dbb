#!/bin/bash
# Round-2 closing check at HEAD: GPU suite, smoke(), the driver's bench command.
set -o pipefail
OUT=gpurun_out/r02t
mkdir -p $OUT
echo "[$(date +%T)] gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.txt 2>&1
rc=$?; tail -3 $OUT/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
echo "[$(date +%T)] smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || exit $?
tail -1 $OUT/smoke.txt
echo "[$(date +%T)] bench"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
cat $OUT/bench_c2.json
echo "[$(date +%T)] done"
