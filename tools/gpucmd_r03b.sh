#!/bin/bash
# Round 3: GPU suite at HEAD, then the driver's bench line and the PRIMAL leg.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03b
mkdir -p $OUT
echo "[$(date +%T)] gpu tests"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.txt 2>&1
rc=$?; tail -5 $OUT/gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
echo "[$(date +%T)] bench c2"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
echo "[$(date +%T)] bench primal"
timeout -k 10 300 python3 bench.py --env primal > $OUT/bench_primal.json 2> $OUT/bench_primal.err || exit $?
tail -c 400 $OUT/bench_primal.json
echo "[$(date +%T)] done"
