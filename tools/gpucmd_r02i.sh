#!/bin/bash
# round-2 call i: runner + drop-in tests, runner bench (one-call step).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02i
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_runner.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "runner or dropin" > $OUT/tests_new.log 2>&1
rc=$?
tail -3 $OUT/tests_new.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
for i in 1 2; do
timeout -k 10 300 python3 bench.py --env runner --steps 500 --warmup 100 --cpu-seconds 0 > $OUT/bench_runner$i.json 2> $OUT/bench_runner$i.err || exit $?
cut -c1-300 $OUT/bench_runner$i.json
done
