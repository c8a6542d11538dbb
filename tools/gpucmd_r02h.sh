#!/bin/bash
# round-2 call h: runner (F2) + drop-in single-sync tests, full GPU suite, runner / partial bench.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02h
mkdir -p $OUT
echo "[$(date +%T)] runner + drop-in tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_runner.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "runner or dropin" > $OUT/tests_new.log 2>&1
rc=$?
tail -15 $OUT/tests_new.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
echo "[$(date +%T)] full gpu suite"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -5 $OUT/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
echo "[$(date +%T)] runner bench"
timeout -k 10 300 python3 bench.py --env runner --steps 500 --warmup 100 --cpu-seconds 0 > $OUT/bench_runner.json 2> $OUT/bench_runner.err || exit $?
cat $OUT/bench_runner.json
timeout -k 10 300 python3 bench.py --env marl_partial --steps 500 --warmup 100 --cpu-seconds 0 > $OUT/bench_partial.json 2> $OUT/bench_partial.err || exit $?
cat $OUT/bench_partial.json
echo "[$(date +%T)] done"
