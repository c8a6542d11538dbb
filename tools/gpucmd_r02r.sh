#!/bin/bash
# round-2 call r: kernarg preload of the hot pointers -- full GPU suite, bench lines.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02r
mkdir -p $OUT
echo "[$(date +%T)] gpu tests"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
echo "[$(date +%T)] c2 driver flags"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/c2.json 2> $OUT/c2.err || exit $?
cat $OUT/c2.json
echo "[$(date +%T)] c5"
timeout -k 10 300 python3 bench.py --config c5 --gpus 1 --cpu-seconds 0 > $OUT/c5.json 2> $OUT/c5.err || exit $?
cat $OUT/c5.json
