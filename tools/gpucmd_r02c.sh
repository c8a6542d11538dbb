#!/bin/bash
# round-2 call c: parity after the action-prefetch change, timing probe, driver bench.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02c
mkdir -p $OUT
echo "[$(date +%T)] gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
echo "[$(date +%T)] wall probe"
timeout -k 10 300 python3 tools/wall_probe.py > $OUT/wall_probe.json 2> $OUT/wall_probe.err || exit $?
echo "[$(date +%T)] bench"
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/bench$i.json 2> $OUT/bench$i.err || exit $?
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 512 --warmup 64 --cpu-seconds 0 --per-step-steps 0 > $OUT/bench_t64.json 2> $OUT/bench_t64.err || exit $?
echo "[$(date +%T)] done"
