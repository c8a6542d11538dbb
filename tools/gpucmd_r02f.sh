#!/bin/bash
# round-2 call f: parity after the cell-format / fast-build change, stamps, bench.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02f
mkdir -p $OUT
echo "[$(date +%T)] gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -15 $OUT/tests.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 200 python3 tools/pstamps.py --envs 64,4096 --T 20 > $OUT/pstamps.txt 2>&1 || exit $?
cat $OUT/pstamps.txt
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/bench$i.json 2> $OUT/bench$i.err || exit $?
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 512 --warmup 64 --cpu-seconds 0 --per-step-steps 0 > $OUT/bench_t64.json 2> $OUT/bench_t64.err || exit $?
for c in c1 c3; do
timeout -k 10 300 python3 bench.py --config $c --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit $?
done
echo "[$(date +%T)] done"
