#!/bin/bash
# round-2 call g: parity after the bitmap prefetch, stamps (kernarg placement A/B), bench.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02g
mkdir -p $OUT
echo "[$(date +%T)] gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 200 python3 tools/pstamps.py --envs 4096 --T 20 > $OUT/pstamps.txt 2>&1 || exit $?
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python3 tools/pstamps.py --envs 4096 --T 20 > $OUT/pstamps_devka1.txt 2>&1 || exit $?
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 200 python3 tools/pstamps.py --envs 4096 --T 20 > $OUT/pstamps_devka0.txt 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/bench$i.json 2> $OUT/bench$i.err || exit $?
done
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/bench_devka1.json 2> $OUT/bench_devka1.err || exit $?
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/bench_devka0.json 2> $OUT/bench_devka0.err || exit $?
echo "[$(date +%T)] done"
