#!/bin/bash
# Round 3, first check: the whole GPU suite at HEAD (new: tiled runner at B=4096/1100,
# exact edge counts at N=256/300, trajectory pinning), then the driver's bench line.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03a
mkdir -p $OUT
echo "[$(date +%T)] gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.txt 2>&1
rc=$?; tail -5 $OUT/gpu_tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
echo "[$(date +%T)] bench c2"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
tail -c 600 $OUT/bench_c2.json
echo "[$(date +%T)] done"
