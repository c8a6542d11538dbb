#!/bin/bash
# Round 3: PRIMAL seq kernel with snapshot-only phase A, C5 edge scan by ballot popcounts;
# GPU tests of both, then A/B against the previous commit's library (libmapfx_prev.so).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03ad
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_primal.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  > $OUT/tests.txt 2>&1 || { tail -40 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
for rep in 1 2; do
for v in "" _prev; do
  MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 200 python3 bench.py --env primal --cpu-seconds 0 \
    > $OUT/primal$v.json 2> $OUT/primal$v.err || { tail -20 $OUT/primal$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/primal$v.json')); print('primal lib$v', d['kernel_ms_per_launch'])"
  MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 200 python3 bench.py --config c5 --cpu-seconds 0 \
    --per-step-steps 0 --no-gather > $OUT/c5$v.json 2> $OUT/c5$v.err || { tail -20 $OUT/c5$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c5$v.json')); print('c5 lib$v', d['kernel_ms_per_launch'])"
done
done
