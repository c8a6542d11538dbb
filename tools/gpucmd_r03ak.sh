#!/bin/bash
# Round 3: edge scan candidates by readlane, fold chain at s_setprio 3: generic-rollout
# parity tests, C5 A/B vs the previous commit and without the priority, C5 stamps.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03ak
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "rollout or stacked or invalid or autoreset or edge" > $OUT/tests.txt 2>&1 || { tail -40 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
for rep in 1 2; do
for v in "" _prev _noprio; do
  MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 200 python3 bench.py --config c5 --cpu-seconds 0 \
    --per-step-steps 0 --no-gather > $OUT/c5$v.json 2> $OUT/c5$v.err || { tail -20 $OUT/c5$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c5$v.json')); print('c5 lib$v', d['kernel_ms_per_launch'], d['timing']['kernel_ms_replays'])"
done
done
timeout -k 10 200 python3 tools/stamps_c5.py > $OUT/stamps.txt 2>&1 || { tail -20 $OUT/stamps.txt; exit 1; }
cat $OUT/stamps.txt
