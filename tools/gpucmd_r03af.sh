#!/bin/bash
# Round 3: C5 deferred fold (code ring), ballot-popcount edge scan, batched window rows; GPU suite, A/B vs HEAD lib


set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03af
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $OUT/tests.txt 2>&1 || { tail -40 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
for rep in 1 2; do
for v in "" _prev; do
  MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 200 python3 bench.py --config c5 --cpu-seconds 0 \
    --per-step-steps 0 --no-gather > $OUT/c5$v.json 2> $OUT/c5$v.err || { tail -20 $OUT/c5$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c5$v.json')); print('c5 lib$v', d['kernel_ms_per_launch'], d['timing']['kernel_ms_replays'], d['roofline']['frac'])"
done
done
