#!/bin/bash
# Round 3: C5 A/B of the shipped lib vs libmapfx_exp.so (edge-scan candidates by
# readlane, fold chain at s_setprio 3; built from a patched copy, not shipped).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03al
mkdir -p $OUT
for rep in 1 2; do
for v in "" _exp; do
  MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 200 python3 bench.py --config c5 --cpu-seconds 0 \
    --per-step-steps 0 --no-gather > $OUT/c5$v.json 2> $OUT/c5$v.err || { tail -20 $OUT/c5$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c5$v.json')); print('c5 lib$v', d['kernel_ms_per_launch'], d['timing']['kernel_ms_replays'])"
done
done
