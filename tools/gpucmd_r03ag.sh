#!/bin/bash
# Round 3: C5 ablation of the round-3 generic-rollout changes (deferred fold ring depth
# 8 / 4 / off, window rows in flight per thread, wave 0 writing records) vs HEAD's lib.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03ag
mkdir -p $OUT
for rep in 1 2; do
for v in "" _prev _fold4 _fold0 _u1 _now0; do
  MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 200 python3 bench.py --config c5 --cpu-seconds 0 \
    --per-step-steps 0 --no-gather > $OUT/c5$v.json 2> $OUT/c5$v.err || { tail -20 $OUT/c5$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c5$v.json')); print('c5 lib$v', d['kernel_ms_per_launch'], d['timing']['kernel_ms_replays'])"
done
done
