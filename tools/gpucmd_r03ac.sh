#!/bin/bash
# Round 3: where the C5 generic rollout kernel's time goes (MAPFX_GABL ablations:
# 1 no reward fold, 2 no window records, 3 neither, 8 no edge scan), T = 64 (bench default).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03ac
mkdir -p $OUT
for rep in 1 2; do
for v in "" _gabl1 _gabl2 _gabl3 _gabl8; do
  MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 200 python3 bench.py --config c5 --cpu-seconds 0 \
    --per-step-steps 0 --no-gather > $OUT/c5$v.json 2> $OUT/c5$v.err || { tail -20 $OUT/c5$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c5$v.json')); print('lib$v', d['kernel_ms_per_launch'], d['timing']['kernel_ms_replays'])"
done
done
