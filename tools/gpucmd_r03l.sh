#!/bin/bash
# Round 3: split-kernel ablations: no hand-over barrier (1024), + idle store waves
# (1280), info-only images (2048), idle store waves (256).  Timing only.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03l
mkdir -p $OUT
for v in "" _abl256 _abl1024 _abl1280 _abl2048; do
  for T in 20 64; do
    MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 120 python3 bench.py --gpus 1 --steps $T --warmup $T \
      --cpu-seconds 0 --per-step-steps 0 > $OUT/c2$v.T$T.json 2>$OUT/c2$v.T$T.err || exit $?
    python3 -c "import json; d=json.load(open('$OUT/c2$v.T$T.json')); print('lib$v T$T', d['kernel_ms_per_launch'], d['timing']['kernel_ms_replays'])"
  done
done
echo "[$(date +%T)] done"
