#!/bin/bash
# Round 3: what of the store waves slows the step wave: SWAR VALU (4096 keeps the
# staging writes, drops the SWAR), staging LDS writes (8192 keeps the VALU, one
# write), global stores (512), everything (256), info-only images (2048).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03m
mkdir -p $OUT
for rep in 1 2; do
for v in "" _abl256 _abl512 _abl2048 _abl4096 _abl8192; do
  for T in 20 64; do
    MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 120 python3 bench.py --gpus 1 --steps $T --warmup $T \
      --cpu-seconds 0 --per-step-steps 0 > $OUT/c2$v.T$T.json 2>$OUT/c2$v.T$T.err || exit $?
    python3 -c "import json; d=json.load(open('$OUT/c2$v.T$T.json')); print('lib$v T$T', d['kernel_ms_per_launch'], d['timing']['kernel_ms_replays'])"
  done
done
done
echo "[$(date +%T)] done"
