#!/bin/bash
# Round 3: record stores of register data (no staged-record LDS read, 32768) vs
# no record stores (16384) vs shipped.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03p
mkdir -p $OUT
for rep in 1 2; do
for v in "" _abl32768 _abl16384; do
  for T in 20 64; do
    MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 120 python3 bench.py --gpus 1 --steps $T --warmup $T \
      --cpu-seconds 0 --per-step-steps 0 > $OUT/c2$v.T$T.json 2>$OUT/c2$v.T$T.err || exit $?
    python3 -c "import json; d=json.load(open('$OUT/c2$v.T$T.json')); print('lib$v T$T', d['kernel_ms_per_launch'], d['timing']['kernel_ms_replays'])"
  done
done
done
echo "[$(date +%T)] done"
