#!/bin/bash
# Round 3: C2 rollout length sweep (T = 1, 4, 20, 64) of the shipped split kernel, the
# store waves ablated (256) and the store waves' global stores ablated (512):
# separates the prologue, the step-wave chain and the HBM store stream.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03f
mkdir -p $OUT
for v in "" _abl256 _abl512; do
  for T in 1 4 20 64; do
    MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 120 python3 bench.py --gpus 1 --steps $T --warmup $T \
      --cpu-seconds 0 --per-step-steps 0 > $OUT/c2$v.T$T.json 2>$OUT/c2$v.T$T.err || exit $?
    python3 -c "import json; d=json.load(open('$OUT/c2$v.T$T.json')); print('lib$v T$T', d['kernel_ms_per_launch'], d['timing']['kernel_ms_replays'])"
  done
done
echo "[$(date +%T)] done"
