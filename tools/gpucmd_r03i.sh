#!/bin/bash
# Round 3: wave priorities of the split (the step wave is now the critical chain).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03i
mkdir -p $OUT
for rep in 1 2; do
for v in "" _prio_step3 _prio0; do
  for T in 20 64; do
    MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 120 python3 bench.py --gpus 1 --steps $T --warmup $T \
      --cpu-seconds 0 --per-step-steps 0 > $OUT/c2$v.T$T.json 2>$OUT/c2$v.T$T.err || exit $?
    python3 -c "import json; d=json.load(open('$OUT/c2$v.T$T.json')); print('lib$v T$T', d['kernel_ms_per_launch'], d['timing']['kernel_ms_replays'])"
  done
done
done
MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx_stamps_ps3.so MAPFX_PROBE_E=4096 timeout -k 10 120 python3 tools/stamps.py || exit $?
echo "[$(date +%T)] done"
