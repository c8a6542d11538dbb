#!/bin/bash
# Round 4: A/B of the MARL_PARTIAL kernel (this round's vs round 3's) and of the per-step
# drop-in kernel's record stores (staged 16-byte vs direct).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
# MARL_PARTIAL: this round's kernel vs round 3's (carried goal distance, early lookups)
mkdir -p $O/r04b_runner; bash tools/ab_bench.sh $O/r04b_pab 2 "--env marl_partial" mapf-marl_amd/mapfx/libmapfx.so \
  mapf-marl_amd/mapfx/libmapfx_oldpartial.so || true
# per-step drop-in kernel: records staged in LDS + 16-byte stores (MAPFX_DIRECT_REC=0) vs direct
bash tools/ab_bench.sh $O/r04b_stepab 2 "--gpus 1 --steps 20 --warmup 5 --per-step-steps 200" \
  mapf-marl_amd/mapfx/libmapfx.so mapf-marl_amd/mapfx/libmapfx_stagerec.so || true
