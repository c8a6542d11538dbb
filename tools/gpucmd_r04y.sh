#!/bin/bash
# Round 4: C5 A/B of the generic rollout's fold ring depth (4 / 8 / 16) and occupancy rows
# in flight (MAPFX_OCC_U 0 / 1).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04y
L=mapf-marl_amd/mapfx
bash tools/ab_bench.sh $OUT/ab_c5 2 "--config c5 --gpus 1" $L/libmapfx.so $L/libmapfx_foldr16.so $L/libmapfx_foldr4.so \
  $L/libmapfx_occu0.so || exit 1
