#!/bin/bash
# Round 4: C2 (driver shape, T = 20) A/B of split-kernel tunables: action block 8 / 32,
# store-wave priority 1, step-wave priority 2.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04p
L=mapf-marl_amd/mapfx
bash tools/ab_bench.sh $OUT/ab20 3 "--gpus 1 --steps 20 --warmup 5" $L/libmapfx.so $L/libmapfx_ab8.so $L/libmapfx_ab32.so \
  $L/libmapfx_prst1.so $L/libmapfx_prstep2.so || exit 1
