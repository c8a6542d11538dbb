#!/bin/bash
# Round 4: C2 action block size (MAPFX_AB) 16 / 8 / 4 / 2 at T = 20 and 64.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04q
L=mapf-marl_amd/mapfx
bash tools/ab_bench.sh $OUT/ab20 2 "--gpus 1 --steps 20 --warmup 5" $L/libmapfx.so $L/libmapfx_ab8.so $L/libmapfx_ab4.so \
  || exit 1
bash tools/ab_bench.sh $OUT/ab64 2 "--gpus 1 --steps 512 --warmup 64" $L/libmapfx.so $L/libmapfx_ab8.so $L/libmapfx_ab4.so || exit 1
