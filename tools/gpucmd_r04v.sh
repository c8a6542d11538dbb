#!/bin/bash
# Round 4: C2 A/B of the XCD-aware block renumbering (MAPFX_XCD=0 vs shipped).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04v
L=mapf-marl_amd/mapfx
bash tools/ab_bench.sh $OUT/ab20 3 "--gpus 1 --steps 20 --warmup 5" $L/libmapfx.so $L/libmapfx_xcd0.so || exit 1
bash tools/ab_bench.sh $OUT/ab64 2 "--gpus 1 --steps 512 --warmup 64" $L/libmapfx.so $L/libmapfx_xcd0.so || exit 1
