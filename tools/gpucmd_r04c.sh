#!/bin/bash
# Round 4: the lagged step-image ring (MAPFX_SPLIT_LAG) -- rollout parity, then A/B
# against the same build without it at the driver's T = 20 and at T = 64.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04c
mkdir -p $OUT
L=mapf-marl_amd/mapfx
timeout -k 10 800 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_runner.py tests/test_gpu_partial.py tests/test_partial_output_mode.py -x -q --timeout 300 \
  --timeout-method thread > $OUT/tests.txt 2>&1 || { grep -E "FAIL|Error" $OUT/tests.txt | head -30; tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
bash tools/ab_bench.sh $OUT/ab20 3 "--gpus 1 --steps 20 --warmup 5" $L/libmapfx.so $L/libmapfx_nolag.so || exit 1
bash tools/ab_bench.sh $OUT/ab64 2 "--gpus 1 --steps 512 --warmup 64" $L/libmapfx.so $L/libmapfx_nolag.so || exit 1
# C5: carried neighbour bits (no B1) vs without
bash tools/ab_bench.sh $OUT/ab_c5 2 "--config c5 --gpus 1" $L/libmapfx.so $L/libmapfx_nocarry.so || exit 1
