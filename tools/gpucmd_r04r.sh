#!/bin/bash
# Round 4: split kernel with an 8-step action block for T <= 32 -- parity, A/B at T = 20 / 64.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04r
mkdir -p $OUT
L=mapf-marl_amd/mapfx
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_runner.py -x -q \
  --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1 || { grep -E "FAIL|Error" $OUT/tests.txt | head -30; tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
bash tools/ab_bench.sh $OUT/ab20 3 "--gpus 1 --steps 20 --warmup 5" $L/libmapfx.so $L/libmapfx_prev.so $L/libmapfx_ab8.so || exit 1
bash tools/ab_bench.sh $OUT/ab64 2 "--gpus 1 --steps 512 --warmup 64" $L/libmapfx.so $L/libmapfx_prev.so || exit 1
