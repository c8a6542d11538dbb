#!/bin/bash
# Round 4: the two-map split kernel (MAPFX_SPLIT_DBM) -- split-path parity (every step
# against single-step launches, the long-horizon oracle run, autoreset, the gather
# tests), then A/B against the same build without it at T = 20 and T = 64.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04e
mkdir -p $OUT
L=mapf-marl_amd/mapfx
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_runner.py -x -q \
  --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1 || { grep -E "FAIL|Error" $OUT/tests.txt | head -30; tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
bash tools/ab_bench.sh $OUT/ab20 3 "--gpus 1 --steps 20 --warmup 5" $L/libmapfx.so $L/libmapfx_nodbm.so || exit 1
bash tools/ab_bench.sh $OUT/ab64 2 "--gpus 1 --steps 512 --warmup 64" $L/libmapfx.so $L/libmapfx_nodbm.so || exit 1
