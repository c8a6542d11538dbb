#!/bin/bash
# Round 4: split kernel with an first action block issued before the bitmap prefetch -- parity, A/B at T = 20 / 64.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04t
mkdir -p $OUT
L=mapf-marl_amd/mapfx
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_runner.py -x -q \
  --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1 || { grep -E "FAIL|Error" $OUT/tests.txt | head -30; tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
bash tools/ab_bench.sh $OUT/ab20 3 "--gpus 1 --steps 20 --warmup 5" $L/libmapfx.so $L/libmapfx_prev.so || exit 1
bash tools/ab_bench.sh $OUT/ab64 2 "--gpus 1 --steps 512 --warmup 64" $L/libmapfx.so $L/libmapfx_prev.so || exit 1
bash tools/ab_bench.sh $OUT/abc3 2 "--config c3 --gpus 1" $L/libmapfx.so $L/libmapfx_prev.so || exit 1
MAPFX_PROBE_T=20 timeout -k 10 120 python3 tools/stamps.py > $OUT/c2_stamps_t20.txt 2>&1 && head -3 $OUT/c2_stamps_t20.txt
