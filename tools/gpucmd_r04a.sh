#!/bin/bash
# Round 4, first GPU call: A/B measurements first (diagnostic builds), then the full GPU
# suite and the driver's bench line.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04a
mkdir -p $OUT
L=mapf-marl_amd/mapfx
# LDS-traffic ablations of the C2 split kernel (diagnostic builds, results garbage):
# 2048 step wave writes the info chunk only; 65536 store waves read one chunk;
# 131072 step wave reads 3 window rows; 262144 store waves read the rows from the map
bash tools/ab_bench.sh $OUT/ab 2 "--gpus 1 --steps 20 --warmup 5" $L/libmapfx.so $L/libmapfx_ab2048.so \
  $L/libmapfx_ab65536.so $L/libmapfx_ab131072.so $L/libmapfx_ab262144.so || exit 1
# C5: 16-byte occupancy groups + readlane edge scan + fold priority vs round 3's kernel
bash tools/ab_bench.sh $OUT/ab_c5 2 "--config c5 --gpus 1" $L/libmapfx.so $L/libmapfx_occrows.so \
  $L/libmapfx_r3base.so || exit 1
# MARL_PARTIAL per-step kernel: envs per wave 4 (default) / 2 / 1 (more waves per SIMD)
for epw in 4 2 1 4 2 1; do
  MAPFX_PARTIAL_EPW=$epw timeout -k 10 200 python3 bench.py --env marl_partial --cpu-seconds 0 \
    > $OUT/partial_epw$epw.json 2> $OUT/partial_epw$epw.err || { tail -20 $OUT/partial_epw$epw.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/partial_epw$epw.json')); print('partial EPW $epw', d['kernel_ms_per_step'], d['roofline']['frac'])"
done
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $OUT/tests.txt 2>&1 || { grep -E "FAIL|Error|error" $OUT/tests.txt | head -30; tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c2.json 2> $OUT/bench_c2.err \
  || { tail -20 $OUT/bench_c2.err; exit 1; }
tail -c 600 $OUT/bench_c2.json; echo
