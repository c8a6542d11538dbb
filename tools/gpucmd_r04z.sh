#!/bin/bash
# Round 4: MARL_PARTIAL with the step's results stored before the observation rows are
# built -- parity, A/B against the late write-back, runner line.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04z
mkdir -p $OUT
L=mapf-marl_amd/mapfx
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_partial.py tests/test_gpu_partial_full_range.py tests/test_gpu_runner.py \
  tests/test_partial_output_mode.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1 \
  || { grep -E "FAIL|Error" $OUT/tests.txt | head -30; tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
bash tools/ab_bench.sh $OUT/ab 3 "--env marl_partial" $L/libmapfx.so $L/libmapfx_latewb.so || exit 1
