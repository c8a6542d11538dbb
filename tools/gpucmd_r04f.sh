#!/bin/bash
# Round 4: MARL_PARTIAL with every state load issued up front -- partial / runner parity,
# the per-phase stamps, A/B against round 3's kernel, the runner and partial bench lines.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04f
mkdir -p $OUT
L=mapf-marl_amd/mapfx
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_partial.py tests/test_gpu_partial_full_range.py tests/test_gpu_runner.py \
  tests/test_partial_output_mode.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1 \
  || { grep -E "FAIL|Error" $OUT/tests.txt | head -30; tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
timeout -k 10 120 python3 tools/pstamps_partial.py > $OUT/pstamps.txt 2>&1 && cat $OUT/pstamps.txt
bash tools/ab_bench.sh $OUT/ab 2 "--env marl_partial" $L/libmapfx.so $L/libmapfx_oldpartial.so || exit 1
timeout -k 10 300 python3 bench.py --env runner --cpu-seconds 0 > $OUT/runner.json 2> $OUT/runner.err || { tail $OUT/runner.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/runner.json')); print('runner', d['value'], d['ms_per_step'])"
