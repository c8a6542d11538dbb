#!/bin/bash
# Round 4: MARL_PARTIAL with the window and K-nearest rows in one branch-free block --
# parity, stamps, bench, runner.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04m
mkdir -p $OUT
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_partial.py tests/test_gpu_partial_full_range.py tests/test_gpu_runner.py \
  tests/test_partial_output_mode.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1 \
  || { grep -E "FAIL|Error" $OUT/tests.txt | head -30; tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
timeout -k 10 120 python3 tools/pstamps_partial.py > $OUT/pstamps.txt 2>&1 && cat $OUT/pstamps.txt || exit 1
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --env marl_partial --cpu-seconds 0 > $OUT/partial.r$r.json 2> $OUT/partial.r$r.err \
    || { tail -20 $OUT/partial.r$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/partial.r$r.json')); print('partial r$r', d['kernel_ms_per_step'], d['roofline']['frac'])"
done
timeout -k 10 300 python3 bench.py --env runner --cpu-seconds 0 > $OUT/runner.json 2> $OUT/runner.err || { tail $OUT/runner.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/runner.json')); print('runner', d['value'], d['ms_per_step'])"
