#!/bin/bash
# Round 3: primal_seq_kernel (world per wave, phase A / phase B): PRIMAL GPU tests,
# then the primal bench leg and its kernel trace.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03y
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_primal.py -x -q --timeout 120 --timeout-method thread \
  > $OUT/primal_tests.txt 2>&1 || { tail -40 $OUT/primal_tests.txt; exit 1; }
tail -2 $OUT/primal_tests.txt
timeout -k 10 200 python3 bench.py --env primal --cpu-seconds 0 > $OUT/primal.json 2> $OUT/primal.err || { tail -20 $OUT/primal.err; exit 1; }
tail -c 700 $OUT/primal.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv \
  -- python3 bench.py --env primal --cpu-seconds 0 > $OUT/primal_traced.json 2> $OUT/trace.err || exit 1
grep -h primal $OUT/trace/*/run_kernel_stats.csv $OUT/trace/run_kernel_stats.csv 2>/dev/null | cut -c1-200
