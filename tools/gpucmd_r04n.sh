#!/bin/bash
# Round 4: MARL_PARTIAL back to per-round KNN branches (+ 4-wave blocks, DPP edge scan) --
# parity, bench; the per-step drop-in kernel's phase stamps; a runner kernel trace.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04n
mkdir -p $OUT
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_partial.py tests/test_gpu_partial_full_range.py tests/test_gpu_runner.py \
  tests/test_partial_output_mode.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1 \
  || { grep -E "FAIL|Error" $OUT/tests.txt | head -30; tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --env marl_partial --cpu-seconds 0 > $OUT/partial.r$r.json 2> $OUT/partial.r$r.err \
    || { tail -20 $OUT/partial.r$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/partial.r$r.json')); print('partial r$r', d['kernel_ms_per_step'], d['roofline']['frac'])"
done
timeout -k 10 120 python3 tools/pstamps_step.py > $OUT/step_stamps.txt 2>&1 && cat $OUT/step_stamps.txt || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/rtrace -o run -- python3 bench.py --env runner --cpu-seconds 0 \
  > $OUT/runner_trace.log 2>&1 || { tail -20 $OUT/runner_trace.log; exit 1; }
f=$(find $OUT/rtrace -name "*kernel_stats.csv" | head -1); python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:9]:
    print("%-70s %5s %8.2f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1000))
PY
