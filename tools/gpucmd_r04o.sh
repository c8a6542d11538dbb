#!/bin/bash
# Round 4: split kernel with the edge collisions counted by the store waves (DBM info word
# carries old / new cell, action, occupant move and count) -- parity, A/B against the
# committed build, stamps; a runner kernel trace.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04o
mkdir -p $OUT
L=mapf-marl_amd/mapfx
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread \
  > $OUT/tests.txt 2>&1 || { grep -E "FAIL|Error" $OUT/tests.txt | head -30; tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
bash tools/ab_bench.sh $OUT/ab20 3 "--gpus 1 --steps 20 --warmup 5" $L/libmapfx.so $L/libmapfx_headc2.so || exit 1
bash tools/ab_bench.sh $OUT/ab64 2 "--gpus 1 --steps 512 --warmup 64" $L/libmapfx.so $L/libmapfx_headc2.so || exit 1
timeout -k 10 120 python3 tools/stamps.py > $OUT/c2_stamps.txt 2>&1 && cat $OUT/c2_stamps.txt || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rtrace -o run -- python3 bench.py --env runner --cpu-seconds 0 \
  > $OUT/runner_trace.log 2>&1 || { tail -20 $OUT/runner_trace.log; exit 1; }
f=$(find $OUT/rtrace -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:9]:
    print("%-70s %5s %8.2f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1000))
PY
