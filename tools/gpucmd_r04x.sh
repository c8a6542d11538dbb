#!/bin/bash
# Round 4: runner compaction kernel time, register-cached flags vs reloaded (kernel traces).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04x
mkdir -p $OUT
L=mapf-marl_amd/mapfx
for lib in libmapfx libmapfx_prev; do
  MAPFX_LIB=$PWD/$L/$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$lib -o run \
    -- python3 bench.py --env runner --cpu-seconds 0 > $OUT/$lib.log 2>&1 || { tail -20 $OUT/$lib.log; exit 1; }
  f=$(find $OUT/$lib -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$lib" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "compact" in r["Name"] or "partial_kernel" in r["Name"]:
        print(sys.argv[2], r["Name"][:60], r["Calls"], "%.2f us" % (float(r["AverageNs"]) / 1000))
PY
done
