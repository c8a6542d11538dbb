#!/bin/bash
# Round 5, call AA: MARL_PARTIAL observation rows copied out with nontemporal stores (the
# goal tables may then stay in L2 across steps) against plain stores: interleaved bench
# lines, FETCH_SIZE of each, the partial + runner GPU tests.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05aa
mkdir -p $O
OUT=r05aa bash tools/gpucmd_r05r.sh || exit 1
for v in new old; do
  if [ $v = new ]; then L=""; else L=$PWD/varlibs/libmapfx_old.so; fi
  MAPFX_LIB=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$v -o run --output-format csv \
    -- python3 bench.py --env marl_partial --cpu-seconds 0 > $O/fetch_$v.json 2> $O/fetch_$v.err || { tail $O/fetch_$v.err; exit 1; }
  python3 - $O/fetch_$v <<'PY'
import csv, glob, sys
vals = []
for p in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if "partial_kernel" in r.get("Kernel_Name", "") and r.get("Counter_Name") == "FETCH_SIZE":
            vals.append(float(r["Counter_Value"]))
print(sys.argv[1], "FETCH_SIZE KB per launch (raw, x2 for gfx950):", sum(vals) / max(1, len(vals)), len(vals))
PY
done
