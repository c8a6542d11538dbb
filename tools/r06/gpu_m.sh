#!/bin/bash
# Round 6, call M: where MARL_PARTIAL's extra reads come from -- FETCH_SIZE of the
# bench's partial leg with the neighbour goal-distance lookups removed (diagnostic build
# varlibs/libmapfx_nolookup.so, -DMAPFX_PARTIAL_ABL_NBLOOKUP: results wrong, bytes and
# time only) against the shipped build, rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06m
mkdir -p $O
for v in shipped nolookup; do
  if [ $v = shipped ]; then L=""; else L=$PWD/varlibs/libmapfx_nolookup.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    MAPFX_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $c -d $O/${v}_$c -o run --output-format csv \
      -- python3 bench.py --env marl_partial --cpu-seconds 0 > $O/${v}_$c.json 2> $O/${v}_$c.err || { tail $O/${v}_$c.err; exit 1; }
  done
  python3 -c "import json; d=json.load(open('$O/${v}_FETCH_SIZE.json')); print('$v kernel_ms_per_step', d['kernel_ms_per_step'])"
done
python3 - <<'PY'
import csv, glob
for v in ("shipped", "nolookup"):
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = []
        for p in glob.glob("gpurun_out/r06m/%s_%s/**/*counter_collection.csv" % (v, c), recursive=True):
            for r in csv.DictReader(open(p)):
                if "partial_kernel" in r["Kernel_Name"] and r["Counter_Name"] == c:
                    vals.append(float(r["Counter_Value"]))
        if vals:
            vals.sort()
            print(v, c, "median KB per dispatch", vals[len(vals) // 2], "n", len(vals))
PY
