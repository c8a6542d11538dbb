#!/bin/bash
# Round 6, call L: the driver's command (C2, T = 20) with the split store waves' stores
# nontemporal (varlibs/libmapfx_nt.so, -DMAPFX_NT_STORE) vs plain (shipped): wall per
# step as well as kernel time -- dirty L2 lines are written back at the kernel's end,
# which the wall clock sees.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06l
mkdir -p $O
for rep in 1 2 3 4 5; do
  for v in plain nt; do
    if [ $v = plain ]; then L=""; else L=$PWD/varlibs/libmapfx_nt.so; fi
    MAPFX_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 0 > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || { tail $O/c2_${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c2_${v}_$rep.json')); print('$v $rep wall_ms', d['timing']['wall_ms'], 'kernel', d['kernel_ms_per_launch'], 'value', d['value'])"
  done
done
