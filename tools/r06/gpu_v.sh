#!/bin/bash
# Round 6, call V: the driver's launch (C2, T = 20) with 4-step action blocks
# (varlibs/libmapfx_ab4.so) against the shipped 8-step blocks, interleaved, four rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06v
mkdir -p $O
for rep in 1 2 3 4; do
  for v in ab4 ab8; do
    if [ $v = ab4 ]; then L=$PWD/varlibs/libmapfx_ab4.so; else L=""; fi
    MAPFX_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 0 > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || { tail $O/c2_${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c2_${v}_$rep.json')); print('$v', $rep, d['kernel_ms_per_launch'], d['ms_per_step'], d['kernel'][:70])"
  done
done
