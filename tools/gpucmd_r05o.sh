#!/bin/bash
# Round 5, call O: mapfx.hip built without the IR load/store vectorizer (C3 / C5 kernels:
# fewer SGPR spill reloads) against the shipped build: the driver's C2 line, C3, C5,
# interleaved three rounds (varlibs/libmapfx_nolsv_all.so).
set -o pipefail
O=gpurun_out/r05o
mkdir -p $O
for rep in 1 2 3; do
  for v in cur nolsv; do
    if [ $v = cur ]; then L=""; else L=$PWD/varlibs/libmapfx_nolsv_all.so; fi
    MAPFX_LIB=$L timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || { tail $O/c2_${v}_$rep.err; exit 1; }
    MAPFX_LIB=$L timeout -k 10 200 python3 bench.py --config c3 --cpu-seconds 0 --per-step-steps 0 > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || { tail $O/c3_${v}_$rep.err; exit 1; }
    MAPFX_LIB=$L timeout -k 10 200 python3 bench.py --config c5 --cpu-seconds 0 --per-step-steps 0 > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || { tail $O/c5_${v}_$rep.err; exit 1; }
    python3 -c "
import json
a=json.load(open('$O/c2_${v}_$rep.json')); b=json.load(open('$O/c3_${v}_$rep.json')); c=json.load(open('$O/c5_${v}_$rep.json'))
print('$v $rep c2', a['kernel_ms_per_launch'], 'step', a['per_step']['kernel_ms'], 'c3', b['kernel_ms_per_launch'], 'c5', c['kernel_ms_per_launch'])"
  done
done
