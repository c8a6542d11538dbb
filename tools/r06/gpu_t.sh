#!/bin/bash
# Round 6, call T: generic kernel -- the u16 occupancy window writer issues a group's LDS reads
# together (new cells, then every row: two round trips per group) -- generic parity tests, then C5
# (T = 64) interleaved against the previous build (varlibs/libmapfx_base.so).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06t
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "generic or c5 or bench_leg or window_occ or primal or full or stacked or n200 or n300 or dense" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for rep in 1 2 3; do
  for v in new base; do
    if [ $v = new ]; then L=""; else L=$PWD/varlibs/libmapfx_base.so; fi
    MAPFX_LIB=$L timeout -k 10 200 python3 bench.py --config c5 --steps 64 --warmup 5 --chunk 64 --cpu-seconds 0 --per-step-steps 0 > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || { tail $O/c5_${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c5_${v}_$rep.json')); print('$v c5 T64 $rep', d['kernel_ms_per_launch'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
