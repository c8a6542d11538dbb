#!/bin/bash
# Round 6, call K: generic rollout actions read 4 steps per block (one drain of the
# step's stores per block instead of per step) -- generic-kernel parity tests, then C5
# interleaved against the previous build (varlibs/libmapfx_r6a.so).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "generic_rollout or rollout_equals or full_size or bench_leg or stacked_swap or autoreset or invalid" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for rep in 1 2 3; do
  for v in new r6a; do
    if [ $v = new ]; then L=""; else L=$PWD/varlibs/libmapfx_r6a.so; fi
    MAPFX_LIB=$L timeout -k 10 200 python3 bench.py --config c5 --cpu-seconds 0 --per-step-steps 0 > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || { tail $O/c5_${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c5_${v}_$rep.json')); print('$v c5 $rep', d['kernel_ms_per_launch'], d['roofline']['frac'])"
  done
done
