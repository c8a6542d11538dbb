#!/bin/bash
# Round 6, call B: step-wave body instanced per (map parity, autoreset, invalid-action
# check) -- C2 T = 20 / 64 interleaved against the previous build (varlibs/libmapfx_base.so),
# then the split kernel's parity tests.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "runner_rollout or bench_leg or autoreset or invalid_action" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for rep in 1 2 3; do
  for v in new base; do
    if [ $v = new ]; then L=""; else L=$PWD/varlibs/libmapfx_base.so; fi
    for T in 20 64; do
      MAPFX_LIB=$L timeout -k 10 200 python3 bench.py --steps $T --warmup 5 --chunk 64 --cpu-seconds 0 --per-step-steps 0 > $O/c2_${v}_T${T}_$rep.json 2> $O/c2_${v}_T${T}_$rep.err || { tail $O/c2_${v}_T${T}_$rep.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/c2_${v}_T${T}_$rep.json')); print('$v T$T $rep', d['kernel_ms_per_launch'], d['roofline']['frac'], d['ms_per_step'])"
    done
  done
done
