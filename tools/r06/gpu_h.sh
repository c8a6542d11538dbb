#!/bin/bash
# Round 6, call H: the store-wave split at 64 agents per env (C3's runner rollout; u16
# reward codes) -- split parity tests, then C3 interleaved against the previous build
# (varlibs/libmapfx_pre64.so: the one-wave kernel for N = 64).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "runner_rollout or split64 or autoreset or back_to_back or (bench_leg and not c3-T64)" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for rep in 1 2 3; do
  for v in new pre64; do
    if [ $v = new ]; then L=""; else L=$PWD/varlibs/libmapfx_pre64.so; fi
    for T in 64 20; do
      MAPFX_LIB=$L timeout -k 10 200 python3 bench.py --config c3 --steps $T --warmup 5 --chunk 64 --cpu-seconds 0 --per-step-steps 0 > $O/c3_${v}_T${T}_$rep.json 2> $O/c3_${v}_T${T}_$rep.err || { tail $O/c3_${v}_T${T}_$rep.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/c3_${v}_T${T}_$rep.json')); print('$v c3 T$T $rep', d['kernel_ms_per_launch'], d['roofline']['frac'], d['kernel'][40:90])"
    done
  done
done
