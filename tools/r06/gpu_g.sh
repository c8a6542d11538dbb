#!/bin/bash
# Round 6, call G: the step wave with the invalid-action test as a uniform branch in
# two step bodies (MAPFX_CHK_RT: map parity instanced only) against the four-body form
# -- C2 T = 20 / 64 kernel times interleaved, then block-0 stamps of both.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
for rep in 1 2 3; do
  for v in new chkrt; do
    if [ $v = new ]; then L=""; else L=$PWD/varlibs/libmapfx_chkrt.so; fi
    for T in 20 64; do
      MAPFX_LIB=$L timeout -k 10 200 python3 bench.py --steps $T --warmup 5 --chunk 64 --cpu-seconds 0 --per-step-steps 0 > $O/c2_${v}_T${T}_$rep.json 2> $O/c2_${v}_T${T}_$rep.err || { tail $O/c2_${v}_T${T}_$rep.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/c2_${v}_T${T}_$rep.json')); print('$v T$T $rep', d['kernel_ms_per_launch'], d['roofline']['frac'], d['ms_per_step'])"
    done
  done
done
for v in stamps6 chkrt_st; do
  MAPFX_LIB=$PWD/varlibs/libmapfx_$v.so MAPFX_PROBE_E=4096 MAPFX_PROBE_T=20 timeout -k 10 120 python3 tools/stamps.py > $O/stamps_$v.txt 2>&1 || { tail $O/stamps_$v.txt; exit 1; }
  echo "== $v"; head -12 $O/stamps_$v.txt | tail -11
done
