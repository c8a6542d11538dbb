#!/bin/bash
# Round 5, call AF: the generic rollout kernel specialised on the runner output set
# (FEAT_RUN: per-output tests compiled away) against the previous build
# (varlibs/libmapfx_old.so): C5 lines interleaved, then the parity suite.
set -o pipefail
O=gpurun_out/r05af
mkdir -p $O
for rep in 1 2 3; do
  for v in new old; do
    if [ $v = new ]; then L=""; else L=$PWD/varlibs/libmapfx_old.so; fi
    MAPFX_LIB=$L timeout -k 10 200 python3 bench.py --config c5 --cpu-seconds 0 --per-step-steps 0 > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || { tail $O/c5_${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c5_${v}_$rep.json')); print('$v $rep c5', d['kernel_ms_per_launch'], d['roofline']['frac'], d['kernel'][40:90])"
  done
done
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
