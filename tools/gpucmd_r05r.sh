#!/bin/bash
# Round 5, call R (and S: the K-nearest selection by one min per round over key - (last + 1)
# and a per-wave float32 sqrt table): the partial kernel with the runner fusion as a template argument (the
# plain step compiled without it) against the previous build (varlibs/libmapfx_old.so):
# MARL_PARTIAL and runner bench lines interleaved, then the partial / runner GPU tests.
set -o pipefail
O=gpurun_out/${OUT:-r05r}
mkdir -p $O
for rep in 1 2 3; do
  for v in new old; do
    if [ $v = new ]; then L=""; else L=$PWD/varlibs/libmapfx_old.so; fi
    MAPFX_LIB=$L timeout -k 10 200 python3 bench.py --env marl_partial --cpu-seconds 0 > $O/p_${v}_$rep.json 2> $O/p_${v}_$rep.err || { tail $O/p_${v}_$rep.err; exit 1; }
    MAPFX_LIB=$L timeout -k 10 200 python3 bench.py --env runner --cpu-seconds 0 > $O/r_${v}_$rep.json 2> $O/r_${v}_$rep.err || { tail $O/r_${v}_$rep.err; exit 1; }
    python3 -c "import json; p=json.load(open('$O/p_${v}_$rep.json')); r=json.load(open('$O/r_${v}_$rep.json')); print('$v $rep partial', p['ms_per_step'], p['roofline']['frac'], 'runner', r['ms_per_step'], p['kernel'][40:80])"
  done
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_partial.py tests/test_gpu_partial_full_range.py tests/test_gpu_runner.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
