#!/bin/bash
# Round 6, call O: the other kernargs fetched after the first loads are issued (EARLY
# instances) -- the split / wave parity tests, then C2 T = 20 / 64, the per-step kernel
# and C3 interleaved against the previous build (varlibs/libmapfx_base.so).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06o
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "runner_rollout or bench_leg or autoreset or invalid_action or split64 or every_step or step_matches or fused" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for rep in 1 2 3; do
  for v in new base; do
    if [ $v = new ]; then L=""; else L=$PWD/varlibs/libmapfx_base.so; fi
    for T in 20 64; do
      MAPFX_LIB=$L timeout -k 10 200 python3 bench.py --steps $T --warmup 5 --chunk 64 --cpu-seconds 0 --per-step-steps 200 > $O/c2_${v}_T${T}_$rep.json 2> $O/c2_${v}_T${T}_$rep.err || { tail $O/c2_${v}_T${T}_$rep.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/c2_${v}_T${T}_$rep.json')); print('$v c2 T$T $rep', d['kernel_ms_per_launch'], d['ms_per_step'], 'per_step', d['per_step']['kernel_ms'], d['per_step']['ms_per_step'])"
    done
    MAPFX_LIB=$L timeout -k 10 200 python3 bench.py --config c3 --steps 64 --warmup 5 --chunk 64 --cpu-seconds 0 --per-step-steps 0 > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || { tail $O/c3_${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c3_${v}_$rep.json')); print('$v c3 T64 $rep', d['kernel_ms_per_launch'], d['ms_per_step'])"
  done
done
# block-0 stamps at the new sources (diagnostic build varlibs/libmapfx_stamps6.so)
MAPFX_LIB=$PWD/varlibs/libmapfx_stamps6.so MAPFX_PROBE_E=4096 MAPFX_PROBE_T=20 timeout -k 10 120 python3 tools/stamps.py > $O/stamps_t20.txt 2>&1 || { tail $O/stamps_t20.txt; exit 1; }
cat $O/stamps_t20.txt
MAPFX_LIB=$PWD/varlibs/libmapfx_stamps6.so timeout -k 10 180 python3 tools/stamps_c5.py > $O/stamps_c5.txt 2>&1 || { tail $O/stamps_c5.txt; exit 1; }
cat $O/stamps_c5.txt
