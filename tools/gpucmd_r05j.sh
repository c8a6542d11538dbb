#!/bin/bash
# Round 5, call J (diagnostic): MARL_PARTIAL step time against envs per wave and waves
# per block (varlibs/libmapfx_diag.so: -DMAPFX_PARTIAL_DIAG_ENV knobs), interleaved.
set -o pipefail
O=gpurun_out/r05j
mkdir -p $O
L=$PWD/varlibs/libmapfx_diag.so
for rep in 1 2; do
for cfg in "4 4" "2 4" "1 4" "2 2" "4 2" "4 1"; do
  set -- $cfg
  MAPFX_LIB=$L MAPFX_PARTIAL_EPW=$1 MAPFX_PARTIAL_WPB=$2 timeout -k 10 200 python3 bench.py --env marl_partial --cpu-seconds 0 \
    > $O/b_$1_$2_$rep.json 2> $O/b_$1_$2_$rep.err || { tail -20 $O/b_$1_$2_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$1_$2_$rep.json')); print('EPW $1 WPB $2', d['ms_per_step'], d['roofline']['frac'])"
done
done
