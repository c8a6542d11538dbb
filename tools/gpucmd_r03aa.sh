#!/bin/bash
# Round 3: where primal_seq_kernel's time goes (MAPFX_QABL ablations: 1 no record stores,
# 2 no phase B, 4 no move chain, 6 neither phase).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03aa
mkdir -p $OUT
for rep in 1 2; do
for v in "" _qabl1 _qabl2 _qabl4 _qabl6; do
  MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 200 python3 bench.py --env primal --cpu-seconds 0 \
    > $OUT/primal$v.json 2> $OUT/primal$v.err || { tail -20 $OUT/primal$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/primal$v.json')); print('lib$v', d['kernel_ms_per_launch'], d['timing']['stream_ms_per_launch'])"
done
done
