#!/bin/bash
# Round 3: PRIMAL kernel A/B on one box: d2cecf5 (p0), 70343ce (p1), read-ahead loop (p2).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03v
mkdir -p $OUT
for rep in 1 2 3; do
for v in p0 p1 p2; do
  MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx_$v.so timeout -k 10 120 python3 bench.py --env primal --cpu-seconds 0 > $OUT/primal_$v.$rep.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('$OUT/primal_$v.$rep.json')); print('$v', d['kernel_ms_per_launch'], d['roofline']['frac'])"
done
done
