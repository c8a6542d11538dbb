#!/bin/bash
# A/B of the shipped library against diagnostic variants on the driver's C2 command
# (and the T=64 chunk), 3 runs each: usage  bash tools/gpucmd_ab.sh TAG VARIANT...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for v in base "$@"; do
  if [ $v = base ]; then unset MAPFX_LIB; else export MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx_$v.so; fi
  for i in 1 2 3; do
    timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps ${PS:-0} > $OUT/$v.$i.json 2> $OUT/$v.err || exit $?
  done
  timeout -k 10 200 python3 bench.py --gpus 1 --cpu-seconds 0 --per-step-steps 0 > $OUT/${v}_t64.json 2>> $OUT/$v.err || exit $?
  python3 -c "
import json
ks = [json.load(open('$OUT/$v.%d.json' % i))['kernel_ms_per_launch'] for i in (1, 2, 3)]
vs = [json.load(open('$OUT/$v.%d.json' % i))['value'] for i in (1, 2, 3)]
ps = [(json.load(open('$OUT/$v.%d.json' % i)).get('per_step') or {}).get('kernel_ms') for i in (1, 2, 3)]
d = json.load(open('$OUT/${v}_t64.json'))
print('$v', 'per-step kernel_ms', ps, 'T20 kernel_ms', ks, 'value', ['%.3g' % x for x in vs], '| T64 kernel_ms', d['kernel_ms_per_launch'], 'value %.3g' % d['value'])"
done
