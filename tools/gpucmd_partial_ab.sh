#!/bin/bash
# partial env: GPU parity, then the marl_partial bench for the shipped library and a
# variant (usage: bash tools/gpucmd_partial_ab.sh TAG [VARIANT])
set -o pipefail
TAG=$1; V=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_partial.py tests/test_gpu_runner.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for v in base $V; do
  if [ $v = base ]; then unset MAPFX_LIB; else export MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx_$v.so; fi
  timeout -k 10 300 python3 bench.py --env marl_partial --cpu-seconds 0 > $OUT/partial_$v.json 2> $OUT/partial_$v.err || exit $?
  timeout -k 10 300 python3 bench.py --env runner --cpu-seconds 0 > $OUT/runner_$v.json 2> $OUT/runner_$v.err || exit $?
  python3 -c "
import json
for k in ('partial', 'runner'):
    d = json.load(open('$OUT/%s_$v.json' % k)); print('$v', k, d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'))"
done
