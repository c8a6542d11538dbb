#!/bin/bash
# round-2 call o: generic kernel with LDS-only barriers + action prefetch: parity,
# then C5 bench for the build and its ablation variants (diagnostic).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${OUTTAG:-r02o}
mkdir -p $OUT
echo "[$(date +%T)] gpu tests (generic kernel)"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "occ or full_size or rollout_equals or batched_step or primal or autoreset or invalid" > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
B="--config c5 --gpus 1 --cpu-seconds 0 --per-step-steps 0"
for v in base nofw; do
  if [ $v = base ]; then unset MAPFX_LIB; else export MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx_$v.so; fi
  echo "[$(date +%T)] $v"
  timeout -k 10 300 python3 bench.py $B --steps 20 --warmup 5 > $OUT/$v.json 2> $OUT/$v.err || exit $?
  timeout -k 10 300 python3 bench.py $B > $OUT/${v}_t64.json 2>> $OUT/$v.err || exit $?
  python3 -c "
import json
for f in ('$OUT/$v.json', '$OUT/${v}_t64.json'):
    d = json.load(open(f)); print('$v', d['config']['chunk_T'], d['value'], d['kernel_ms_per_launch'], d['roofline']['frac'])"
done
