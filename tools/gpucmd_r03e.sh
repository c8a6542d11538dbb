#!/bin/bash
# Round 3: PRIMAL kernel (next-move prefetch, pow2 pitch) parity + lane-width A/B;
# C2 with the store waves ablated (step-wave chain alone).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03e
mkdir -p $OUT
echo "[$(date +%T)] primal tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_primal.py -q -x --timeout 120 --timeout-method thread > $OUT/primal_tests.txt 2>&1
rc=$?; tail -3 $OUT/primal_tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  for L in "" 16 64; do
    MAPFX_PRIMAL_LANES=$L timeout -k 10 120 python3 bench.py --env primal --cpu-seconds 0 > $OUT/primal_L$L.$rep.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('$OUT/primal_L$L.$rep.json')); print('lanes[$L]', d['value'], d['kernel_ms_per_launch'], d['roofline']['frac'])"
  done
done
for v in "" _abl256; do
  MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 \
    --cpu-seconds 0 --per-step-steps 0 > $OUT/c2$v.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('$OUT/c2$v.json')); print('c2 lib$v', d['kernel_ms_per_launch'], d['timing']['kernel_ms_replays'])"
  MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 120 python3 bench.py --gpus 1 --steps 64 --warmup 64 \
    --cpu-seconds 0 --per-step-steps 0 > $OUT/c2t64$v.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('$OUT/c2t64$v.json')); print('c2 T64 lib$v', d['kernel_ms_per_launch'], d['timing']['kernel_ms_replays'])"
done
echo "[$(date +%T)] done"
