#!/bin/bash
# Round 3: the alternating two-store-wave split (MAPFX_SPLIT_ALT=1, default build)
# against the one-store-wave split (libmapfx_alt0.so): parity of the split kernel,
# then the driver's bench command with each library, interleaved.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03c
mkdir -p $OUT
echo "[$(date +%T)] split-kernel parity"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread \
  -k "runner_rollout_every_step or long_horizon or rollout_equals_repeated or full_size or rollout_timed" > $OUT/split_tests.txt 2>&1
rc=$?; tail -3 $OUT/split_tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2 3; do
  for v in "" _alt0; do
    echo "[$(date +%T)] bench lib$v rep $rep"
    MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 \
      --cpu-seconds 0 --per-step-steps 0 > $OUT/c2$v.$rep.json 2>/dev/null || exit $?
    python3 -c "import json,sys; d=json.load(open('$OUT/c2$v.$rep.json')); print('lib$v', d['value'], d['kernel_ms_per_launch'], d['timing']['kernel_ms_replays'])"
  done
done
for v in "" _alt0; do
  MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 120 python3 bench.py --gpus 1 --cpu-seconds 0 --per-step-steps 0 > $OUT/c2t64$v.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('$OUT/c2t64$v.json')); print('T64 lib$v', d['value'], d['kernel_ms_per_launch'], d['roofline']['frac'])"
done
echo "[$(date +%T)] done"
