#!/bin/bash
# Round 3: plain-store three-wave split (shipped): split parity, the four-wave option's
# parity, then the measurement recipe on the driver's command.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03s
mkdir -p $OUT
echo "[$(date +%T)] parity (shipped)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_runner.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; tail -3 $OUT/tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
echo "[$(date +%T)] parity (MAPFX_SPLIT_MOVE=1 build)"
MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx_move1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q \
  --timeout 120 --timeout-method thread -k "runner_rollout or long_horizon" > $OUT/tests_move1.txt 2>&1
rc=$?; tail -3 $OUT/tests_move1.txt
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/r03_profile.sh r03_c2 --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 0 || exit $?
echo "[$(date +%T)] done"
