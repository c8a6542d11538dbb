#!/bin/bash
# round-2 GPU call: gpu tests, then the driver's bench command profiled (C2) and C5.
set -o pipefail
mkdir -p gpurun_out/r02a
echo "[$(date +%T)] tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r02a/tests.log 2>&1
rc=$?
tail -3 gpurun_out/r02a/tests.log
# 1 = a test failed (keep measuring); anything else (timeout, abort, segfault) ends the call
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
bash tools/r02_profile.sh r02a_c2 --gpus 1 --steps 20 --warmup 5 || exit $?
bash tools/r02_profile.sh r02a_c5 --config c5 --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 0
