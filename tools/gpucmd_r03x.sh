#!/bin/bash
# Round 3 (re-entry): GPU suite at HEAD, then the C5 measurement recipe with the SQ
# issue / wait pass (name C5's bound).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03x
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r03x/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r03x/gpu_tests.txt; exit 1; }
tail -3 gpurun_out/r03x/gpu_tests.txt
bash tools/r03_profile.sh r03_c5 --config c5 --gpus 1 --cpu-seconds 0 --per-step-steps 0 || exit $?
