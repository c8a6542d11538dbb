#!/bin/bash
# Round 3: ALT split A/B (tools/gpucmd_r03c.sh), then profiles of the PRIMAL leg and C5.
set -o pipefail
export TMPDIR=/tmp
bash tools/gpucmd_r03c.sh || exit $?
bash tools/r03_profile.sh r03_primal --env primal --cpu-seconds 0 || exit $?
bash tools/r03_profile.sh r03_c5 --config c5 --gpus 1 --cpu-seconds 0 --per-step-steps 0 || exit $?
echo "[$(date +%T)] all done"
