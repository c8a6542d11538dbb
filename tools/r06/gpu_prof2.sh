#!/bin/bash
# Round 6, profiling call 2: c5, MARL_PARTIAL and PRIMAL through tools/r06/profile_leg.sh.
set -o pipefail
export TMPDIR=/tmp
P="bash tools/r06/profile_leg.sh"
$P c5 "--config c5 --T 64 --E 1024" --config c5 --cpu-seconds 0 --per-step-steps 0 || exit 1
$P partial "--config marl_partial --T 1 --E 4096 --match N=15 --match S=8" --env marl_partial --cpu-seconds 0 || exit 1
$P primal "--config primal --T 64 --E 4096" --env primal --cpu-seconds 0 || exit 1
