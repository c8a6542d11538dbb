#!/bin/bash
# round-2 call s: profiles of the current kernels -- C5 at the bench default (T=64)
# and the driver's C2 command.
set -o pipefail
bash tools/r02_profile.sh r02s_c5 --config c5 --gpus 1 --cpu-seconds 0 --per-step-steps 0 || exit $?
bash tools/r02_profile.sh r02s_c2 --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 0 || exit $?
