#!/bin/bash
# Round 6, profiling call 1: the mapfx-unit legs at the round-6 kernels -- c2 (the
# driver's command), c2_step, c3 -- each through tools/r06/profile_leg.sh (kernel trace
# + stats, FETCH_SIZE, WRITE_SIZE, LDS and SQ passes of the same bench command).
set -o pipefail
export TMPDIR=/tmp
P="bash tools/r06/profile_leg.sh"
$P c2 "--config c2 --T 20 --E 4096" --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 0 || exit 1
$P c2_step "--config c2_step --T 1 --E 4096 --bench-kernel-key per_step.kernel" --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 200 || exit 1
$P c3 "--config c3 --T 64 --E 2048" --config c3 --cpu-seconds 0 --per-step-steps 0 || exit 1
