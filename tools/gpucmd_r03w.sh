#!/bin/bash
# Round 3: measurement recipe for the marl_partial leg (pmc_partial.json) and the
# runner leg's bench line.
set -o pipefail
export TMPDIR=/tmp
bash tools/r03_profile.sh r03_partial --env marl_partial --cpu-seconds 0 || exit $?
mkdir -p gpurun_out/r03w
timeout -k 10 300 python3 bench.py --env runner --cpu-seconds 0 > gpurun_out/r03w/runner.json 2> gpurun_out/r03w/runner.err || exit $?
tail -c 600 gpurun_out/r03w/runner.json
