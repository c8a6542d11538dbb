#!/bin/bash
# Round 6, call J: does the generic rollout (C5) wait on its stores every step?  The
# same launch with actions from HBM vs from the device generator (tools/r06/c5_rng_probe.py).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
timeout -k 10 300 python3 tools/r06/c5_rng_probe.py 2>&1 | tee $O/c5_rng_probe.txt
PROBE_CONFIG=c3 timeout -k 10 300 python3 tools/r06/c5_rng_probe.py 2>&1 | tee $O/c3_rng_probe.txt
