#!/bin/bash
# Round 4: C2 split-kernel stamps at the driver's T = 20, prologue included.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04s
mkdir -p $OUT
MAPFX_PROBE_T=20 timeout -k 10 120 python3 tools/stamps.py > $OUT/c2_stamps_t20.txt 2>&1 && cat $OUT/c2_stamps_t20.txt || exit 1
