#!/bin/bash
# Round 4: where the MARL_PARTIAL launch's time goes across blocks (per-block realtime
# stamps) and the C2 split kernel's per-wave stamps with the two-map (DBM) step wave.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04j
mkdir -p $OUT
timeout -k 10 120 python3 tools/pstamps_partial.py > $OUT/pstamps.txt 2>&1 && cat $OUT/pstamps.txt || exit 1
timeout -k 10 120 python3 tools/stamps.py > $OUT/c2_stamps.txt 2>&1 && cat $OUT/c2_stamps.txt || exit 1
MAPFX_PROBE_E=4096 timeout -k 10 120 python3 tools/stamps.py > $OUT/c2_stamps_b.txt 2>&1 || exit 1
