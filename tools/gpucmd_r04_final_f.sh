#!/bin/bash
# Round 4 end: stamps of the final kernels (diagnostic builds) into gpurun_out/profiles.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/profiles
mkdir -p $O
timeout -k 10 120 python3 tools/pstamps_partial.py > $O/r04_pstamps_partial.txt 2>&1 && cat $O/r04_pstamps_partial.txt || exit 1
MAPFX_PROBE_T=20 timeout -k 10 120 python3 tools/stamps.py > $O/r04_c2_stamps_t20.txt 2>&1 && cat $O/r04_c2_stamps_t20.txt || exit 1
