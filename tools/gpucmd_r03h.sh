#!/bin/bash
# Round 3: per-interval busy time of the step wave and both store waves (block 0,
# s_memtime stamps, diagnostic build libmapfx_stamps.so).
set -o pipefail
export TMPDIR=/tmp
for E in 256 4096; do
  MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx_stamps.so MAPFX_PROBE_E=$E timeout -k 10 120 python3 tools/stamps.py || exit $?
done
