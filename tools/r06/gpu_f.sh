#!/bin/bash
# Round 6, call F: block-0 s_memtime stamps of the C2 split kernel (T = 20 and 64) at
# the current sources (diagnostic build varlibs/libmapfx_stamps6.so, -DMAPFX_STAMPS).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
for T in 20 64; do
  MAPFX_LIB=$PWD/varlibs/libmapfx_stamps6.so MAPFX_PROBE_E=4096 MAPFX_PROBE_T=$T timeout -k 10 120 python3 tools/stamps.py > $O/stamps_t$T.txt 2>&1 || { tail $O/stamps_t$T.txt; exit 1; }
  cat $O/stamps_t$T.txt
done
