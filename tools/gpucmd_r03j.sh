#!/bin/bash
# Round 3: prologue / epilogue stamps of the split kernel (block 0, step wave).
set -o pipefail
export TMPDIR=/tmp
MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx_stamps_ps3.so timeout -k 10 120 python3 tools/pstamps.py --envs 4096 --T 20 || exit $?
