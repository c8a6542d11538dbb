#!/bin/bash
# A/B: time the runner rollout + per-step path with alternative builds of libmapfx
# (one process per lib).  Usage: tools/ab_libs.sh lib1.so lib2.so ...
cd ${GRAFT_REPO_ROOT:-.}
for lib in "$@"; do
  echo "== $lib"
  MAPFX_LIB=$PWD/$lib timeout -k 10 100 python tools/ablate.py --quick --rounds 5 2>&1 | grep -E "^(all|nothing|per_step) "
done
