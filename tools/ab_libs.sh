#!/bin/bash
# A/B: time the runner rollout with alternative builds of libmapfx (same process per lib)
cd ${GRAFT_REPO_ROOT:-.}
for lib in "$@"; do
  echo "== $lib"
  MAPFX_LIB=$PWD/$lib timeout -k 10 100 python tools/ablate.py --rounds 3 2>&1 | grep -E "^(all|nothing|no_window) "
done
