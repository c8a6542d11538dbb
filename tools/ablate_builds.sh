#!/bin/bash
# time the runner rollout with diagnostic ablation builds (MAPFX_ABLATE bit masks)
cd ${GRAFT_REPO_ROOT:-.}
for m in 0 1 2 4 8 15; do
  lib=mapf-marl_amd/mapfx/libmapfx_abl$m.so; [ $m = 0 ] && lib=mapf-marl_amd/mapfx/libmapfx.so
  echo "== ABLATE=$m"
  MAPFX_LIB=$PWD/$lib timeout -k 10 100 python tools/ablate.py --rounds 3 2>&1 | grep "^all "
done
