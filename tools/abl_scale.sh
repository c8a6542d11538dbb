#!/bin/bash
# Fused-rollout us/step vs env count for alternative builds of libmapfx (one process each).
# usage: tools/abl_scale.sh ENVS suffix1 suffix2 ...   ("" = the shipped libmapfx.so)
cd ${GRAFT_REPO_ROOT:-.}
envs=$1; shift
for v in "$@"; do
  [ "$v" = base ] && v=""
  echo "== lib$v"
  MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 120 python tools/scale_e.py --envs $envs --launches 4 || exit 1
done
