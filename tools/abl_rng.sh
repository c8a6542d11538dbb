#!/bin/bash
# HBM actions vs device-generated actions, per lib variant
cd ${GRAFT_REPO_ROOT:-.}
envs=$1; shift
for v in "$@"; do
  [ "$v" = base ] && v=""
  for r in "" --rng; do
    echo "== lib$v $r"
    MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 120 python tools/scale_e.py --envs $envs --launches 4 $r || exit 1
  done
done
