#!/bin/bash
# A/B of the per-step launch path (tools/scale_step.py) for library variants.
cd ${GRAFT_REPO_ROOT:-.}
envs=$1; shift
for v in "$@"; do
  [ "$v" = base ] && v=""
  echo "== lib$v"
  MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 120 python tools/scale_step.py --envs $envs || exit 1
done
