#!/bin/bash
cd ${GRAFT_REPO_ROOT:-.}
for lib in stamps stamps_ns; do
  for E in 256 4096; do
    echo "== $lib"
    MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx_$lib.so MAPFX_PROBE_E=$E timeout -k 10 120 python tools/stamps.py || exit 1
  done
done
