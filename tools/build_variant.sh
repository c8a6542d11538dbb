#!/bin/bash
# Build a diagnostic variant of libmapfx.so: tools/build_variant.sh NAME [MAPFX_SRC] [extra hipcc flags...]
# -> mapf-marl_amd/mapfx/libmapfx_NAME.so   (MAPFX_SRC defaults to the working-tree mapfx.hip;
#    partial.hip is always the working-tree one)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
src=${1:-mapf-marl_amd/csrc/mapfx.hip}; [ $# -gt 0 ] && shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -mllvm -amdgpu-kernarg-preload-count=16 \
  -Wno-unused-result -I include -I mapf-marl_amd/csrc "$@" -o mapf-marl_amd/mapfx/libmapfx_$name.so \
  "$src" mapf-marl_amd/csrc/partial.hip mapf-marl_amd/csrc/primal.hip mapf-marl_amd/csrc/runner.hip
