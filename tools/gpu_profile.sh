#!/bin/bash
# GPU-box measurement recipe: bench line, kernel trace + stats, two PMC passes.
# usage: bash tools/gpu_profile.sh TAG [bench args...]
set -eo pipefail
TAG=${1:-r01}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
echo "[$(date +%T)] bench"
timeout -k 10 400 python3 bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
echo "[$(date +%T)] kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 bench.py --cpu-seconds 0 "$@" > "$OUT/bench_traced.json" 2> "$OUT/trace.err"
echo "[$(date +%T)] pmc FETCH_SIZE"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv \
  -- python3 bench.py --cpu-seconds 0 --per-step-steps 0 "$@" > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err"
echo "[$(date +%T)] pmc WRITE_SIZE"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv \
  -- python3 bench.py --cpu-seconds 0 --per-step-steps 0 "$@" > "$OUT/bench_write.json" 2> "$OUT/write.err"
echo "[$(date +%T)] done"
