#!/bin/bash
# Measurement recipe for ONE bench command (round 3): the bench line, a kernel trace +
# stats pass, FETCH_SIZE and WRITE_SIZE passes (separate: TCC slots), an LDS pass and
# an SQ issue/wait pass, each a rocprofv3 run of the SAME python3 bench.py arguments.
# usage: bash tools/r03_profile.sh TAG [bench args...]
set -eo pipefail
TAG=${1:?tag}
shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
echo "python3 bench.py $*" > "$OUT/command.txt"
echo "[$(date +%T)] $TAG bench"
timeout -k 10 300 python3 bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
tail -c 300 "$OUT/bench.json"
echo "[$(date +%T)] kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 bench.py "$@" > "$OUT/bench_traced.json" 2> "$OUT/trace.err"
echo "[$(date +%T)] pmc FETCH_SIZE"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv \
  -- python3 bench.py "$@" > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err"
echo "[$(date +%T)] pmc WRITE_SIZE"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv \
  -- python3 bench.py "$@" > "$OUT/bench_write.json" 2> "$OUT/write.err"
echo "[$(date +%T)] pmc LDS"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  -d "$OUT/pmc_lds" -o run --output-format csv \
  -- python3 bench.py "$@" > "$OUT/bench_lds.json" 2> "$OUT/lds.err"
echo "[$(date +%T)] pmc SQ issue / wait"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  -d "$OUT/pmc_sq" -o run --output-format csv \
  -- python3 bench.py "$@" > "$OUT/bench_sq.json" 2> "$OUT/sq.err"
echo "[$(date +%T)] $TAG done"
