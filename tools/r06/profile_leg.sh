#!/bin/bash
# Measurement recipe (round 6; tools/r05_profile.sh with the round tag a parameter) for ONE bench leg at HEAD: the bench line, a kernel trace +
# stats pass, FETCH_SIZE and WRITE_SIZE passes (separate: TCC slots), an LDS pass and an
# SQ issue / wait pass, each a rocprofv3 run of the SAME python3 bench.py arguments; then
# tools/pmc_traffic.py writes gpurun_out/profiles/pmc_<name>.json, keyed to the exact
# kernel instance and build the traced bench line reports (bench.py cites it only then).
# usage: bash tools/r05_profile.sh NAME "PMC_TRAFFIC ARGS" [bench args...]
set -eo pipefail
NAME=${1:?name}
PARGS=${2:?pmc_traffic args}
shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${ROUND:-r06}_$NAME
mkdir -p "$OUT" "$ROOT/gpurun_out/profiles"
export TMPDIR=/tmp
cd "$ROOT"
echo "python3 bench.py $*" > "$OUT/command.txt"
echo "[$(date +%T)] $NAME kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 bench.py "$@" > "$OUT/bench_traced.json" 2> "$OUT/trace.err"
tail -c 400 "$OUT/bench_traced.json"
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
# shellcheck disable=SC2086
python3 tools/pmc_traffic.py --trace "$OUT/trace" --fetch "$OUT/pmc_fetch" --write "$OUT/pmc_write" \
  --lds "$OUT/pmc_lds" --sq "$OUT/pmc_sq" --bench-json "$OUT/bench_traced.json" --tag "${ROUND:-r06}_$NAME" \
  --command "python3 bench.py $*" --out "$ROOT/gpurun_out/profiles/pmc_$NAME.json" $PARGS > "$OUT/summary.json"
python3 - "$ROOT/gpurun_out/profiles/pmc_$NAME.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = d["trace"]["kernels"][0]
print(d["kernel"][:90], "| avg_ns", k["avg_ns"], "| traffic", d.get("traffic_bytes_per_launch"),
      "| wait_any", round((d.get("sq") or {}).get("wait_any_frac_of_wave_cycles", -1), 3),
      "| bank_conf", round((d.get("lds") or {}).get("bank_conflict_cycles_frac", -1), 3),
      "| min gap_ns", min(d["trace"].get("gap_ns") or [0]))
PY
echo "[$(date +%T)] $NAME done"
