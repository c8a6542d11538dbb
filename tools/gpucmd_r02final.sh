#!/bin/bash
# Round-2 record: GPU suite, bench lines of every leg, profiles of the driver's
# command (C2) and of C5 at the bench default.  Outputs under gpurun_out/r02final.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02final
mkdir -p $OUT
echo "[$(date +%T)] gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.txt 2>&1
rc=$?; tail -3 $OUT/gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
run() {  # name, bench args...
  local n=$1; shift
  echo "[$(date +%T)] bench $n"
  timeout -k 10 300 python3 bench.py "$@" > $OUT/bench_$n.json 2> $OUT/bench_$n.err || exit $?
}
run c2 --gpus 1 --steps 20 --warmup 5
run c2_t64 --gpus 1 --cpu-seconds 0
run c1 --config c1 --gpus 1 --steps 20 --warmup 5
run c3 --config c3 --gpus 1 --steps 20 --warmup 5
run c5 --config c5 --gpus 1 --steps 20 --warmup 5
run c5_t64 --config c5 --gpus 1 --cpu-seconds 0
run partial --env marl_partial
run runner --env runner
run primal --env primal
bash tools/r02_profile.sh r02final_c2 --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 0 || exit $?
bash tools/r02_profile.sh r02final_c5 --config c5 --gpus 1 --cpu-seconds 0 --per-step-steps 0 || exit $?
echo "[$(date +%T)] done"
