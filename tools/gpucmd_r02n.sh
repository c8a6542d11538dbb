#!/bin/bash
# round-2 call n: generic kernel rework (C5 block < 40 KB, block-cooperative window
# writer, occupancy-plane window) -- parity, then C5 / C2 bench lines, C5 profile.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02n
mkdir -p $OUT
echo "[$(date +%T)] gpu tests (generic kernel)"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "occ or full_size or rollout_equals or batched_step or primal or autoreset or invalid" > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
echo "[$(date +%T)] c5 driver flags"
timeout -k 10 300 python3 bench.py --config c5 --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/c5_k20.json 2> $OUT/c5_k20.err || exit $?
cat $OUT/c5_k20.json
echo "[$(date +%T)] c5 T=64"
timeout -k 10 300 python3 bench.py --config c5 --gpus 1 --cpu-seconds 0 --per-step-steps 0 > $OUT/c5_t64.json 2> $OUT/c5_t64.err || exit $?
cat $OUT/c5_t64.json
echo "[$(date +%T)] c2 driver flags"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/c2.json 2> $OUT/c2.err || exit $?
cat $OUT/c2.json
bash tools/r02_profile.sh r02n_c5 --config c5 --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 0
