#!/bin/bash
# round-2 call d: per-wave prologue / loop / epilogue clocks of the C2 rollout (diagnostic build).
set -o pipefail
OUT=gpurun_out/r02d
mkdir -p $OUT
timeout -k 10 300 python3 tools/clocks.py --envs 256,4096 --T 20 > $OUT/clocks_t20.txt 2>&1 || exit $?
timeout -k 10 300 python3 tools/clocks.py --envs 256,4096 --T 64 > $OUT/clocks_t64.txt 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/bench.json 2>&1 || exit $?
cat $OUT/*.txt $OUT/bench.json
