#!/bin/bash
# Round 5, call AC: the driver command's profile retaken with >= 15 event-timed replay
# launches in the bench (so the trace averages 17 launches of the instance, not 7), and
# the driver line beside it.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ac
mkdir -p $O
bash tools/r05_profile.sh c2 "--config c2 --T 20 --E 4096" --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 0 || exit 1
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c2_t20.json 2> $O/bench_c2_t20.err || { tail -20 $O/bench_c2_t20.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c2_t20.json')); r=d['roofline']; print('c2_t20', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'], r['frac'], r['traffic'], r['traffic_source'][:60])"
