#!/bin/bash
# Round 5, call B: where the per-step launch and the T = 20 headline spend their time now.
# Graph back-to-back floor, per-step time vs env count, block-0 stamps (diagnostic build).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 120 python3 tools/graph_gap.py > $O/graph_gap.txt 2>&1 && cat $O/graph_gap.txt || exit 1
timeout -k 10 300 python3 tools/scale_step.py --envs 64,256,1024,4096,16384 > $O/scale_step.txt 2>&1 && cat $O/scale_step.txt || exit 1
timeout -k 10 200 python3 tools/pstamps_step.py > $O/pstamps_step.txt 2>&1 && cat $O/pstamps_step.txt || exit 1
MAPFX_PROBE_T=20 timeout -k 10 200 python3 tools/stamps.py > $O/stamps_t20.txt 2>&1 && cat $O/stamps_t20.txt || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['kernel_ms_per_launch'], d['timing']['kernel_ms_replays'], d['per_step']['kernel_ms'], d['per_step']['ms_per_step'])"
