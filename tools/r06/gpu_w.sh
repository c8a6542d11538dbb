#!/bin/bash
# Round 6, call W: the store-wave split kernel at T = 1 (rollout chunks of one step)
# against the per-step drop-in kernel, same box, three rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06w
mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 16 --warmup 4 --chunk 1 --cpu-seconds 0 --per-step-steps 200 > $O/t1_$rep.json 2> $O/t1_$rep.err || { tail $O/t1_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/t1_$rep.json')); print('T1', $rep, 'split launch', d['kernel_ms_per_launch'], 'wall/step', d['ms_per_step'], '| per-step kernel', d['per_step']['kernel_ms'], d['per_step']['ms_per_step'], d['kernel'][:60])"
done
