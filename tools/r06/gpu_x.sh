#!/bin/bash
# Round 6, call X: the two-rank rehearsal at the final build (2 ranks on cuda:0, gloo).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06x
mkdir -p $O
timeout -k 10 300 python3 bench.py --gpus 2 --rehearse-shared-gpu --steps 40 --warmup 20 --chunk 20 --cpu-seconds 0 --per-step-steps 0 > $O/rehearse.json 2> $O/rehearse.err || { tail $O/rehearse.err; exit 1; }
grep '^{' $O/rehearse.json > $O/rehearse_line.json
python3 -c "import json; d=json.load(open('$O/rehearse_line.json')); print(d['n_gpus'], d['value'], d['config']['parallelism'], d['gather']['collective'][:60], d['build_id'][:30])"
