#!/bin/bash
# Round 6, call N: the N-rank bench path rehearsed on the one-GPU box (2 ranks on cuda:0,
# collectives over gloo -- never a scaling number; the line's collective label says gloo)
# and the whole GPU suite + smoke() at the current sources.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06n
mkdir -p $O
timeout -k 10 300 python3 bench.py --gpus 2 --rehearse-shared-gpu --steps 40 --warmup 20 --chunk 20 --cpu-seconds 0 --per-step-steps 0 > $O/rehearse.json 2> $O/rehearse.err || { tail $O/rehearse.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/rehearse.json')); print(d['n_gpus'], d['config']['parallelism'], d['gather']['collective'])"
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?
tail -3 $O/gpu_tests.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
exit $rc
