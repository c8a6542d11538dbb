#!/bin/bash
# Round 6, call S: box-to-box spread -- the driver's command and the runner line, three
# times each, at the final build (lines under gpurun_out/r06s/).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s
mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/c2_t20_$rep.json 2> $O/c2_t20_$rep.err || { tail $O/c2_t20_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c2_t20_$rep.json')); print('c2_t20', $rep, d['value'], d['ms_per_step'], d['kernel_ms_per_launch'], d['per_step']['kernel_ms'])"
  timeout -k 10 300 python3 bench.py --env runner > $O/runner_$rep.json 2> $O/runner_$rep.err || { tail $O/runner_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/runner_$rep.json')); print('runner', $rep, d['value'], d['ms_per_step'])"
done
# the T = 15 / 16 boundary cases of the split parity test
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "runner_rollout_every_step" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
