#!/bin/bash
# Round 6, call A: the race fix in the split's last fold + the per-leg bench parity
# tests (test_bench_leg_matches_oracle, FEAT_RUN cases), then the default bench line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "generic_rollout_every_step or test_autoreset or bench_leg" > $O/tests.txt 2>&1
rc=$?
tail -3 $O/tests.txt
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.txt | head -40; exit 1; fi
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_c2_t20.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
tail -c 600 $O/bench_c2_t20.json
