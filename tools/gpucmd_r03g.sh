#!/bin/bash
# Round 3: C2 split kernel with the batched reward fold (code ring + table) and
# fetch-time action addresses: split / runner parity, then the T sweep.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03g
mkdir -p $OUT
echo "[$(date +%T)] parity"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_runner.py -q -x --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; tail -3 $OUT/tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
for T in 1 4 20 64; do
  timeout -k 10 120 python3 bench.py --gpus 1 --steps $T --warmup $T --cpu-seconds 0 --per-step-steps 0 > $OUT/c2.T$T.json 2>$OUT/c2.T$T.err || exit $?
  python3 -c "import json; d=json.load(open('$OUT/c2.T$T.json')); print('T$T', d['value'], d['kernel_ms_per_launch'], d['timing']['kernel_ms_replays'], d['roofline']['frac'])"
done
echo "[$(date +%T)] done"
