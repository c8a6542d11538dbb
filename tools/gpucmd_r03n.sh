#!/bin/bash
# Round 3: four-wave split (MOVE + MAP + 2 store waves): parity first, then T sweep.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03n
mkdir -p $OUT
echo "[$(date +%T)] parity"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_runner.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; tail -5 $OUT/tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
for T in 1 20 64; do
  timeout -k 10 120 python3 bench.py --gpus 1 --steps $T --warmup $T --cpu-seconds 0 --per-step-steps 0 > $OUT/c2.T$T.json 2>$OUT/c2.T$T.err || exit $?
  python3 -c "import json; d=json.load(open('$OUT/c2.T$T.json')); print('T$T', d['value'], d['kernel_ms_per_launch'], d['timing']['kernel_ms_replays'], d['roofline']['frac'])"
done
done
echo "[$(date +%T)] done"
