#!/bin/bash
# Round 3: PRIMAL call loop with two-deep read-ahead and forwarded records: parity,
# then the bench line twice and the measurement recipe.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03t
mkdir -p $OUT
echo "[$(date +%T)] primal tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_primal.py -q -x --timeout 120 --timeout-method thread > $OUT/primal_tests.txt 2>&1
rc=$?; tail -3 $OUT/primal_tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  timeout -k 10 120 python3 bench.py --env primal --cpu-seconds 0 > $OUT/primal.$rep.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('$OUT/primal.$rep.json')); print('primal', d['value'], d['kernel_ms_per_launch'], d['roofline']['frac'])"
done
bash tools/r03_profile.sh r03_primal2 --env primal --cpu-seconds 0 || exit $?
echo "[$(date +%T)] done"
