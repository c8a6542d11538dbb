#!/bin/bash
# Round 3 (re-entry): full GPU suite at HEAD, the driver's bench line, and the C5
# generic rollout kernel's MAPFX_GABL ablations (1 no reward fold, 2 no window
# records, 3 neither, 8 no edge scan), T = 64 (bench default for c5).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03ae
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $OUT/tests.txt 2>&1 || { tail -40 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
timeout -k 10 200 python3 bench.py > $OUT/c2.json 2> $OUT/c2.err || { tail -20 $OUT/c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c2.json')); print('c2', d['value'], d['kernel_ms_per_launch'], d['roofline']['frac'])"
for v in "" _gabl1 _gabl2 _gabl3 _gabl8; do
  MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 200 python3 bench.py --config c5 --cpu-seconds 0 \
    --per-step-steps 0 --no-gather > $OUT/c5$v.json 2> $OUT/c5$v.err || { tail -20 $OUT/c5$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c5$v.json')); print('c5 lib$v', d['kernel_ms_per_launch'], d['timing']['kernel_ms_replays'])"
done
