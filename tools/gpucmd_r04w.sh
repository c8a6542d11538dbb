#!/bin/bash
# Round 4: runner compaction with the chunk's flags kept in registers -- runner parity, A/B.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04w
mkdir -p $OUT
L=mapf-marl_amd/mapfx
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_runner.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1 \
  || { grep -E "FAIL|Error" $OUT/tests.txt | head -30; tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
for r in 1 2; do
  for lib in libmapfx libmapfx_prev; do
    MAPFX_LIB=$PWD/$L/$lib.so timeout -k 10 300 python3 bench.py --env runner --cpu-seconds 0 > $OUT/$lib.r$r.json 2> $OUT/$lib.r$r.err \
      || { tail -20 $OUT/$lib.r$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$lib.r$r.json')); print('$lib r$r', d['value'], d['ms_per_step'])"
  done
done
