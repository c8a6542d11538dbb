#!/bin/bash
# Round 4, first GPU call: the full GPU suite at the round's starting point (plus the
# new compact-gather, fold-placement and PRIMAL parity tests) and the driver's bench line.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04a
mkdir -p $OUT
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $OUT/tests.txt 2>&1 || { tail -60 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c2.json 2> $OUT/bench_c2.err \
  || { tail -20 $OUT/bench_c2.err; exit 1; }
tail -c 600 $OUT/bench_c2.json; echo
