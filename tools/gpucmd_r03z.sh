#!/bin/bash
# Round 3: primal_seq_kernel with the slim phase A (biased cells, branch-free) against the
# first seq kernel (libmapfx_seq0.so), PRIMAL tests, then an SQ pass of the new one.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03z
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_primal.py -x -q --timeout 120 --timeout-method thread \
  > $OUT/primal_tests.txt 2>&1 || { tail -40 $OUT/primal_tests.txt; exit 1; }
tail -2 $OUT/primal_tests.txt
for rep in 1 2; do
for v in "" _seq0; do
  MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 200 python3 bench.py --env primal --cpu-seconds 0 \
    > $OUT/primal$v.json 2> $OUT/primal$v.err || { tail -20 $OUT/primal$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/primal$v.json')); print('lib$v', d['kernel_ms_per_launch'], d['timing'].get('kernel_ms_replays'))"
done
done
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/pmc_sq -o run --output-format csv \
  -- python3 bench.py --env primal --cpu-seconds 0 > $OUT/bench_sq.json 2> $OUT/sq.err || exit 1
echo done
