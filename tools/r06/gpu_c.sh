#!/bin/bash
# Round 6, call C: the runner's next-MAC-call compaction fused into the env step
# (one launch per runner step) -- runner / partial GPU tests, then bench --env runner
# interleaved against the same sources built with the round-5 separate compaction
# kernel (varlibs/libmapfx_sepcmp.so, -DMAPFX_RUNNER_SEPARATE_CMP; the macro was removed
# from runner.hip after this A/B, profiles/r06_runner_fused_cmp_ab.txt).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_runner.py tests/test_gpu_partial.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for rep in 1 2 3; do
  for v in new sep; do
    if [ $v = new ]; then L=""; else L=$PWD/varlibs/libmapfx_sepcmp.so; fi
    MAPFX_LIB=$L timeout -k 10 200 python3 bench.py --env runner --cpu-seconds 0 > $O/runner_${v}_$rep.json 2> $O/runner_${v}_$rep.err || { tail $O/runner_${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/runner_${v}_$rep.json')); print('$v $rep runner', d['ms_per_step'], d['value'])"
  done
done
