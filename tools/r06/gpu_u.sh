#!/bin/bash
# Round 6, call U: the runner's next-run EpisodeBatch made one run ahead on a side stream
# (mapfx.runners.ParallelRunner._prefetch_batch) -- runner GPU tests, then the runner
# line with and without it, interleaved, three rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06u
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_runner.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for rep in 1 2 3; do
  for v in prefetch reset; do
    if [ $v = prefetch ]; then F=""; else F="--no-batch-prefetch"; fi
    timeout -k 10 300 python3 bench.py --env runner $F > $O/runner_${v}_$rep.json 2> $O/runner_${v}_$rep.err || { tail $O/runner_${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/runner_${v}_$rep.json')); print('$v', $rep, d['value'], d['ms_per_step'])"
  done
done
