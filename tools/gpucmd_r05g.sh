#!/bin/bash
# Round 5, call G: the runner's bs compaction fused into the env step (its last wave).
# Runner GPU tests, the runner bench line twice, and a kernel trace of the runner bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_runner.py -x -q --timeout 300 --timeout-method thread \
  > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --env runner --cpu-seconds 0 > $O/bench_runner_$i.json 2> $O/bench_runner_$i.err \
    || { tail -20 $O/bench_runner_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_runner_$i.json')); print('runner', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv \
  -- python3 bench.py --env runner --cpu-seconds 0 > $O/bench_traced.json 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
python3 tools/trace_gaps.py $O/trace > $O/gaps.txt && cat $O/gaps.txt
