#!/bin/bash
# Round 6, call E: the fused compaction as the launch's FIRST workgroup (dispatched
# before the env workgroups; 16-flag chunks as one 16-byte load) -- runner tests, the
# runner bench line three times and a kernel trace of it.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_runner.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for rep in 1 2 3; do
  timeout -k 10 200 python3 bench.py --env runner --cpu-seconds 0 > $O/runner_$rep.json 2> $O/runner_$rep.err || { tail $O/runner_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/runner_$rep.json')); print('new $rep runner', d['ms_per_step'], d['value'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv \
  -- python3 bench.py --env runner --steps 300 --warmup 100 --cpu-seconds 0 > $O/bench_traced.json 2> $O/trace.err || { tail $O/trace.err; exit 1; }
python3 tools/trace_gaps.py $O/trace --tail 2000 > $O/gaps.txt
head -8 $O/gaps.txt
