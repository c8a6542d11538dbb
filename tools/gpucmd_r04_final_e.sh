#!/bin/bash
# Round 4 end (last kernel change: partial early write-back): full GPU suite, smoke(),
# the partial and runner lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04_final_e
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 \
  || { grep -E "FAIL|Error" $O/gpu_tests.txt | head -30; tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python3 bench.py --env marl_partial > $O/bench_partial.json 2> $O/bench_partial.err || { tail $O/bench_partial.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_partial.json')); print('partial', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 300 python3 bench.py --env runner > $O/bench_runner.json 2> $O/bench_runner.err || { tail $O/bench_runner.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_runner.json')); print('runner', d['value'], d['ms_per_step'])"
