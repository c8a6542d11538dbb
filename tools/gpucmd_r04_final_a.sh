#!/bin/bash
# Round 4 end: the full GPU test suite, smoke(), and every bench line (the driver's
# default command first), into gpurun_out/r04_final/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04_final
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 \
  || { grep -E "FAIL|Error" $O/gpu_tests.txt | head -30; tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$tag.json')); r=d.get('roofline') or {}; print('$tag', d['value'], d['unit'], d['ms_per_step'], r.get('frac'), r.get('traffic'))"
}
run c2
run c3 --config c3
run c5 --config c5
run c1 --config c1
run partial --env marl_partial
run primal --env primal
run runner --env runner
