#!/bin/bash
# Round 4 end, after the last kernel changes: full GPU suite, smoke(), the driver's
# C2 line (T = 20) and the default C2 / C3 lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04_final_c
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 \
  || { grep -E "FAIL|Error" $O/gpu_tests.txt | head -30; tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
run() {
  local tag=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$tag.json')); r=d.get('roofline') or {}; print('$tag', d['value'], d['unit'], d['ms_per_step'], d.get('kernel_ms_per_launch'), r.get('frac'), r.get('traffic'))"
}
run c2_t20 --gpus 1 --steps 20 --warmup 5
run c2
run c3 --config c3
