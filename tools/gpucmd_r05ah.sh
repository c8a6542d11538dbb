#!/bin/bash
# Round 5, call AH: the whole GPU suite, smoke() and the driver line at the final build.
set -o pipefail
O=gpurun_out/r05ah
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default.json')); r=d['roofline']; print('default', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'], r['frac'], r['traffic'], r['traffic_source'][:60])"
