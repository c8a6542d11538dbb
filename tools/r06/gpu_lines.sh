#!/bin/bash
# Round 6: every bench line with the round-6 profiles in place (profiles/pmc_*.json):
# the driver's command (C2, T = 20), C2 default args, C3, C5, C1, MARL_PARTIAL, PRIMAL
# and the runner, each once; lines under gpurun_out/r06_lines/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_lines
mkdir -p $O
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$tag.json')); r=d.get('roofline') or {}; print('$tag', d['value'], d['unit'], d['ms_per_step'], d.get('kernel_ms_per_launch', d.get('kernel_ms_per_step')), r.get('frac'), r.get('traffic'), (r.get('traffic_source') or '')[:40])"
}
run c2_t20 --gpus 1 --steps 20 --warmup 5
run c2
run c3 --config c3
run c5 --config c5
run c1 --config c1
run partial --env marl_partial
run primal --env primal
run runner --env runner
