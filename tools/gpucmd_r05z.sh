#!/bin/bash
# Round 5, call Z: after the last partial.hip change, the MARL_PARTIAL leg profiled again
# (tools/r05_profile.sh) and the partial, runner and driver (C2 T = 20) lines with every
# profile in place (the C2 / C3 / C5 / primal profiles stay valid: their units' hashes
# are unchanged).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05z
mkdir -p $O
bash tools/r05_profile.sh partial "--config marl_partial --T 1 --E 4096 --match N=15 --match S=8" --env marl_partial --cpu-seconds 0 || exit 1
cp gpurun_out/profiles/pmc_partial.json profiles/
run() {
  local tag=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$tag.json')); r=d.get('roofline') or {}; print('$tag', d['value'], d['unit'], d['ms_per_step'], d.get('kernel_ms_per_launch', d.get('kernel_ms_per_step')), r.get('frac'), r.get('traffic'), (r.get('traffic_source') or '')[:70])"
}
run c2_t20 --gpus 1 --steps 20 --warmup 5
run partial --env marl_partial
run runner --env runner
