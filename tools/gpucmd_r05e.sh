#!/bin/bash
# Round 5, call E: every bench leg profiled at HEAD (trace + FETCH / WRITE + LDS + SQ
# passes of the same command, tools/r05_profile.sh -> gpurun_out/profiles/pmc_*.json keyed
# to the kernel instance and build the traced line reports), then every bench line with
# those profiles in place.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
P="bash tools/r05_profile.sh"
$P c2 "--config c2 --T 20 --E 4096" --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 0 || exit 1
$P c2_step "--config c2_step --T 1 --E 4096 --bench-kernel-key per_step.kernel" --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 200 || exit 1
$P c3 "--config c3 --T 64 --E 2048" --config c3 --cpu-seconds 0 --per-step-steps 0 || exit 1
$P c5 "--config c5 --T 64 --E 1024" --config c5 --cpu-seconds 0 --per-step-steps 0 || exit 1
$P partial "--config marl_partial --T 1 --E 4096 --match N=15 --match S=8" --env marl_partial --cpu-seconds 0 || exit 1
$P primal "--config primal --T 64 --E 4096" --env primal --cpu-seconds 0 || exit 1
cp gpurun_out/profiles/pmc_*.json profiles/
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$tag.json')); r=d.get('roofline') or {}; print('$tag', d['value'], d['unit'], d['ms_per_step'], d.get('kernel_ms_per_launch', d.get('kernel_ms_per_step')), r.get('frac'), r.get('traffic'), (r.get('traffic_source') or '')[:60])"
}
run c2_t20 --gpus 1 --steps 20 --warmup 5
run c2
run c3 --config c3
run c5 --config c5
run c1 --config c1
run partial --env marl_partial
run primal --env primal
run runner --env runner
