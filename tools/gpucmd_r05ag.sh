#!/bin/bash
# Round 5, call AG: the mapfx-unit legs re-profiled after the FEAT_RUN change (c2 as the
# driver command, c2_step, c3, c5 through tools/r05_profile.sh), then their bench lines
# with those profiles in place.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ag
mkdir -p $O
P="bash tools/r05_profile.sh"
$P c2 "--config c2 --T 20 --E 4096" --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 0 || exit 1
$P c2_step "--config c2_step --T 1 --E 4096 --bench-kernel-key per_step.kernel" --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 200 || exit 1
$P c3 "--config c3 --T 64 --E 2048" --config c3 --cpu-seconds 0 --per-step-steps 0 || exit 1
$P c5 "--config c5 --T 64 --E 1024" --config c5 --cpu-seconds 0 --per-step-steps 0 || exit 1
cp gpurun_out/profiles/pmc_c2.json gpurun_out/profiles/pmc_c2_step.json gpurun_out/profiles/pmc_c3.json gpurun_out/profiles/pmc_c5.json profiles/
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
