#!/bin/bash
# Wall vs kernel time of the driver's bench command under HIP / ROCr runtime
# settings that affect launch and completion latency (diagnostic).
set -o pipefail
OUT=gpurun_out/launch_env
mkdir -p $OUT
B="--gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 0"
run() {  # tag, env assignments...
  local tag=$1; shift
  for i in 1 2 3; do
    timeout -k 10 120 env "$@" python3 bench.py $B > $OUT/$tag.$i.json 2> $OUT/$tag.$i.err || return $?
  done
  python3 -c "
import json
for i in (1, 2, 3):
    d = json.load(open('$OUT/$tag.%d.json' % i)); t = d['timing']
    print('$tag', i, t['wall_ms'], t['kernel_ms_events'], t['wall_over_kernel'])"
}
run default A=1 || exit $?
run nointr HSA_ENABLE_INTERRUPT=0 || exit $?
run actwait ROC_ACTIVE_WAIT_TIMEOUT=100 || exit $?
run kernarg0 HIP_FORCE_DEV_KERNARG=0 || exit $?
run kernarg1 HIP_FORCE_DEV_KERNARG=1 || exit $?
# per-step path: the default library vs one built with kernarg preload (16 SGPRs)
P="--gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 400"
for v in base preload16; do
  if [ $v = base ]; then unset MAPFX_LIB; else export MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx_$v.so; fi
  timeout -k 10 120 python3 bench.py $P > $OUT/ps_$v.json 2> $OUT/ps_$v.err || exit $?
  python3 -c "
import json
d = json.load(open('$OUT/ps_$v.json')); p = d['per_step']
print('$v per_step', p['ms_per_step'], p['kernel_ms'], 'fused', d['kernel_ms_per_launch'])"
done
