#!/bin/bash
# Round 5, call K (diagnostic): the driver's command (bench.py --gpus 1 --steps 20
# --warmup 5) under HIP runtime wait / kernel-argument settings, interleaved.
set -o pipefail
O=gpurun_out/r05k
mkdir -p $O
run() {  # tag, env assignments...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 0 \
    > $O/b_$tag.json 2> $O/b_$tag.err || { tail -20 $O/b_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$tag.json')); print('$tag', '$*', d['value'], d['ms_per_step'], d.get('kernel_ms_per_launch'))"
}
for rep in 1 2 3; do
  run base_$rep X=1
  run wait200_$rep ROC_ACTIVE_WAIT_TIMEOUT=200
  run wait0_$rep ROC_ACTIVE_WAIT_TIMEOUT=0
  run devka_$rep HIP_FORCE_DEV_KERNARG=1
  run both_$rep ROC_ACTIVE_WAIT_TIMEOUT=200 HIP_FORCE_DEV_KERNARG=1
done
