#!/bin/bash
# round-2 call b: host-side timing probe + SQ instruction/wait counters of the C2 rollout.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02b
mkdir -p $OUT
echo "[$(date +%T)] wall probe"
timeout -k 10 300 python3 tools/wall_probe.py > $OUT/wall_probe.json 2> $OUT/wall_probe.err || exit $?
cat $OUT/wall_probe.json
B="--gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 0"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES SQ_INSTS_BRANCH"; do
  i=$((i+1))
  echo "[$(date +%T)] sq pass $i"
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/sq$i -o run --output-format csv -- python3 bench.py $B > $OUT/sq$i.json 2> $OUT/sq$i.err || exit $?
done
echo "[$(date +%T)] done"
