#!/bin/bash
# SQ instruction / wait counters of the rollout kernel (separate passes).
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-sq}
V=${2:-all}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES SQ_INSTS_BRANCH" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_WAVE32_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set -d "$OUT/p$i" -o run --output-format csv -- python3 tools/pmc_probe.py $V > "$OUT/p$i.log" 2>&1 || echo "pass $i failed"
done
