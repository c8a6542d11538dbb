#!/bin/bash
# SQ / TA / TD / TCP counters of the runner rollout at several env counts (one pass per set).
# usage: tools/pmc_cmp.sh TAG "E1 E2 ..."   (MAPFX_LIB selects the library variant)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-cmp}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
sets=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
      "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_SCA SQ_IFETCH SQ_INST_CYCLES_VMEM_WR TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES"
      "TD_TD_BUSY TD_TC_STALL TCP_TCC_WRITE_REQ_LATENCY TCP_PENDING_STALL_CYCLES TCP_WRITE_TAGCONFLICT_STALL_CYCLES TCP_TCC_WRITE_REQ SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR")
for E in $2; do
  i=0
  for set in "${sets[@]}"; do
    i=$((i+1))
    MAPFX_PROBE_E=$E timeout -k 10 120 rocprofv3 --pmc $set -d "$OUT/e${E}_p$i" -o run --output-format csv -- python3 tools/pmc_probe.py all > "$OUT/e${E}_p$i.log" 2>&1 || { echo "pass $E/$i failed"; exit 1; }
  done
done
