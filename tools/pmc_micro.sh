#!/bin/bash
# TD / TCP / TA counters of the store microbenchmark (tools/micro/outputs)
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-micro}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 60 rocprofv3 --pmc TD_TD_BUSY TD_TC_STALL TCP_TCC_WRITE_REQ_LATENCY TCP_PENDING_STALL_CYCLES TCP_TCC_WRITE_REQ TCP_WRITE_TAGCONFLICT_STALL_CYCLES GRBM_GUI_ACTIVE -d "$OUT/p1" -o run --output-format csv -- tools/micro/outputs > "$OUT/p1.log" 2>&1 || exit 1
timeout -k 10 60 rocprofv3 --pmc TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d "$OUT/p2" -o run --output-format csv -- tools/micro/outputs > "$OUT/p2.log" 2>&1 || exit 1
