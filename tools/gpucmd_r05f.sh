#!/bin/bash
# Round 5, call F: the split kernel's last step with its a + b parts in one interval
# (parity: the split suite; A/B against the previous build libmapfx_prev.so; T sweep).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f
mkdir -p $O
L=$PWD/mapf-marl_amd/mapfx
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -1 $O/tests.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.txt | head -30; exit 1; }
for r in 1 2 3; do
  for v in new prev; do
    lib=$L/libmapfx.so; [ $v = prev ] && lib=$L/libmapfx_prev.so
    MAPFX_LIB=$lib timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 0 > $O/c2_${v}_$r.json 2> $O/c2_${v}_$r.err || { tail $O/c2_${v}_$r.err; exit 1; }
    MAPFX_LIB=$lib timeout -k 10 300 python3 bench.py --cpu-seconds 0 --per-step-steps 0 > $O/c2d_${v}_$r.json 2> $O/c2d_${v}_$r.err || { tail $O/c2d_${v}_$r.err; exit 1; }
    python3 -c "import json; a=json.load(open('$O/c2_${v}_$r.json')); b=json.load(open('$O/c2d_${v}_$r.json')); print('$v $r T20', a['kernel_ms_per_launch'], a['timing']['kernel_ms_replays'], '| T64', b['kernel_ms_per_launch'])"
  done
done
MAPFX_LIB=$L/libmapfx.so timeout -k 10 300 python3 tools/tsweep.py > $O/tsweep_new.txt 2>&1 && cat $O/tsweep_new.txt || exit 1
MAPFX_LIB=$L/libmapfx_prev.so timeout -k 10 300 python3 tools/tsweep.py > $O/tsweep_prev.txt 2>&1 && cat $O/tsweep_prev.txt || exit 1
