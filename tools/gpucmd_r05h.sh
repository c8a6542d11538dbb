#!/bin/bash
# Round 5, call H (diagnostic): where the fused compaction's time goes. Runner bench +
# kernel trace with the shipped library and three timing-only variants
# (varlibs/libmapfx_cmpV.so, -DMAPFX_CMP_DIAG=V: 1 no compaction tail, 2 no bit ORs,
# 3 the separate compaction kernel).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05h
mkdir -p $O
for v in 0 1 2 3 0; do
  if [ $v = 0 ]; then L=""; else L=$PWD/varlibs/libmapfx_cmp$v.so; fi
  MAPFX_LIB=$L timeout -k 10 300 python3 bench.py --env runner --cpu-seconds 0 > $O/bench_$v.json 2> $O/bench_$v.err \
    || { tail -20 $O/bench_$v.err; exit 1; }
  MAPFX_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_$v -o run --output-format csv \
    -- python3 bench.py --env runner --cpu-seconds 0 > $O/traced_$v.json 2> $O/trace_$v.err || { tail -20 $O/trace_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); print('variant $v', d['value'], d['ms_per_step'])"
  python3 tools/trace_gaps.py $O/trace_$v | head -4
done
