#!/bin/bash
# Round 5, call P (diagnostic, timing only): what the runner's env step pays over the plain
# step -- varlibs/libmapfx_ablV.so (-DMAPFX_RUN_ABL=V): 1 no EpisodeBatch row writes
# (actions, one-hot, reward, terminated, state, avail, filled), 2 no action-row lookup
# (row = env), 3 both; runner bench + kernel trace, interleaved.
set -o pipefail
O=gpurun_out/r05p
mkdir -p $O
for rep in 1 2; do
for v in 0 1 2 3; do
  if [ $v = 0 ]; then L=""; else L=$PWD/varlibs/libmapfx_abl$v.so; fi
  MAPFX_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_${v}_$rep -o run --output-format csv \
    -- python3 bench.py --env runner --cpu-seconds 0 > $O/b_${v}_$rep.json 2> $O/b_${v}_$rep.err || { tail $O/b_${v}_$rep.err; exit 1; }
  echo "variant $v rep $rep: $(python3 tools/trace_gaps.py $O/trace_${v}_$rep | grep -E 'partial_kernel|compact' | awk '{print $3}' | tr '\n' ' ')"
done
done
