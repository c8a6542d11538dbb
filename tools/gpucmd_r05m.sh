#!/bin/bash
# Round 5, call M (diagnostic): C2 kernel time per launch (tools/tsweep.py, launch events,
# median of 7 replays) with kernel arguments in host memory (the HIP default) or device
# memory (HIP_FORCE_DEV_KERNARG=1), six interleaved rounds.
set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
for rep in 1 2 3 4 5 6; do
  timeout -k 10 200 python3 tools/tsweep.py --T 1,20,64 > $O/host_$rep.txt 2>&1 || { tail $O/host_$rep.txt; exit 1; }
  HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python3 tools/tsweep.py --T 1,20,64 > $O/dev_$rep.txt 2>&1 || { tail $O/dev_$rep.txt; exit 1; }
  echo "round $rep host: $(grep -E '^T=' $O/host_$rep.txt | awk '{print $4}' | tr '\n' ' ') dev: $(grep -E '^T=' $O/dev_$rep.txt | awk '{print $4}' | tr '\n' ' ')"
done
