#!/bin/bash
# Round 5, call V (diagnostic): the driver launch's host side under HIP wait settings
# (tools/launch_probe.py): default, hipDeviceScheduleSpin / Yield / BlockingSync, and
# ROC_ACTIVE_WAIT_TIMEOUT; then the driver's command with spin scheduling via the env.
set -o pipefail
O=gpurun_out/r05v
mkdir -p $O
for rep in 1 2; do
  for cfg in "-1" "1" "2" "4"; do
    timeout -k 10 200 python3 tools/launch_probe.py --sched $cfg > $O/p_${cfg}_$rep.txt 2>&1 || { tail $O/p_${cfg}_$rep.txt; exit 1; }
    echo "sched $cfg rep $rep: $(grep -E 'plan call|tiny' $O/p_${cfg}_$rep.txt | awk '{print $(NF-1)}' | tr '\n' ' ')"
  done
  for w in 0 100 5000; do
    ROC_ACTIVE_WAIT_TIMEOUT=$w timeout -k 10 200 python3 tools/launch_probe.py > $O/w_${w}_$rep.txt 2>&1 || { tail $O/w_${w}_$rep.txt; exit 1; }
    echo "ROC_ACTIVE_WAIT_TIMEOUT=$w rep $rep: $(grep -E 'plan call|tiny' $O/w_${w}_$rep.txt | awk '{print $(NF-1)}' | tr '\n' ' ')"
  done
done
