#!/usr/bin/env python3
"""Summarise tools/pmc_cmp.sh output: mean counter value per dispatch of the rollout kernel."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "mapf_wave_kernel<5, true"
tab = collections.defaultdict(dict)
for p in sorted(glob.glob(os.path.join(root, "e*_p*", "run_counter_collection.csv"))):
    e = os.path.basename(os.path.dirname(p)).split("_")[0]
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(p)):
        if kern in r["Kernel_Name"]:
            d[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in d.items():
        tab[k][e] = sum(v) / len(v)
es = sorted({e for v in tab.values() for e in v}, key=lambda x: int(x[1:]))
print("%-36s" % "counter" + "".join("%16s" % e for e in es))
for k in sorted(tab):
    print("%-36s" % k + "".join("%16.0f" % tab[k].get(e, float("nan")) for e in es))
