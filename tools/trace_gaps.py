#!/usr/bin/env python3
"""Timeline summary of a rocprofv3 --kernel-trace directory: per-kernel count and mean
duration over the last `--tail` dispatches, and the idle gaps between consecutive
kernels there (the GPU waiting on the host or on launch latency).
usage: python3 tools/trace_gaps.py TRACE_DIR [--tail N]"""
import argparse
import csv
import glob
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--tail", type=int, default=3000)
    args = ap.parse_args()
    rows = []
    for p in glob.glob(os.path.join(args.trace, "**", "*kernel_trace.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    rows = rows[-args.tail:]
    if not rows:
        print("no kernels")
        return
    per = {}
    for s, e, n in rows:
        per.setdefault(n, []).append(e - s)
    span = rows[-1][1] - rows[0][0]
    busy = sum(e - s for s, e, _ in rows)
    print("dispatches %d over %.1f us, kernels busy %.1f%%" % (len(rows), span / 1e3, 100.0 * busy / span))
    for n, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print("%6d x %8.2f us  %5.1f%%  %s" % (len(d), statistics.mean(d) / 1e3, 100.0 * sum(d) / span, n[:110]))
    gaps = [rows[i + 1][0] - rows[i][1] for i in range(len(rows) - 1)]
    gaps.sort()
    q = lambda f: gaps[min(len(gaps) - 1, int(f * len(gaps)))] / 1e3  # noqa: E731
    print("gaps us: p10 %.2f p50 %.2f p90 %.2f p99 %.2f mean %.2f" % (q(.1), q(.5), q(.9), q(.99),
                                                                       statistics.mean(gaps) / 1e3))


if __name__ == "__main__":
    main()
