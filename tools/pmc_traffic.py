#!/usr/bin/env python3
"""Summarise rocprofv3 outputs of bench.py into profiles/.

  python tools/pmc_traffic.py --trace DIR --fetch DIR --write DIR [--lds DIR] --out profiles/pmc_c2.json
      [--kernel mapf_rollout_kernel] [--config c2 --T 64 --E 4096] [--command "..."]
      [--bench-json DIR/bench_traced.json]

* --bench-json: the bench line of the profiled command.  Its "kernel" (the exact
  instance the bench launched, mapfx_last_kernel) selects the kernel in every pass
  instead of the --kernel substring, and its "build_id" (mapfx_build_id: source
  hash + git head) is recorded: bench.py cites the profile only for that same build
  and kernel instance.

* --trace: a `rocprofv3 --kernel-trace --stats --output-format csv` directory; the
  per-kernel stats CSV is copied and the kernel's average duration recorded.
* --fetch / --write: separate `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE`
  passes (TCC FETCH_SIZE costs 3 of the 4 TCC slots, so they cannot share a pass).
  Units are KB.  gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reads
  half of a wide coalesced stream's bytes, so it is doubled; WRITE_SIZE is taken
  as is.  Per-launch HBM traffic = (2*FETCH_SIZE + WRITE_SIZE) * 1024 bytes,
  averaged over the kernel's full-size dispatches.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import shutil
import statistics


def _rows(d, pattern):
    out = []
    for p in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        with open(p, newline="") as f:
            out.extend(csv.DictReader(f))
    return out


def _col(row, *names):
    for n in names:
        if n in row:
            return row[n]
    raise KeyError(names)


def instance(name):
    """The kernel instance part of a demangled name: up to the parameter list that
    follows the template arguments (rocprofv3 and __cxa_demangle agree on it)."""
    i = name.find("<")
    j = name.find("(", i) if i >= 0 else -1
    return (name[:j] if j > 0 else name).strip()


def kernel_match(kernel, name):
    """--kernel is a substring; a full demangled name (from --bench-json) must name the
    same instance."""
    if "<" in kernel:
        return instance(kernel) == instance(name)
    return kernel in name


def pmc_values(d, kernel, counter):
    per_dispatch = {}
    for r in _rows(d, "*counter_collection.csv"):
        if not kernel_match(kernel, _col(r, "Kernel_Name", "KernelName")):
            continue
        if _col(r, "Counter_Name", "CounterName") != counter:
            continue
        did = _col(r, "Dispatch_Id", "DispatchId", "Correlation_Id")
        per_dispatch[did] = per_dispatch.get(did, 0.0) + float(_col(r, "Counter_Value",
                                                                     "CounterValue"))
    vals = sorted(per_dispatch.values())
    if not vals:
        return None, 0
    big = [v for v in vals if v >= 0.5 * vals[-1]]  # full-size launches only
    return statistics.mean(big), len(big)


def trace_stats(d, kernel, out_dir, tag):
    stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    res = {}
    for p in stats:
        dst = os.path.join(out_dir, "%s_kernel_stats.csv" % tag)
        shutil.copy(p, dst)
        res["stats_csv"] = os.path.relpath(dst, os.path.dirname(out_dir))
        with open(p, newline="") as f:
            for r in csv.DictReader(f):
                name = _col(r, "Name", "KERNEL_NAME", "Kernel_Name")
                if kernel_match(kernel, name):
                    res.setdefault("kernels", []).append({
                        "name": name, "calls": int(float(_col(r, "Calls"))),
                        "avg_ns": float(_col(r, "AverageNs", "Average_Ns")),
                        "total_ns": float(_col(r, "TotalDurationNs", "Total_Duration_Ns"))})
    # per-dispatch durations from the kernel trace
    durs = []
    rows = [r for r in _rows(d, "*kernel_trace.csv")
            if kernel_match(kernel, _col(r, "Kernel_Name", "KernelName"))]
    rows.sort(key=lambda r: int(_col(r, "Start_Timestamp")))
    starts, ends = [], []
    for r in rows:
        s0, e0 = int(_col(r, "Start_Timestamp")), int(_col(r, "End_Timestamp"))
        starts.append(s0)
        ends.append(e0)
        durs.append(e0 - s0)
    if durs:
        res["dispatches"] = len(durs)
        res["median_ns"] = statistics.median(durs)
        res["dispatch_ns"] = durs   # in launch order
        # begin of dispatch i + 1 minus end of dispatch i (negative: the two overlapped)
        res["gap_ns"] = [starts[i + 1] - ends[i] for i in range(len(starts) - 1)]
    return res


LDS_COUNTERS = ("SQ_WAVES", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE",
                "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES")


def lds_summary(d, kernel):
    """LDS counters of the kernel (one `rocprofv3 --pmc` pass of 8 SQ counters),
    averaged over its full-size dispatches, with the derived ratios."""
    out = {}
    for c in LDS_COUNTERS:
        v, n = pmc_values(d, kernel, c)
        if v is not None:
            out[c] = v
            out["dispatches"] = n
    if out.get("SQ_LDS_IDX_ACTIVE"):
        out["bank_conflict_cycles_frac"] = out.get("SQ_LDS_BANK_CONFLICT", 0.0) / out["SQ_LDS_IDX_ACTIVE"]
    if out.get("SQ_WAVES"):
        out["lds_insts_per_wave"] = out.get("SQ_INSTS_LDS", 0.0) / out["SQ_WAVES"]
    if out.get("SQ_WAVE_CYCLES"):
        out["lds_issue_stall_frac_of_wave_cycles"] = out.get("SQ_WAIT_INST_LDS", 0.0) / out["SQ_WAVE_CYCLES"]
        out["lds_active_frac_of_wave_cycles"] = out.get("SQ_ACTIVE_INST_LDS", 0.0) / out["SQ_WAVE_CYCLES"]
    out["note"] = ("SQ_LDS_BANK_CONFLICT = extra LDS-array cycles from bank conflicts, "
                   "SQ_LDS_IDX_ACTIVE = all LDS-array cycles (MI355X_MICROARCH.md LDS)")
    return out


SQ_COUNTERS = ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAIT_ANY",
               "SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES")


def sq_summary(d, kernel):
    """Issue / wait counters of the kernel (one pass of 8 SQ counters), per wave and as
    fractions of the wave cycles: where a wave's time goes (issue vs dependency wait)."""
    out = {}
    for c in SQ_COUNTERS:
        v, n = pmc_values(d, kernel, c)
        if v is not None:
            out[c] = v
            out["dispatches"] = n
    w = out.get("SQ_WAVES")
    if w:
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
            if c in out:
                out[c.lower()[3:] + "_per_wave"] = out[c] / w
    wc = out.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
            if c in out:
                out[c.lower()[3:] + "_frac_of_wave_cycles"] = out[c] / wc
    out["note"] = ("SQ_WAIT_ANY: wave cycles waiting on any dependency (vmcnt / lgkmcnt / "
                   "expcnt); SQ_WAIT_INST_ANY: cycles waiting for an instruction issue slot")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--out", required=True)
    ap.add_argument("--kernel", default="mapf_rollout_kernel")
    ap.add_argument("--config", default="c2")
    ap.add_argument("--T", type=int, default=64)
    ap.add_argument("--E", type=int, default=4096)
    ap.add_argument("--tag", required=True, help="stats CSV name: profiles/<tag>_kernel_stats.csv")
    ap.add_argument("--lds", default=None)
    ap.add_argument("--command", default=None)
    ap.add_argument("--sq", default=None, help="a `rocprofv3 --pmc` pass of SQ_COUNTERS")
    ap.add_argument("--bench-json", default=None,
                    help="bench line of the profiled command: exact kernel instance + build id")
    ap.add_argument("--bench-kernel-key", default="kernel",
                    help="dotted key of the kernel name in the bench line (per_step.kernel for the "
                         "per-step leg)")
    ap.add_argument("--match", action="append", default=[],
                    help="key=int stored in the summary (bench.py only uses a profile whose "
                         "keys equal its workload's)")
    a = ap.parse_args()
    out_dir = os.path.dirname(os.path.abspath(a.out))
    os.makedirs(out_dir, exist_ok=True)
    if a.bench_json:
        with open(a.bench_json) as f:
            line = json.loads([x for x in f.read().splitlines() if x.startswith("{")][-1])
        kname = line
        for part in a.bench_kernel_key.split("."):
            kname = (kname or {}).get(part)
        if not kname or not line.get("build_id"):
            raise SystemExit("%s carries no %s / build_id" % (a.bench_json, a.bench_kernel_key))
        a.kernel = kname
    res = {"config": a.config, "T": a.T, "E": a.E, "kernel": a.kernel}
    if a.bench_json:
        res["build_id"] = line["build_id"]
    for kv in a.match:
        k, v = kv.split("=", 1)
        res[k] = int(v)
    if a.command:
        res["command"] = a.command
    if a.trace:
        res["trace"] = trace_stats(a.trace, a.kernel, out_dir, a.tag)
        if not res["trace"].get("kernels"):
            raise SystemExit("no kernel matching %r in %s" % (a.kernel, a.trace))
    fetch = write = None
    if a.fetch:
        fetch, nf = pmc_values(a.fetch, a.kernel, "FETCH_SIZE")
        res["FETCH_SIZE_kb"] = fetch
        res["fetch_dispatches"] = nf
    if a.write:
        write, nw = pmc_values(a.write, a.kernel, "WRITE_SIZE")
        res["WRITE_SIZE_kb"] = write
        res["write_dispatches"] = nw
    if fetch is not None and write is not None:
        res["traffic_bytes_per_launch"] = int((2.0 * fetch + write) * 1024)
        res["traffic_note"] = "(2*FETCH_SIZE + WRITE_SIZE)*1024: gfx950 FETCH_SIZE halving corrected"
    if a.lds:
        res["lds"] = lds_summary(a.lds, a.kernel)
    if a.sq:
        res["sq"] = sq_summary(a.sq, a.kernel)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
