#!/bin/bash
# Round 5, call A: the full GPU suite (new: the driver's T = 20 instance every step vs the
# oracle, back-to-back C3 launches, the partial bench episode, carried-vs-lookup
# distances, unfused runner, world-3 uneven gather), smoke(), the driver's C2 line and a
# C3 kernel trace (dispatch begin / end of the 8 timed launches: the wall < kernel check).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?
tail -3 $O/gpu_tests.txt
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/gpu_tests.txt | head -40; exit 1; fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c2_t20.json 2> $O/bench_c2_t20.err || { tail $O/bench_c2_t20.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c2_t20.json')); print(d['value'], d['kernel_ms_per_launch'], d['kernel'][:80], d['build_id'], d['roofline']['traffic_source'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c3_trace -o run --output-format csv \
  -- python3 bench.py --config c3 --cpu-seconds 0 --per-step-steps 0 > $O/bench_c3_traced.json 2> $O/c3_trace.err || { tail $O/c3_trace.err; exit 1; }
timeout -k 10 300 python3 bench.py --config c3 --cpu-seconds 0 --per-step-steps 0 > $O/bench_c3.json 2> $O/bench_c3.err || { tail $O/bench_c3.err; exit 1; }
python3 - <<'PY'
import csv, glob, json
O = "gpurun_out/r05a"
line = json.load(open(O + "/bench_c3_traced.json"))
name = line["kernel"]
def inst(n):
    i = n.find("<")
    j = n.find("(", i) if i >= 0 else -1
    return n[:j] if j > 0 else n
rows = []
for p in glob.glob(O + "/c3_trace/**/*kernel_trace.csv", recursive=True):
    rows += [r for r in csv.DictReader(open(p)) if inst(r["Kernel_Name"]) == inst(name)]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
s = [int(r["Start_Timestamp"]) for r in rows]
e = [int(r["End_Timestamp"]) for r in rows]
print("c3 dispatches", len(rows), "dur_us", [round((b - a) / 1e3, 1) for a, b in zip(s, e)])
print("c3 gap_us (start[i+1]-end[i])", [round((s[i + 1] - e[i]) / 1e3, 2) for i in range(len(s) - 1)])
print("c3 traced line", line["timing"])
print("c3 plain line", json.load(open(O + "/bench_c3.json"))["timing"])
PY
