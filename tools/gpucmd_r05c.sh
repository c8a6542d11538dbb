#!/bin/bash
# Round 5, call C: u8 partial tables (parity + bench), wide-bitmap variant (parity + A/B).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05c
mkdir -p $O
L=mapf-marl_amd/mapfx
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_partial.py tests/test_gpu_partial_full_range.py tests/test_gpu_runner.py -x -q --timeout 300 --timeout-method thread > $O/partial_tests.txt 2>&1
rc=$?; tail -2 $O/partial_tests.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/partial_tests.txt | head -30; exit 1; }
MAPFX_LIB=$PWD/$L/libmapfx_wide.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "runner_rollout_every_step or batched_step_matches or bench_rollout or back_to_back or rollout_equals or full_size or wave_partial" > $O/wide_tests.txt 2>&1
rc=$?; tail -2 $O/wide_tests.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/wide_tests.txt | head -30; exit 1; }
timeout -k 10 300 python3 bench.py --env marl_partial > $O/bench_partial.json 2> $O/bench_partial.err || { tail $O/bench_partial.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_partial.json')); print('partial', d['value'], d['kernel_ms_per_step'], d['roofline']['frac'])"
for r in 1 2; do
  for v in base wide; do
    lib=$PWD/$L/libmapfx.so; [ $v = wide ] && lib=$PWD/$L/libmapfx_wide.so
    MAPFX_LIB=$lib timeout -k 10 200 python3 tools/scale_step.py --envs 64,4096 > $O/scale_${v}_$r.txt 2>&1 || exit 1
    MAPFX_LIB=$lib timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/c2_${v}_$r.json 2> $O/c2_${v}_$r.err || { tail $O/c2_${v}_$r.err; exit 1; }
    MAPFX_LIB=$lib timeout -k 10 300 python3 bench.py --config c3 --cpu-seconds 0 --per-step-steps 50 > $O/c3_${v}_$r.json 2> $O/c3_${v}_$r.err || { tail $O/c3_${v}_$r.err; exit 1; }
    python3 - $v $r <<'PY'
import json, sys
v, r = sys.argv[1:]
O = "gpurun_out/r05c"
c2 = json.load(open("%s/c2_%s_%s.json" % (O, v, r))); c3 = json.load(open("%s/c3_%s_%s.json" % (O, v, r)))
sc = open("%s/scale_%s_%s.txt" % (O, v, r)).read().split()
print(v, r, "| c2 T20 kernel", c2["kernel_ms_per_launch"], "per_step", c2["per_step"]["kernel_ms"],
      "| c3 kernel", c3["kernel_ms_per_launch"], "per_step", c3["per_step"]["kernel_ms"], "| scale", " ".join(x for x in sc if x[0].isdigit() and "." in x))
PY
  done
done
