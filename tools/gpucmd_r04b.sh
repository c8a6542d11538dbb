#!/bin/bash
# Round 4: profiles of what had none: C3's rollout and the per-step
# drop-in kernel (mapf_wave_kernel<5, false, ...>): trace + FETCH / WRITE + LDS + SQ passes
# of the bench command each line is taken with, summarised into profiles/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O/r04b
# generic rollouts with the two-deep action prefetch (MAPFX_GEN_CARRY): parity, then C5 A/B
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "generic or full_size or rollout or autoreset or invalid" > $O/r04b/tests.txt 2>&1 \
  || { grep -E "FAIL|Error" $O/r04b/tests.txt | head -30; tail -30 $O/r04b/tests.txt; exit 1; }
tail -1 $O/r04b/tests.txt
bash tools/ab_bench.sh $O/r04b/ab_c5 2 "--config c5 --gpus 1" mapf-marl_amd/mapfx/libmapfx.so \
  mapf-marl_amd/mapfx/libmapfx_nocarry.so || exit 1
bash tools/r03_profile.sh r04b_c3 --config c3 --gpus 1 --cpu-seconds 0 --per-step-steps 0 || exit 1
bash tools/r03_profile.sh r04b_step --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 200 || exit 1
python3 tools/pmc_traffic.py --trace $O/r04b_c3/trace --fetch $O/r04b_c3/pmc_fetch --write $O/r04b_c3/pmc_write \
  --lds $O/r04b_c3/pmc_lds --sq $O/r04b_c3/pmc_sq --kernel "mapf_wave_kernel<5, true" --config c3 --T 64 --E 2048 \
  --tag r04_c3 --command "python3 bench.py --config c3 --gpus 1 --cpu-seconds 0 --per-step-steps 0" \
  --out $O/profiles/pmc_c3.json > /dev/null || exit 1
python3 tools/pmc_traffic.py --trace $O/r04b_step/trace --fetch $O/r04b_step/pmc_fetch --write $O/r04b_step/pmc_write \
  --lds $O/r04b_step/pmc_lds --sq $O/r04b_step/pmc_sq --kernel "mapf_wave_kernel<5, false" --config c2_step --T 1 --E 4096 \
  --tag r04_c2_step --command "python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 200" \
  --out $O/profiles/pmc_c2_step.json > /dev/null || exit 1
python3 -c "
import json
for f in ('pmc_c3', 'pmc_c2_step'):
    d = json.load(open('$O/profiles/%s.json' % f))
    print(f, d['trace']['kernels'][0]['avg_ns'], d.get('traffic_bytes_per_launch'), (d.get('sq') or {}).get('wait_any_frac_of_wave_cycles'))
"
# the runner's per-step kernels (where its ~66 us per step go)
mkdir -p $O/r04b_runner
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r04b_runner/trace -o run --output-format csv \
  -- python3 bench.py --env runner --cpu-seconds 0 --steps 200 --warmup 100 > $O/r04b_runner/bench.json 2> $O/r04b_runner/err.txt || exit 1
tail -c 300 $O/r04b_runner/bench.json; echo
# MARL_PARTIAL per-phase stamps (diagnostic build)
timeout -k 10 120 python3 tools/pstamps_partial.py > $O/r04b_pstamps.txt 2>&1 && cat $O/r04b_pstamps.txt
# C2 split kernel, block-0 per-segment stamps (diagnostic build) at T = 64
timeout -k 10 120 python3 tools/stamps.py > $O/r04b_c2_stamps.txt 2>&1 && cat $O/r04b_c2_stamps.txt
