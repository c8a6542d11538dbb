#!/bin/bash
# Round 4 end: profiles of the headline (C2, the driver's command) and MARL_PARTIAL
# (trace + FETCH / WRITE + LDS + SQ passes), and the diagnostic stamps.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
bash tools/r03_profile.sh r04_c2 --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 0 || exit 1
python3 tools/pmc_traffic.py --trace $O/r04_c2/trace --fetch $O/r04_c2/pmc_fetch --write $O/r04_c2/pmc_write \
  --lds $O/r04_c2/pmc_lds --sq $O/r04_c2/pmc_sq --kernel "mapf_wave_kernel" --config c2 --T 20 --E 4096 \
  --tag r04_c2 --command "python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 0" \
  --out $O/profiles/pmc_c2.json > /dev/null || exit 1
bash tools/r03_profile.sh r04_partial --env marl_partial --cpu-seconds 0 || exit 1
python3 tools/pmc_traffic.py --trace $O/r04_partial/trace --fetch $O/r04_partial/pmc_fetch --write $O/r04_partial/pmc_write \
  --lds $O/r04_partial/pmc_lds --sq $O/r04_partial/pmc_sq --kernel "partial_kernel" --config marl_partial --T 1 --E 4096 \
  --match N=15 --match S=8 --tag r04_partial --command "python3 bench.py --env marl_partial --cpu-seconds 0" \
  --out $O/profiles/pmc_partial.json > /dev/null || exit 1
python3 -c "
import json
for f in ('pmc_c2', 'pmc_partial'):
    d = json.load(open('$O/profiles/%s.json' % f))
    print(f, d['trace']['kernels'][0]['avg_ns'], d.get('traffic_bytes_per_launch'), (d.get('sq') or {}).get('wait_any_frac_of_wave_cycles'))
"
timeout -k 10 120 python3 tools/stamps.py > $O/profiles/r04_c2_stamps.txt 2>&1 && cat $O/profiles/r04_c2_stamps.txt || exit 1
timeout -k 10 120 python3 tools/pstamps_partial.py > $O/profiles/r04_pstamps_partial.txt 2>&1 || exit 1
timeout -k 10 120 python3 tools/pstamps_step.py > $O/profiles/r04_pstamps_step.txt 2>&1 || exit 1
