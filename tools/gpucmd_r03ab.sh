#!/bin/bash
# Round 3: measurement recipe of the PRIMAL leg with primal_seq_kernel (pmc_primal.json).
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_primal.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r03ab_primal_tests.txt 2>&1 || { tail -40 gpurun_out/r03ab_primal_tests.txt; exit 1; }
tail -1 gpurun_out/r03ab_primal_tests.txt
bash tools/r03_profile.sh r03_primal --env primal --cpu-seconds 0 || exit $?
timeout -k 10 200 python3 bench.py --env primal > gpurun_out/r03_primal/bench_cpu.json 2> gpurun_out/r03_primal/bench_cpu.err || exit 1
tail -c 400 gpurun_out/r03_primal/bench_cpu.json
