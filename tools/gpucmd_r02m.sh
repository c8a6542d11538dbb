#!/bin/bash
# round-2 call m: the driver's bench command profiled (C2, final kernel), per_step sweep legs.
set -o pipefail
export TMPDIR=/tmp
bash tools/r02_profile.sh r02m_c2 --gpus 1 --steps 20 --warmup 5 || exit $?
for i in 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02m_c2/bench_rep$i.json 2>/dev/null || exit $?
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 512 --warmup 64 --cpu-seconds 0 > gpurun_out/r02m_c2/bench_t64.json 2>/dev/null || exit $?
for c in c1 c3; do
  timeout -k 10 300 python3 bench.py --config $c --gpus 1 --steps 20 --warmup 5 --cpu-seconds 5 > gpurun_out/r02m_c2/bench_$c.json 2>/dev/null || exit $?
done
timeout -k 10 300 python3 bench.py --env runner --steps 500 --warmup 100 > gpurun_out/r02m_c2/bench_runner.json 2>/dev/null || exit $?
timeout -k 10 300 python3 bench.py --env marl_partial --steps 500 --warmup 100 > gpurun_out/r02m_c2/bench_partial.json 2>/dev/null || exit $?
echo done
