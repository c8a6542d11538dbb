set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "runner_rollout_every or full_size or batched_step" > gpurun_out/t_c3.log 2>&1; rc=$?; tail -3 gpurun_out/t_c3.log; [ $rc -eq 0 ] || exit $rc
for v in base nosplit64; do
  if [ $v = base ]; then unset MAPFX_LIB; else export MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx_$v.so; fi
  for i in 1 2; do timeout -k 10 200 python3 bench.py --config c3 --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --per-step-steps 0 > gpurun_out/c3_$v.$i.json 2>/dev/null || exit $?; done
  timeout -k 10 200 python3 bench.py --config c3 --gpus 1 --cpu-seconds 0 --per-step-steps 0 > gpurun_out/c3_${v}_t64.json 2>/dev/null || exit $?
  python3 -c "
import json
for f in ('gpurun_out/c3_$v.1.json','gpurun_out/c3_$v.2.json','gpurun_out/c3_${v}_t64.json'):
    d=json.load(open(f)); print('$v', d['config']['chunk_T'], '%.4g' % d['value'], d['kernel_ms_per_launch'], d['roofline']['frac'])"
done
