#!/bin/bash
# Round 6, call D: where a runner step's time goes after the fused compaction -- a
# rocprofv3 kernel trace of bench.py --env runner (per-kernel mean duration and the
# idle gaps between kernels) and the host-side probe of one runner step.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv \
  -- python3 bench.py --env runner --steps 300 --warmup 100 --cpu-seconds 0 > $O/bench_traced.json 2> $O/trace.err || { tail $O/trace.err; exit 1; }
python3 tools/trace_gaps.py $O/trace --tail 2000 > $O/gaps.txt
cat $O/gaps.txt
timeout -k 10 300 python3 tools/runner_host_probe.py > $O/host_probe.txt 2>&1 || { tail $O/host_probe.txt; exit 1; }
cat $O/host_probe.txt
