#!/bin/bash
# Round 3 closing records: full GPU suite; C5 A/B (this commit vs the previous lib) and
# per-phase stamps; the bench line of every leg (driver command first); the C5 profile
# recipe (trace, FETCH/WRITE, LDS, SQ passes).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03aj
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $OUT/tests.txt 2>&1 || { tail -40 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
for v in "" _prev "" _prev; do
  MAPFX_LIB=$PWD/mapf-marl_amd/mapfx/libmapfx$v.so timeout -k 10 200 python3 bench.py --config c5 --cpu-seconds 0 \
    --per-step-steps 0 --no-gather > $OUT/c5ab$v.json 2> $OUT/c5ab$v.err || { tail -20 $OUT/c5ab$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c5ab$v.json')); print('c5 lib$v', d['kernel_ms_per_launch'], d['timing']['kernel_ms_replays'])"
done
timeout -k 10 200 python3 tools/stamps_c5.py > $OUT/stamps.txt 2>&1 || { tail -20 $OUT/stamps.txt; exit 1; }
cat $OUT/stamps.txt
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
tail -c 400 $OUT/bench_c2.json; echo
for leg in "--config c5" "--env marl_partial" "--env primal" "--env runner" "--config c3" "--config c1"; do
  tag=$(echo $leg | awk '{print $2}')
  timeout -k 10 300 python3 bench.py $leg > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail -20 $OUT/bench_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$tag.json')); print('$tag', d['value'], (d.get('roofline') or {}).get('frac'), d.get('kernel_ms_per_launch'))"
done
bash tools/r03_profile.sh r03aj_c5 --config c5 --gpus 1 --cpu-seconds 0 --per-step-steps 0
