#!/bin/bash
# Interleaved A/B of libmapfx builds on bench.py's kernel timing (event-timed launches).
# usage: tools/ab_bench.sh OUTDIR ROUNDS "bench args" lib1.so lib2.so ...
# Prints, per lib and round, kernel_ms_per_launch and the replay list.
set -o pipefail
OUT=$1; R=$2; ARGS=$3; shift 3
mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for lib in "$@"; do
    tag=$(basename "$lib" .so)
    MAPFX_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --per-step-steps 0 $ARGS --cpu-seconds 0 \
      > "$OUT/$tag.r$r.json" 2> "$OUT/$tag.r$r.err" || { tail -20 "$OUT/$tag.r$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/$tag.r$r.json')); k=d.get('kernel_ms_per_launch', d.get('kernel_ms_per_step')); print('%-22s r$r %.5f' % ('$tag', k), (d.get('timing') or {}).get('kernel_ms_replays'), d['roofline']['frac'], 'per_step', (d.get('per_step') or {}).get('kernel_ms'))"
  done
done
