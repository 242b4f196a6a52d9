#!/bin/bash
# GPU-box A/B of engine configurations on the config-2 bench (no CPU baseline), one JSON line each.
# Usage: bash scripts/gpu_ab.sh <tag> "<cfg1>" "<cfg2>" ...   (cfg "" = defaults)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
i=0
for cfg in "$@"; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --warmup 5 --engine-config "$cfg" > "$OUT/ab_$i.json" 2> "$OUT/ab_$i.err" || { echo "bench failed: $cfg"; tail -20 "$OUT/ab_$i.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/ab_$i.json')); print(repr(sys.argv[1]), 'ms/query %.4f' % d['ms_per_step'], 'kernel', {k: round(v['avg_ms'],4) for k,v in d['roofline']['kernels'].items()}, 'frac %.3f' % d['roofline']['frac'])" "$cfg"
  i=$((i+1))
done
