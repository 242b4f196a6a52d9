#!/bin/bash
# Same-box A/B of engine configurations on one workload: bench.py lines (kernel avg from HIP events, p50 query).
# Usage: scripts/gpu_cfgs.sh <tag> <workload> "<cfg 1>" "<cfg 2>" ...
set -o pipefail
tag=$1; wl=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
for rep in 1 2; do
for cfg in "$@"; do
  name=$(echo "${cfg:-default}" | tr '=,.;' '____')_$rep
  timeout -k 10 300 python bench.py --workload $wl --steps 30 --warmup 5 --no-cpu-baseline --no-verify --engine-config "$cfg" > $out/$name.json 2> $out/$name.err || { echo "FAILED $cfg"; tail -5 $out/$name.err; exit 1; }
  python -c "import json; d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels']; print('%-40s ms/step %.4f p50 %.4f kernel %s' % ('${cfg:-default}', d['ms_per_step'], d['p50_query_ms'], {n: round(v['avg_ms'], 4) for n, v in k.items()}))"
done
done
