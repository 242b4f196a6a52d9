#!/bin/bash
# GPU-box: PMC passes over config 4's group-by kernels (one counter group per run).
# Usage: bash scripts/gpu_c4pmc.sh <tag> "<counters pass 1>" "<counters pass 2>" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for ctr in "$@"; do
  timeout -s KILL 200 rocprofv3 --pmc $ctr -d "$OUT/pmc_$i" -o run -- python3 scripts/bench_workloads.py --workload config4 --steps 1 --warmup 0 > "$OUT/pmc_$i.log" 2>&1 || { echo "pmc pass failed: $ctr"; tail -5 "$OUT/pmc_$i.log"; exit 1; }
  python3 scripts/pmc_summary.py "$OUT/pmc_$i/run_results.db" > "$OUT/pmc_$i.txt"
  grep -E "group_query|partition" "$OUT/pmc_$i.txt"
  i=$((i+1))
done
echo done
