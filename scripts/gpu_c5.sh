#!/bin/bash
# GPU-box: group-by parity tests, config 4 and config 5 (distributed partials + RCCL all-reduce, world 1).
# Usage: bash scripts/gpu_c5.sh <tag> [prof|-] [nopytest]
set -o pipefail
TAG=${1:-r01c5}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
[ "$3" = "nopytest" ] || timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "group or distributed" > "$OUT/pytest_group.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_group.log"; exit 1; }
[ "$3" = "nopytest" ] || tail -2 "$OUT/pytest_group.log"
timeout -k 10 300 python -u scripts/bench_workloads.py --workload config4 --steps 5 --warmup 2 > "$OUT/config4.json" 2> "$OUT/config4.err" || { echo "config4 failed"; tail -20 "$OUT/config4.err"; exit 1; }
cat "$OUT/config4.json"
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 scripts/bench_workloads.py --workload config5 --steps 5 --warmup 2 > "$OUT/config5.json" 2> "$OUT/config5.err" || { echo "config5 failed"; tail -20 "$OUT/config5.err"; exit 1; }
cat "$OUT/config5.json"
echo done
if [ "$2" = "prof" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/c4prof" -o run -- python3 scripts/bench_workloads.py --workload config4 --steps 2 --warmup 1 > "$OUT/c4prof.log" 2>&1 || { echo "config4 rocprof failed"; exit 1; }
  python3 scripts/prof_kernels.py "$OUT/c4prof/run_results.db" > "$OUT/config4_rocprof_kernels.txt"
  head -20 "$OUT/config4_rocprof_kernels.txt"
fi
