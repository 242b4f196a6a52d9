#!/bin/bash
# GPU-box: configs 3 and 4 (scripts/bench_workloads.py) + rocprofv3 kernel stats of config 4 + a PMC pass
# for the group-by's LDS bank conflicts / LDS instructions / memory-side atomics.
# Usage (from the repo root, on the GPU box via gpurun): bash scripts/gpu_workloads.sh [tag]
set -o pipefail
TAG=${1:-r01w}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/bench_workloads.py --workload config4 --steps 5 --warmup 1 > "$OUT/config4.json" 2> "$OUT/config4.err" || { echo "config4 failed"; tail -20 "$OUT/config4.err"; exit 1; }
cat "$OUT/config4.json"
timeout -k 10 400 python -u scripts/bench_workloads.py --workload config3 --steps 10 --warmup 2 > "$OUT/config3.json" 2> "$OUT/config3.err" || { echo "config3 failed"; tail -20 "$OUT/config3.err"; exit 1; }
cat "$OUT/config3.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/c4prof" -o run -- python3 scripts/bench_workloads.py --workload config4 --steps 1 --warmup 1 > "$OUT/c4prof.log" 2>&1 || { echo "config4 rocprof failed"; exit 1; }
python3 scripts/prof_kernels.py "$OUT/c4prof/run_results.db"
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS TCC_EA0_ATOMIC_sum -d "$OUT/c4pmc" -o run -- python3 scripts/bench_workloads.py --workload config4 --steps 1 --warmup 0 > "$OUT/c4pmc.log" 2>&1 || { echo "config4 pmc failed"; tail -5 "$OUT/c4pmc.log"; exit 1; }
echo done
