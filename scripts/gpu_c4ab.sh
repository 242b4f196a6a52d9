#!/bin/bash
# GPU-box: group-by parity tests, then config 4 under engine configurations (one JSON line each) and a
# rocprofv3 kernel summary of the default.
# Usage: bash scripts/gpu_c4ab.sh <tag> "<cfg1>" "<cfg2>" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -k "group" --durations=12 --timeout 120 --timeout-method thread > "$OUT/pytest_group.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_group.log"; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -16 "$OUT/pytest_group.log"
i=0
for cfg in "$@"; do
  timeout -k 10 300 python -u scripts/bench_workloads.py --workload config4 --steps 3 --warmup 1 --engine-config "$cfg" > "$OUT/c4_$i.json" 2> "$OUT/c4_$i.err" || { echo "config4 failed: $cfg"; tail -20 "$OUT/c4_$i.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/c4_$i.json')); print(repr(sys.argv[1]), 'c_abi %.2f ms' % d['p50_c_abi_ms'], 'device %.2f' % d['device_ms'], 'match', d['check']['match'])" "$cfg"
  i=$((i+1))
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/c4prof" -o run -- python3 scripts/bench_workloads.py --workload config4 --steps 1 --warmup 1 > "$OUT/c4prof.log" 2>&1 || { echo "config4 rocprof failed"; exit 1; }
python3 scripts/prof_kernels.py "$OUT/c4prof/run_results.db" > "$OUT/c4prof_kernels.txt" && head -12 "$OUT/c4prof_kernels.txt"
if [ -n "$PMC" ]; then  # HBM bytes per group-by kernel (FETCH_SIZE x2 for gfx950 wide reads, MI355X_MICROARCH.md)
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$OUT/c4fetch" -o run -- python3 scripts/bench_workloads.py --workload config4 --steps 1 --warmup 0 > "$OUT/c4fetch.log" 2>&1 || { echo "fetch pmc failed"; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d "$OUT/c4write" -o run -- python3 scripts/bench_workloads.py --workload config4 --steps 1 --warmup 0 > "$OUT/c4write.log" 2>&1 || { echo "write pmc failed"; exit 1; }
  python3 scripts/pmc_summary.py "$OUT/c4fetch/run_results.db" > "$OUT/c4_pmc.txt"
  python3 scripts/pmc_summary.py "$OUT/c4write/run_results.db" >> "$OUT/c4_pmc.txt"
  grep -E "group_query|partition" "$OUT/c4_pmc.txt"
fi
echo done
