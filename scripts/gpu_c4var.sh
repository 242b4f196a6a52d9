#!/bin/bash
# GPU-box: ring-plan parity tests, then config 4 under engine configurations, each as a rocprofv3 kernel trace
# (k_group_ring / k_ring_reduce averages) plus its C-ABI / device line.
# Usage: bash scripts/gpu_c4var.sh <tag> "<cfg1>" "<cfg2>" ...   (SKIP_TESTS=1: no pytest; PMC=1: + FETCH/WRITE of cfg1)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 800 python -u -m pytest ${TESTS:-tests/test_gpu_ring.py tests/test_gpu_configs.py tests/test_gpu_datatable.py tests/test_gpu_raw.py} -m gpu -x -v --durations=8 --timeout 240 --timeout-method thread > "$OUT/pytest_ring.log" 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" "$OUT/pytest_ring.log" | head -20; tail -30 "$OUT/pytest_ring.log"; exit 1; }
  grep -E "passed|failed" "$OUT/pytest_ring.log" | tail -3
fi
i=0
for cfg in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/p$i" -o run -- python3 scripts/bench_workloads.py --workload config4 --steps ${C4STEPS:-12} --warmup 3 --engine-config "$cfg" > "$OUT/c4_$i.json" 2> "$OUT/c4_$i.err" || { echo "config4 failed: $cfg"; tail -20 "$OUT/c4_$i.err"; exit 1; }
  python3 scripts/prof_kernels.py "$OUT/p$i/run_results.db" > "$OUT/k_$i.txt"
  python3 -c "
import json,sys
d=json.loads(open('$OUT/c4_$i.json').read().strip().splitlines()[-1])
print(repr(sys.argv[1]), 'c_abi %.2f ms' % d['p50_c_abi_ms'], 'device %.2f' % d['device_ms'], 'match', d['check']['match'])
" "$cfg"
  python3 scripts/prof_medians.py "$OUT/p$i/run_results.db" k_group_ring k_ring_reduce k_trim
  rm -f "$OUT/p$i/run_results.db"
  i=$((i+1))
done
if [ -n "$PMC" ]; then  # HBM bytes per kernel (FETCH_SIZE x2 for gfx950 wide reads, MI355X_MICROARCH.md)
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$OUT/c4fetch" -o run -- python3 scripts/bench_workloads.py --workload config4 --steps 1 --warmup 0 --engine-config "$1" > "$OUT/c4fetch.log" 2>&1 || { echo "fetch pmc failed"; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d "$OUT/c4write" -o run -- python3 scripts/bench_workloads.py --workload config4 --steps 1 --warmup 0 --engine-config "$1" > "$OUT/c4write.log" 2>&1 || { echo "write pmc failed"; exit 1; }
  python3 scripts/pmc_summary.py "$OUT/c4fetch/run_results.db" > "$OUT/c4_pmc.txt"
  python3 scripts/pmc_summary.py "$OUT/c4write/run_results.db" >> "$OUT/c4_pmc.txt"
  rm -f "$OUT/c4fetch/run_results.db" "$OUT/c4write/run_results.db"
  grep -E "ring" "$OUT/c4_pmc.txt"
fi
echo done
