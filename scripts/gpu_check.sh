#!/bin/bash
# GPU-box validation: parity suite, smoke, bench line, rocprofv3 kernel stats (+ optional PMC passes).
# Usage (from the repo root, on the GPU box via gpurun): bash scripts/gpu_check.sh [tag] [pmc]
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== host"; (nproc; lscpu | grep -E 'Model name|^CPU\(s\)'; java -version 2>&1 | head -1) > "$OUT/host.txt" 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -30 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || { echo "rocprof failed"; tail -30 "$OUT/prof.log"; exit 1; }
if [ "$2" = "pmc" ]; then
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch.log" 2>&1 || { echo "pmc fetch failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write.log" 2>&1 || { echo "pmc write failed"; exit 1; }
fi
echo done
