#!/bin/bash
# Round-5 closing measurement after the last kernel change: the default
# bench line (config 2 + the embedded config-4 and LDS lines) and its rocprof summary.
set -o pipefail
tag=${1:-r05final}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/bench_default.json 2> $out/bench_default.err || { tail -20 $out/bench_default.err; exit 1; }
python scripts/show_bench.py $out/bench_default.json | head -20
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
python3 scripts/prof_kernels.py $out/prof/run_results.db > $out/kernels_default.txt; head -12 $out/kernels_default.txt
python3 scripts/prof_window.py $out/prof/run_results.db k_scan_query 5 20 | tee $out/config2_window.json
find $out -name "*.db" -delete
