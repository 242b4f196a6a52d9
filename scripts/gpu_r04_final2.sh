#!/bin/bash
# Round-4 closing measurement after the last kernel change: PMC traffic for config 4 and the LDS group-by, the default
# bench line and its rocprof summary.
set -o pipefail
tag=${1:-r04final2}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
bash scripts/gpu_pmc.sh $tag/pmc config4 lds || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/bench_default.json 2> $out/bench_default.err || { tail -20 $out/bench_default.err; exit 1; }
python scripts/show_bench.py $out/bench_default.json | head -20
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
python3 scripts/prof_kernels.py $out/prof/run_results.db > $out/kernels_default.txt; head -12 $out/kernels_default.txt
python3 scripts/prof_window.py $out/prof/run_results.db k_scan_query 5 20 | tee $out/config2_window.json
find $out -name "*.db" -delete
