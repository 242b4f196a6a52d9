#!/bin/bash
# One GPU session: bench lines (config 2 + config 4) and the rocprofv3 kernel summaries of the same commands.
# Usage: scripts/gpu_bench.sh <tag>   (outputs under gpurun_out/<tag>/)
set -o pipefail
tag=${1:-bench}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python bench.py > $out/bench_config2.json 2> $out/bench_config2.err || exit $?
tail -1 $out/bench_config2.json
timeout -k 10 300 python bench.py --workload config4 --steps 10 --warmup 3 > $out/bench_config4.json 2> $out/bench_config4.err || exit $?
tail -1 $out/bench_config4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_c4 -o run -- python bench.py --workload config4 --steps 5 --warmup 2 --no-cpu-baseline > $out/prof_c4.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_c2 -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-verify > $out/prof_c2.log 2>&1 || exit $?
python scripts/prof_kernels.py $out/prof_c4/run_results.db; python scripts/prof_kernels.py $out/prof_c2/run_results.db
