#!/bin/bash
# Config-4 iteration: group-by parity subset, then the config-4 bench line and its rocprofv3 kernel summary.
set -o pipefail
tag=${1:-c4}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_configs.py -k "config4 or trim" tests/test_gpu_parity.py -k "sinks or partitioned or config4 or trim" \
  > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 300 python bench.py --workload config4 --steps 10 --warmup 3 --cpu-seconds 5 > $out/bench_config4.json 2> $out/bench_config4.err || exit $?
tail -1 $out/bench_config4.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python bench.py --workload config4 --steps 5 --warmup 2 --no-cpu-baseline > $out/prof.log 2>&1 || exit $?
python scripts/prof_kernels.py $out/prof/run_results.db > $out/kernels.txt 2>&1; head -24 $out/kernels.txt
