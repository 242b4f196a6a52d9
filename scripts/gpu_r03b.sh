#!/bin/bash
# Round-3 check: loopback / server / pruner GPU tests, the default bench line (config 2 + embedded config 4), the
# server path at N = 1, and the config-2 step distribution.
set -o pipefail
out=gpurun_out/${1:-r03b}
mkdir -p $out
bash scripts/gpu_tests_subset.sh $(basename $out)_t tests/test_gpu_loopback.py tests/test_gpu_server.py tests/test_gpu_pruner.py || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
python scripts/show_bench.py $out/bench.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --path server --no-cpu-baseline --no-verify > $out/bench_server.json 2> $out/bench_server.err || { tail -30 $out/bench_server.err; exit 1; }
python scripts/show_bench.py $out/bench_server.json
