#!/bin/bash
# Streaming scan kernel check: width sweep + config-2 parity tests, then config-2 bench lines per engine configuration.
set -o pipefail
out=gpurun_out/${1:-r03d}
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py \
  -k "width_sweep or config2" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
for cfg in "" "exec.stream=0" "exec.stream=0;exec.nt=1"; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-config4 --no-cpu-baseline --no-verify --engine-config "$cfg" \
    > $out/bench_$(echo "${cfg:-default}" | tr '=;.' '___').json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
  echo "== ${cfg:-default}"; python scripts/show_bench.py $out/bench_$(echo "${cfg:-default}" | tr '=;.' '___').json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 20 --warmup 5 \
  --no-config4 --no-cpu-baseline --no-verify > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
python3 scripts/prof_kernels.py $out/prof/run_results.db | head -6
