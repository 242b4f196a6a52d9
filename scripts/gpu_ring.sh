#!/bin/bash
# Ring-plan iteration: its GPU parity tests + config-4 shapes + this round's other GPU tests, then the config-4 bench
# line and a rocprofv3 summary.
set -o pipefail
tag=${1:-ring}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest --maxfail=6 -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ring.py \
  tests/test_gpu_configs.py tests/test_gpu_raw.py tests/test_gpu_segment_dir.py tests/test_gpu_startree.py tests/test_gpu_loopback.py tests/test_gpu_mv.py tests/test_gpu_parity.py \
  -k "fixed_byte or ring or config4 or trim or fixture or cache or hll or HLL or limit or admission or loopback_mv or deep_filter or wide_bitmap" > $out/pytest.log 2>&1; rc=$?
grep -E "FAILED|Error" $out/pytest.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -40 $out/pytest.log; exit 1; }  # 1 = test failures (bench still runs)
grep -E "passed|failed" $out/pytest.log | tail -2
timeout -k 10 300 python bench.py --workload config4 --steps 10 --warmup 3 --cpu-seconds 5 > $out/bench_config4.json 2> $out/bench_config4.err || { tail -20 $out/bench_config4.err; exit 1; }
tail -1 $out/bench_config4.json | cut -c1-2500
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python bench.py --workload config4 --steps 5 --warmup 2 --no-cpu-baseline > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
python scripts/prof_kernels.py $out/prof/run_results.db > $out/kernels.txt 2>&1; head -24 $out/kernels.txt
timeout -k 10 300 python bench.py --workload lds --steps 20 --warmup 5 --cpu-seconds 5 > $out/bench_lds.json 2> $out/bench_lds.err || { tail -20 $out/bench_lds.err; exit 1; }
tail -1 $out/bench_lds.json | cut -c1-1500
