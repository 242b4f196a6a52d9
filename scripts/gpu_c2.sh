#!/bin/bash
# Config-2 iteration: the bench line, host phase breakdown, sync-poll variant, rocprofv3 kernel summary.
set -o pipefail
tag=${1:-c2}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "kat or random_aggregations or empty_result or fused" > $out/pytest.log 2>&1 || { tail -20 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python bench.py --cpu-seconds 5 > $out/bench_config2.json 2> $out/bench_config2.err || exit $?
tail -1 $out/bench_config2.json
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-verify --engine-config "debug.host_phases=1" > $out/phases.json 2> $out/phases.err || exit $?
grep "host phases" $out/phases.err | tail -4
for cfg in "plan.cache=1" "plan.cache=0" "sync.flag=0"; do
  name=$(echo "$cfg" | tr '=,.;' '____')
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-verify --engine-config "$cfg" > $out/$name.json 2> $out/$name.err || exit $?
  python -c "import json; d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]); print('$cfg', d['ms_per_step'], d['p50_query_ms'], d['p50_c_abi_ms'], d['roofline']['kernels']['k_scan_query']['avg_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-verify > $out/prof.log 2>&1 || exit $?
python scripts/prof_kernels.py $out/prof/run_results.db > $out/kernels.txt 2>&1; head -8 $out/kernels.txt
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $out/pmc_lds -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify > $out/pmc_lds.log 2>&1 || exit $?
python scripts/pmc_summary.py $out/pmc_lds/run_results.db > $out/pmc_lds.txt 2>&1; grep k_scan_query $out/pmc_lds.txt
