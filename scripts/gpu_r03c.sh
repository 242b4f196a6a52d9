#!/bin/bash
# Round-3 baseline at HEAD: the whole -m gpu suite, smoke(), the default bench line at the driver's settings, its
# rocprofv3 kernel summary, and one PMC pass of LDS / atomic counters over config 4's group-by kernels.
# Usage: scripts/gpu_r03c.sh <tag>   (outputs under gpurun_out/<tag>/)
set -o pipefail
tag=${1:-r03c}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1
test_rc=$?
case $test_rc in 124|134|137|139) tail -30 $out/pytest_gpu.log; exit 1;; esac
grep -E "^FAILED|^ERROR" $out/pytest_gpu.log | head -20
tail -1 $out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
python scripts/show_bench.py $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 20 --warmup 5 \
  --no-cpu-baseline --no-verify > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
python3 scripts/prof_kernels.py $out/prof/run_results.db > $out/rocprof_kernels.txt 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_EA0_ATOMIC_sum -d $out/pmc_lds -o run \
  -- python3 bench.py --workload config4 --steps 2 --warmup 1 --no-cpu-baseline --no-verify > $out/pmc_lds.log 2>&1 \
  || { tail -20 $out/pmc_lds.log; exit 1; }
python3 scripts/pmc_summary.py $out/pmc_lds/run_results.db > $out/pmc_lds_atomics.txt
grep -E "group_query|partition|scan_query" $out/pmc_lds_atomics.txt
echo done
