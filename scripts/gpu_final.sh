#!/bin/bash
# Round-end validation at HEAD: the full -m gpu suite, smoke(), the config-2 and config-4 bench lines with their
# rocprofv3 kernel summaries, then the FETCH/WRITE PMC passes that write profiles/traffic_<workload>.json for these
# exact kernel sources, and the config-2 line again (now reporting the measured traffic).
# Usage: scripts/gpu_final.sh <tag>   (outputs under gpurun_out/<tag>/)
set -o pipefail
tag=${1:-final}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
# the whole suite without -x: a failing test is reported, and the measurements below still run
# (SKIP_TESTS=1: measurements only, when the suite ran in an earlier call)
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1
test_rc=$?
case $test_rc in 124|134|137|139) tail -30 $out/pytest_gpu.log; exit 1;; esac  # timeout / abort / fault: stop
grep -E "^FAILED|^ERROR" $out/pytest_gpu.log | head -20
tail -1 $out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
fi
timeout -k 10 300 python bench.py --workload config4 --steps 20 --warmup 5 --engine-config "debug.host_phases=1" > $out/bench_config4.json 2> $out/bench_config4.err || exit 1
grep "host phases\|outputs (us)" $out/bench_config4.err | tail -3 > $out/config4_host_phases.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_c4 -o run -- python3 bench.py --workload config4 --steps 5 --warmup 2 --no-cpu-baseline > $out/prof_c4.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_c2 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify > $out/prof_c2.log 2>&1 || exit 1
python3 scripts/prof_kernels.py $out/prof_c4/run_results.db > $out/config4_rocprof_kernels.txt 2>&1
python3 scripts/prof_kernels.py $out/prof_c2/run_results.db > $out/config2_rocprof_kernels.txt 2>&1
bash scripts/gpu_pmc.sh $tag config2 config4 || exit 1
timeout -k 10 300 python bench.py > $out/bench_config2.json 2> $out/bench_config2.err || exit 1
tail -1 $out/bench_config2.json | cut -c1-400
tail -1 $out/bench_config4.json | cut -c1-400
