#!/bin/bash
# Round-5 ring plan (decoder + flusher waves, quarter-form filter): its parity tests, then config 4 on the ring plan
# and on the counted plan, with a rocprofv3 kernel summary of the ring run.
set -o pipefail
tag=${1:-r05a}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ring.py \
  tests/test_gpu_configs.py -k "ring or lds_shape or compact or diagnostic or trim or config4_shape" \
  > $out/pytest_ring.log 2>&1
rc=$?
tail -3 $out/pytest_ring.log
[ $rc -le 1 ] || exit $rc   # 0 pass / 1 test failure: go on measuring; anything else (fault, timeout): stop
timeout -k 10 300 python bench.py --workload config4 --steps 10 --warmup 3 --no-cpu-baseline \
  --engine-config "group.ring=1" > $out/c4_ring.json 2> $out/c4_ring.err || exit $?
python scripts/show_bench.py $out/c4_ring.json 2>/dev/null | head -20
timeout -k 10 300 python bench.py --workload config4 --steps 10 --warmup 3 --no-cpu-baseline \
  > $out/c4_counted.json 2> $out/c4_counted.err || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python bench.py --workload config4 --steps 5 \
  --warmup 2 --no-cpu-baseline --engine-config "group.ring=1" > $out/prof.log 2>&1 || exit $?
python scripts/prof_kernels.py $out/prof/run_results.db > $out/kernels.txt 2>&1; head -24 $out/kernels.txt
