#!/bin/bash
# Ring plan (block-synchronous buckets): parity tests, then config 4 under a rocprofv3 kernel trace (ring and counted
# plans) and the ring kernels' SQ counters. Large profiler databases are deleted once summarised (gpurun_out <= 64 MiB).
set -o pipefail
tag=${1:-r05c}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ring.py \
  > $out/pytest_ring.log 2>&1
rc=$?
grep -E "passed|failed" $out/pytest_ring.log | tail -2
[ $rc -le 1 ] || exit $rc
for cfg in "group.ring=1" "group.ring=0"; do
  name=$(echo $cfg | tr '=.;' '___')
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/prof_$name -o run -- python3 bench.py \
    --workload config4 --steps 6 --warmup 2 --no-cpu-baseline --no-verify --engine-config "$cfg" \
    > $out/bench_$name.json 2> $out/bench_$name.err || { echo "$cfg failed"; tail -5 $out/bench_$name.err; exit 1; }
  python3 scripts/prof_kernels.py $out/prof_$name/run_results.db > $out/kernels_$name.txt 2>&1
  rm -f $out/prof_$name/run_results.db
  echo "== $cfg"; head -8 $out/kernels_$name.txt | cut -c1-70,100-150
  python3 scripts/show_bench.py $out/bench_$name.json | head -2
done
i=0
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 150 rocprofv3 --pmc $ctr -d $out/pmc_$i -o run -- python3 bench.py --workload config4 --steps 2 --warmup 1 \
    --no-cpu-baseline --no-verify --engine-config "group.ring=1" > $out/pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $out/pmc_$i.log; exit 1; }
  python3 scripts/pmc_summary.py $out/pmc_$i/run_results.db > $out/pmc_$i.txt
  rm -f $out/pmc_$i/run_results.db
  grep -E "k_group_ring|k_ring_reduce" $out/pmc_$i.txt | cut -c1-40,90-170
  i=$((i+1))
done
