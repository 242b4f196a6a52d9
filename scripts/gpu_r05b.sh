#!/bin/bash
# Ring-plan diagnosis: parity tests of the product build, then config 4 on each variant library (PINOT_GPU_LIB) under
# a rocprofv3 kernel trace, then SQ counters of the product ring kernels.
set -o pipefail
tag=${1:-r05b}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ring.py \
  > $out/pytest_ring.log 2>&1
rc=$?
grep -E "passed|failed" $out/pytest_ring.log | tail -2
[ $rc -le 1 ] || exit $rc
for v in product $(ls incubator-pinot_amd/pinot_amd/variants/ 2>/dev/null | sed 's/\.so$//'); do
  lib=""
  [ "$v" != product ] && lib=$PWD/incubator-pinot_amd/pinot_amd/variants/$v.so
  PINOT_GPU_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/prof_$v -o run -- python3 bench.py \
    --workload config4 --steps 4 --warmup 2 --no-cpu-baseline --no-verify --engine-config "group.ring=1" \
    > $out/bench_$v.json 2> $out/bench_$v.err || { echo "variant $v failed"; tail -5 $out/bench_$v.err; exit 1; }
  python3 scripts/prof_kernels.py $out/prof_$v/run_results.db > $out/kernels_$v.txt 2>&1
  echo "== $v"; grep -E "k_group_ring|k_ring_reduce" $out/kernels_$v.txt | cut -c1-60,100-140
done
i=0
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 150 rocprofv3 --pmc $ctr -d $out/pmc_$i -o run -- python3 bench.py --workload config4 --steps 2 --warmup 1 \
    --no-cpu-baseline --no-verify --engine-config "group.ring=1" > $out/pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $out/pmc_$i.log; exit 1; }
  python3 scripts/pmc_summary.py $out/pmc_$i/run_results.db > $out/pmc_$i.txt
  grep -E "k_group_ring|k_ring_reduce" $out/pmc_$i.txt | cut -c1-40,90-170
  i=$((i+1))
done
