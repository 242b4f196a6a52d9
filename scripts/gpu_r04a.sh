#!/bin/bash
# Round-4 iteration: GB_LDS on the lane-owns-quarter path (parity + LDS bench), MV across GPUs, and the config-4 ring
# plan's time split (debug.ring modes under rocprofv3) + its SQ / TCC counters.
set -o pipefail
tag=${1:-r04a}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest --maxfail=6 -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ring.py tests/test_gpu_loopback.py \
  tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_ragged.py tests/test_gpu_raw.py \
  -k "ring or config4 or loopback_mv or group or config1 or ragged or fixed_byte" > $out/pytest.log 2>&1; rc=$?
grep -E "FAILED|Error|passed|failed" $out/pytest.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -40 $out/pytest.log; exit 1; }
timeout -k 10 300 python bench.py --workload lds --steps 20 --warmup 5 --cpu-seconds 5 > $out/bench_lds.json 2> $out/bench_lds.err || { tail -20 $out/bench_lds.err; exit 1; }
python scripts/show_bench.py $out/bench_lds.json 2>/dev/null | head -20 || tail -1 $out/bench_lds.json | cut -c1-1200
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/probe -o run -- python3 scripts/ring_probe.py --reps 4 > $out/probe.log 2>&1 || { tail -20 $out/probe.log; exit 1; }
grep debug_ring $out/probe.log
python3 scripts/prof_kernels.py $out/probe/run_results.db > $out/probe_kernels.txt 2>&1; head -12 $out/probe_kernels.txt
python3 scripts/probe_split.py $out/probe/run_results.db 4 | tee $out/probe_split.txt
rm -rf $out/probe
for pass in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
            "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_BRANCH" \
            "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_ATOMIC_sum TCC_EA0_WRREQ_64B_sum"; do
  name=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-include-regex "k_group_ring|k_ring_reduce|k_group_query" -d $out/pmc_$name -o run -- \
    python3 scripts/ring_probe.py --reps 2 --modes 0 > $out/pmc_$name.log 2>&1 || { echo "pmc pass $name failed"; tail -5 $out/pmc_$name.log; break; }
  python3 scripts/pmc_summary.py $out/pmc_$name/run_results.db > $out/pmc_$name.txt 2>&1
  rm -rf $out/pmc_$name
done
cat $out/pmc_*.txt | cut -c1-170
ls $out
