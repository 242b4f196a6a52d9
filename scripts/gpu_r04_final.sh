#!/bin/bash
# Round-4 final measurement: the default bench line (config 2 + embedded config 4 + LDS group-by, CPU baselines), rocprofv3
# kernel summaries, the config-2 kernel durations inside the timed window, PMC traffic and SQ counters.
set -o pipefail
tag=${1:-r04final}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 150 python -u -m pytest -v --timeout 100 --timeout-method thread -m gpu tests/test_gpu_datatable.py > $out/pytest_dt.log 2>&1 || { tail -30 $out/pytest_dt.log; exit 1; }
tail -1 $out/pytest_dt.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/bench_default.json 2> $out/bench_default.err || { tail -20 $out/bench_default.err; exit 1; }
python scripts/show_bench.py $out/bench_default.json | head -20
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
python3 scripts/prof_kernels.py $out/prof/run_results.db > $out/kernels_default.txt; head -16 $out/kernels_default.txt
python3 scripts/prof_window.py $out/prof/run_results.db k_scan_query 5 20 | tee $out/config2_window.json
rm -rf $out/prof
bash scripts/gpu_pmc.sh $tag/pmc config2 config4 lds || exit 1
for wl in config4 lds; do
  for pass in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
              "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVES" "TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum"; do
    name=$(echo $pass | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-include-regex "k_group_query|k_partition|k_group_ring|k_ring_reduce" -d $out/sq_${wl}_$name -o run -- \
      python3 bench.py --workload $wl --steps 2 --warmup 1 --no-cpu-baseline > $out/sq_${wl}_$name.log 2>&1 || { echo "pmc $wl $name failed"; tail -5 $out/sq_${wl}_$name.log; break; }
    python3 scripts/pmc_summary.py $out/sq_${wl}_$name/run_results.db > $out/sq_${wl}_$name.txt 2>&1
    rm -rf $out/sq_${wl}_$name
  done
done
find $out -name "*.db" -delete
ls -R $out | head -50
timeout -k 10 200 python scripts/c4_host.py "" > $out/c4host.log 2> $out/c4host.err || { tail -20 $out/c4host.err; exit 1; }
grep step $out/c4host.log | cut -c1-200 | tail -5
