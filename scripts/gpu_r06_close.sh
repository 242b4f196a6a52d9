#!/bin/bash
# Round-6 closing measurements on the final sources, each step under its own time limit:
#   1. PMC traffic (FETCH_SIZE / WRITE_SIZE passes) of the config-2, config-4 and LDS kernels -> profiles/traffic_*.json
#      stamped with the HEAD kernel-source hash (bench.py reports roofline.traffic only while the hash matches)
#   2. SQ counter passes (at most 8 SQ counters each) of the same three workloads
#   3. the default bench line (driver shape 20 / 5) and its rocprofv3 kernel trace + the config-2 window
# Usage: scripts/gpu_r06_close.sh <tag> [steps: pmc,sq,bench]
set -o pipefail
tag=${1:-r06close}
steps=${2:-pmc,sq,bench}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
if [[ $steps == *pmc* ]]; then
  bash scripts/gpu_pmc.sh $tag config2 config4 lds || exit 1
fi
if [[ $steps == *sq* ]]; then
  P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS"
  P2="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_BRANCH"
  for wl in config2 config4 lds; do
    i=1
    for ctr in "$P1" "$P2"; do
      timeout -s KILL 150 rocprofv3 --pmc $ctr -d $out/sq_${wl}_$i -o run -- python3 bench.py --workload $wl --steps 3 --warmup 1 \
        --no-config4 --no-lds --no-cpu-baseline --no-verify > $out/sq_${wl}_$i.log 2>&1 || { echo "sq pass $wl $i failed"; tail -5 $out/sq_${wl}_$i.log; exit 1; }
      python3 scripts/pmc_summary.py $out/sq_${wl}_$i/run_results.db > $out/sq_${wl}_$i.txt
      rm -f $out/sq_${wl}_$i/run_results.db
      i=$((i+1))
    done
  done
  grep -hE "k_group_ring|k_ring_reduce|k_group_query<1|k_scan_query<" $out/sq_*_*.txt | grep -E "BANK_CONFLICT|IDX_ACTIVE|WAIT_ANY|WAVE_CYCLES" | cut -c1-170 | head -20
fi
if [[ $steps == *bench* ]]; then
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/bench_default.json 2> $out/bench_default.err || { tail -20 $out/bench_default.err; exit 1; }
  python scripts/show_bench.py $out/bench_default.json | head -24
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
  python3 scripts/prof_kernels.py $out/prof/run_results.db > $out/kernels_default.txt; head -14 $out/kernels_default.txt
  python3 scripts/prof_window.py $out/prof/run_results.db k_scan_query 5 20 | tee $out/config2_window.json
  python3 scripts/prof_medians.py $out/prof/run_results.db k_scan_query k_group_ring k_ring_reduce "k_group_query<1" > $out/kernel_medians.txt; cat $out/kernel_medians.txt
  find $out -name "*.db" -delete
fi
