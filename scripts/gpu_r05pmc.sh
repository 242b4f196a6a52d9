#!/bin/bash
# Round-5 counters: SQ passes (one rocprofv3 --pmc run each, at most 8 SQ counters) over bench.py's config-4 and LDS
# workloads, then the FETCH_SIZE / WRITE_SIZE traffic passes (scripts/gpu_pmc.sh). Usage: scripts/gpu_r05pmc.sh <tag>
set -o pipefail
tag=${1:-r05pmc}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS"
P2="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_BRANCH"
for wl in config4 lds; do
  i=1
  for ctr in "$P1" "$P2"; do
    timeout -s KILL 150 rocprofv3 --pmc $ctr -d $out/sq_${wl}_$i -o run -- python3 bench.py --workload $wl --steps 3 --warmup 1 \
      --no-config4 --no-lds --no-cpu-baseline --no-verify > $out/sq_${wl}_$i.log 2>&1 || { echo "pass $wl $i failed"; tail -5 $out/sq_${wl}_$i.log; exit 1; }
    python3 scripts/pmc_summary.py $out/sq_${wl}_$i/run_results.db > $out/sq_${wl}_$i.txt
    rm -f $out/sq_${wl}_$i/run_results.db
    i=$((i+1))
  done
  grep -E "k_group_ring|k_ring_reduce|k_group_query" $out/sq_${wl}_*.txt | cut -c1-200 | head -40
done
bash scripts/gpu_pmc.sh $tag config4 lds
