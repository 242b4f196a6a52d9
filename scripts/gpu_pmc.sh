#!/bin/bash
# HBM traffic of the bench kernels: separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per workload, then
# scripts/pmc_traffic.py writes profiles/traffic_<workload>.json (copied back under gpurun_out/<tag>/).
# Usage: scripts/gpu_pmc.sh <tag> [workload ...]   (default: config2 config4)
set -o pipefail
tag=${1:-pmc}; shift
wls=${*:-config2 config4}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for wl in $wls; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c -d $out/pmc_${wl}_$c -o run -- python3 bench.py --workload $wl --steps 3 --warmup 1 --no-config4 --no-lds \
      --no-cpu-baseline --no-verify > $out/pmc_${wl}_$c.log 2>&1 || { tail -20 $out/pmc_${wl}_$c.log; exit 1; }
  done
  python3 scripts/pmc_traffic.py $wl $out/pmc_${wl}_FETCH_SIZE/run_results.db $out/pmc_${wl}_WRITE_SIZE/run_results.db \
    > $out/traffic_$wl.log 2>&1 || { cat $out/traffic_$wl.log; exit 1; }
  cp profiles/traffic_$wl.json $out/
  python3 scripts/pmc_summary.py $out/pmc_${wl}_FETCH_SIZE/run_results.db > $out/pmc_${wl}_summary.txt
  python3 scripts/pmc_summary.py $out/pmc_${wl}_WRITE_SIZE/run_results.db >> $out/pmc_${wl}_summary.txt
  rm -f $out/pmc_${wl}_FETCH_SIZE/run_results.db $out/pmc_${wl}_WRITE_SIZE/run_results.db
  cat $out/traffic_$wl.log
done
