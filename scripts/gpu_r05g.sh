#!/bin/bash
# Ring kernel: product and experiment variants (PINOT_GPU_LIB) under a rocprofv3 kernel trace.
set -o pipefail
out=gpurun_out/${1:-r05g}
mkdir -p $out
export TMPDIR=/tmp
for v in product $(ls incubator-pinot_amd/pinot_amd/variants/ 2>/dev/null | sed 's/\.so$//'); do
  lib=""
  [ "$v" != product ] && lib=$PWD/incubator-pinot_amd/pinot_amd/variants/$v.so
  PINOT_GPU_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/prof_$v -o run -- python3 bench.py \
    --workload config4 --steps 4 --warmup 1 --no-cpu-baseline --no-verify --engine-config "group.ring=1" \
    > $out/bench_$v.json 2> $out/bench_$v.err || { echo "variant $v failed"; tail -5 $out/bench_$v.err; exit 1; }
  python3 scripts/prof_kernels.py $out/prof_$v/run_results.db > $out/kernels_$v.txt 2>&1
  [ "$v" = product ] && python3 scripts/prof_timeline.py $out/prof_$v/run_results.db > $out/timeline_$v.txt 2>&1
  rm -f $out/prof_$v/run_results.db
  echo "== $v"; grep -E "k_group_ring|k_ring_reduce" $out/kernels_$v.txt | cut -c1-60,100-140
done
if [ -n "$C4HOST" ]; then
  PINOT_DATATABLE_PHASES=1 timeout -k 10 240 python3 scripts/c4_host.py "debug.host_phases=1" 8 > $out/c4host.log 2> $out/c4host.err || { tail -5 $out/c4host.err; exit 1; }
  tail -3 $out/c4host.log; grep "host phases\|outputs\|datatable phases" $out/c4host.err | tail -6
fi
