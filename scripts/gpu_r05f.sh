#!/bin/bash
# Ring kernel: phase timing (variants/timing.so) + product bench line (ring plan) with kernel trace.
set -o pipefail
out=gpurun_out/${1:-r05f}
mkdir -p $out
export TMPDIR=/tmp
PINOT_GPU_LIB=$PWD/incubator-pinot_amd/pinot_amd/variants/timing.so timeout -k 10 240 python3 bench.py --workload config4 \
  --steps 1 --warmup 0 --no-cpu-baseline --no-verify --engine-config "group.ring=1" > $out/timing.log 2> $out/timing.err \
  || { tail -5 $out/timing.err; exit 1; }
grep "ring-timing block 0 " $out/timing.log | head -12
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py \
    --workload config4 --steps 6 --warmup 2 --no-cpu-baseline --no-verify --engine-config "group.ring=1" \
    > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
python3 scripts/prof_kernels.py $out/prof/run_results.db > $out/kernels.txt 2>&1
rm -f $out/prof/run_results.db
head -4 $out/kernels.txt | cut -c1-70,100-150
python3 scripts/show_bench.py $out/bench.json | head -2
