#!/bin/bash
# Ring kernel phase timing (experiment build variants/timing.so, RING_EXP_TIMING): per-wave shader-clock totals.
set -o pipefail
out=gpurun_out/${1:-r05e}
mkdir -p $out
PINOT_GPU_LIB=$PWD/incubator-pinot_amd/pinot_amd/variants/timing.so timeout -k 10 240 python3 bench.py --workload config4 \
  --steps 1 --warmup 0 --no-cpu-baseline --no-verify --engine-config "group.ring=1" > $out/timing.log 2> $out/timing.err \
  || { tail -5 $out/timing.err; exit 1; }
grep "ring-timing" $out/timing.log | head -30
