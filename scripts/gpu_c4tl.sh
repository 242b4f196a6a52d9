#!/bin/bash
# Config 4: one rocprofv3 kernel + memory-copy trace of the default plan, and its last query's timeline.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/c4tl
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $out/prof -o run -- python3 bench.py \
  --workload config4 --steps 3 --warmup 2 --no-cpu-baseline --no-verify > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
python3 scripts/prof_timeline.py $out/prof/run_results.db > $out/timeline.txt 2>&1
cat $out/timeline.txt | tail -40
