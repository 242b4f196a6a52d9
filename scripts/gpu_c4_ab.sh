#!/bin/bash
# A/B of the in-tree library against a variant on the config-4 line (tests on the in-tree library first).
# Usage: scripts/gpu_c4_ab.sh <tag> <variant .so> [pytest files...]
set -o pipefail
tag=$1; var=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -q --timeout 240 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
grep -E "passed|failed" $out/tests.log | tail -1
for r in 1 2; do
  for v in tree var; do
    if [ $v = var ]; then export PINOT_GPU_LIB=$var; else unset PINOT_GPU_LIB; fi
    timeout -k 10 200 python bench.py --workload config4 --steps 20 --warmup 5 --no-lds --no-cpu-baseline --no-verify > $out/c4_${v}_$r.json 2> $out/c4_${v}_$r.err || { tail -20 $out/c4_${v}_$r.err; exit 1; }
    echo "$v $r $(python3 scripts/show_bench.py $out/c4_${v}_$r.json | head -1)"
  done
done
