#!/bin/bash
# Config-4 timing experiments: per engine configuration, a short bench under rocprofv3 --kernel-trace --stats and
# the top kernels (debug.emit modes give wrong results: timing only, so --no-verify).
set -o pipefail
tag=${1:-emitexp}
out=gpurun_out/$tag
mkdir -p $out
shift
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for cfg in "$@"; do
  name=$(echo "${cfg:-default}" | tr '=,.;' '____')
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/$name -o run -- python bench.py --workload config4 \
    --steps 3 --warmup 1 --no-cpu-baseline --no-verify --engine-config "$cfg" > $out/$name.log 2>&1 \
    || { echo "FAILED $cfg"; tail -5 $out/$name.log; exit 1; }
  echo "== ${cfg:-default}"
  python scripts/prof_kernels.py $out/$name/run_results.db 2>&1 | grep -v "k_synth_column" | sed -n 2,6p | cut -c1-60,100-
done
