#!/bin/bash
# A/B of engine configurations on the config-2 (or --workload) bench line; optional pytest args first via PYTEST="...".
# Usage: scripts/gpu_ab.sh <tag> <cfg> [<cfg> ...]   ("" = default engine configuration)
set -o pipefail
out=gpurun_out/$1; shift
mkdir -p $out
if [ -n "$PYTEST" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $PYTEST > $out/pytest.log 2>&1 \
    || { tail -30 $out/pytest.log; exit 1; }
  tail -2 $out/pytest.log
fi
i=0
for cfg in "$@"; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-config4 --no-cpu-baseline --no-verify ${BENCH_ARGS} \
    --engine-config "$cfg" > $out/bench_$i.json 2> $out/bench_$i.err || { tail -20 $out/bench_$i.err; exit 1; }
  echo "== ${cfg:-default}"; python scripts/show_bench.py $out/bench_$i.json
  i=$((i+1))
done
