#!/bin/bash
# Compact group-by read-back: group-by parity tests (incl. config-4 shapes, 1M-group export), then config 4 A/B.
set -o pipefail
OUT=gpurun_out/compact
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py \
  tests/test_gpu_parity.py -k "group or config4 or 1m" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for c in 0 1; do
  timeout -k 10 300 python -u bench.py --workload config4 --steps 20 --warmup 5 --no-cpu-baseline --no-verify \
    --engine-config "d2h.compact=$c" > $OUT/c4_c$c.json 2> $OUT/c4_c$c.err || { echo "bench failed c=$c"; tail -20 $OUT/c4_c$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c4_c$c.json')); print('d2h.compact=$c', 'ms_per_step %.3f' % d['ms_per_step'], 'p50 %.3f' % d['p50_query_ms'])"
done
timeout -k 10 300 python -u bench.py --workload config4 --steps 3 --warmup 1 --no-cpu-baseline \
  --engine-config "debug.host_phases=1" > $OUT/c4_phases.json 2> $OUT/c4_phases.err || { echo "phases failed"; tail -20 $OUT/c4_phases.err; exit 1; }
grep -E "outputs" $OUT/c4_phases.err | tail -3
python3 -c "import json; d=json.load(open('$OUT/c4_phases.json')); print('verify', d.get('verify', d.get('check')))"
