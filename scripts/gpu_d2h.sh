#!/bin/bash
# Config-4 D2H fan-out A/B: bench.py --workload config4 at 20/5 under d2h.streams settings.
set -o pipefail
OUT=gpurun_out/d2h
mkdir -p $OUT
for s in 1 2 4; do
  timeout -k 10 300 python -u bench.py --workload config4 --steps 20 --warmup 5 --no-cpu-baseline --no-verify \
    --engine-config "d2h.streams=$s" > $OUT/c4_s$s.json 2> $OUT/c4_s$s.err || { echo "bench failed s=$s"; tail -20 $OUT/c4_s$s.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/c4_s$s.json')); print('d2h.streams=$s', 'ms_per_step %.3f' % d['ms_per_step'], 'p50 %.3f' % d['p50_query_ms'], 'c_abi %.3f' % d.get('p50_c_abi_ms', 0))"
done
timeout -k 10 300 python -u bench.py --workload config4 --steps 3 --warmup 1 --no-cpu-baseline --no-verify \
  --engine-config "debug.host_phases=1" > $OUT/c4_phases.json 2> $OUT/c4_phases.err || { echo "phases failed"; exit 1; }
grep -E "outputs|host phases" $OUT/c4_phases.err | tail -6
