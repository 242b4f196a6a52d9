#!/bin/bash
# Config-2 step-time distribution at the driver's settings (20 steps, 5 warm-ups), repeated, plus host phases.
set -o pipefail
tag=${1:-c2dist}
out=gpurun_out/$tag
mkdir -p $out
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify > $out/b20_$i.json 2> $out/b20_$i.err || exit $?
  python -c "import json; d=json.loads(open('$out/b20_$i.json').read().strip().splitlines()[-1]); print('20/5', d['ms_per_step'], d['p50_query_ms'], d['p50_c_abi_ms'], d['roofline']['kernels']['k_scan_query']['avg_ms'], d['step_ms_detail'])"
done
timeout -k 10 300 python bench.py --steps 200 --warmup 50 --no-cpu-baseline --no-verify > $out/b200.json 2> $out/b200.err || exit $?
python -c "import json; d=json.loads(open('$out/b200.json').read().strip().splitlines()[-1]); print('200/50', d['ms_per_step'], d['p50_query_ms'], d['p50_c_abi_ms'], d['roofline']['kernels']['k_scan_query']['avg_ms'], d['step_ms_detail'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify --engine-config "debug.host_phases=1" > $out/phases.json 2> $out/phases.err || exit $?
grep "host phases" $out/phases.err | tail -22
