#!/bin/bash
# Round-4 iteration: parity (ring, LDS, MV across GPUs), the LDS group-by bench, config 4 on the ring and the counted plan.
set -o pipefail
tag=${1:-r04c}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest --maxfail=6 -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ring.py tests/test_gpu_loopback.py \
  tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_ragged.py tests/test_gpu_raw.py tests/test_gpu_mv.py \
  -k "ring or config4 or loopback_mv or group or config1 or ragged or fixed_byte or admission" > $out/pytest.log 2>&1; rc=$?
grep -E "FAILED|Error|passed|failed" $out/pytest.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -40 $out/pytest.log; exit 1; }
timeout -k 10 300 python bench.py --workload lds --steps 20 --warmup 5 --cpu-seconds 5 > $out/bench_lds.json 2> $out/bench_lds.err || { tail -20 $out/bench_lds.err; exit 1; }
python scripts/show_bench.py $out/bench_lds.json | head -6
for cfg in "" "group.ring=0"; do
  name=c4_$(echo "${cfg:-ring}" | tr '=.' '__')
  timeout -k 10 300 python bench.py --workload config4 --steps 10 --warmup 3 --no-cpu-baseline --engine-config "$cfg" > $out/$name.json 2> $out/$name.err || { tail -20 $out/$name.err; exit 1; }
  echo "== $name"; python scripts/show_bench.py $out/$name.json | head -4
done
