#!/bin/bash
set -o pipefail
out=gpurun_out/${1:-r04h}
mkdir -p $out
for cfg in "" "group.lds_block=256"; do
  name=lds_$(echo "${cfg:-512}" | tr '=.' '__')
  timeout -k 10 300 python bench.py --workload lds --steps 20 --warmup 5 --no-cpu-baseline --engine-config "$cfg" > $out/$name.json 2> $out/$name.err || { tail -20 $out/$name.err; exit 1; }
  echo "== $name"; python scripts/show_bench.py $out/$name.json | head -3
done
timeout -k 10 200 python scripts/c4_host.py "" > $out/c4host.log 2> $out/c4host.err || { tail -20 $out/c4host.err; exit 1; }
grep step $out/c4host.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('%2d top %7.2f dev %6.2f dt %5.2f' % (d['step'], d['group_by_top_ms'], d['device_ms'], d['datatable_ms']))
"
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "group_by" > $out/pytest.log 2>&1; grep -E "FAILED|passed|failed" $out/pytest.log | tail -4
