#!/bin/bash
set -o pipefail
out=gpurun_out/${1:-r04g}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_datatable.py > $out/pytest.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" $out/pytest.log | tail -4
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 200 python scripts/c4_host.py "" > $out/c4host.log 2> $out/c4host.err || { tail -20 $out/c4host.err; exit 1; }
python3 -c "
import json
for l in open('$out/c4host.log'):
    d=json.loads(l); print('%2d top %7.2f dev %6.2f dt %5.2f free %5.2f' % (d['step'], d['group_by_top_ms'], d['device_ms'], d['datatable_ms'], d['free_ms']))
"
