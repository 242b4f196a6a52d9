#!/bin/bash
set -o pipefail
out=gpurun_out/${1:-r04f}
mkdir -p $out
timeout -k 10 600 python -u -m pytest --maxfail=5 -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_ragged.py tests/test_gpu_configs.py tests/test_gpu_datatable.py -k "group or ragged or config1 or config4 or datatable or broker or trim" > $out/pytest.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" $out/pytest.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python bench.py --workload config4 --steps 10 --warmup 3 --no-cpu-baseline > $out/c4.json 2> $out/c4.err || { tail -20 $out/c4.err; exit 1; }
python scripts/show_bench.py $out/c4.json | head -3
timeout -k 10 300 python bench.py --workload lds --steps 20 --warmup 5 --no-cpu-baseline > $out/lds.json 2> $out/lds.err || { tail -20 $out/lds.err; exit 1; }
python scripts/show_bench.py $out/lds.json | head -3
