#!/bin/bash
set -o pipefail
out=gpurun_out/${1:-r04d}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ring.py tests/test_gpu_configs.py -k "ring or config4 or trim" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
grep -E "passed|failed" $out/pytest.log | tail -1
bash scripts/gpu_c4sdma.sh ${1:-r04d}/sdma || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/probe -o run -- python3 scripts/ring_probe.py --reps 4 --modes 0,4,1 > $out/probe.log 2>&1 || { tail -20 $out/probe.log; exit 1; }
grep debug_ring $out/probe.log | cut -c1-250
python3 scripts/probe_split.py $out/probe/run_results.db 4 0,4,1 | tee $out/probe_split.txt
rm -rf $out/probe
