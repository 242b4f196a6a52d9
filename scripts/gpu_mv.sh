#!/bin/bash
# Round-3 widening tests on the GPU: MV columns, raw STRING, exact filter stats, pruners, segment dirs.
set -o pipefail
mkdir -p gpurun_out/mv
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_stats.py tests/test_gpu_mv.py tests/test_gpu_raw.py tests/test_gpu_pruner.py \
  tests/test_gpu_segment_dir.py > gpurun_out/mv/pytest.log 2>&1
rc=$?
tail -40 gpurun_out/mv/pytest.log
exit $rc
