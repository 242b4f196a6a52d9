#!/bin/bash
# MV + pruner + segment-dir GPU tests (round 3).
set -o pipefail
mkdir -p gpurun_out/mv
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_mv.py tests/test_gpu_pruner.py tests/test_gpu_segment_dir.py > gpurun_out/mv/pytest.log 2>&1
rc=$?
tail -30 gpurun_out/mv/pytest.log
exit $rc
