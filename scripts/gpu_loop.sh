#!/bin/bash
# Loopback multi-rank tests (incl. MV / star-tree aggregation merge) + star-tree tests.
set -o pipefail
mkdir -p gpurun_out/loop
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_loopback.py tests/test_gpu_startree.py > gpurun_out/loop/pytest.log 2>&1
rc=$?
tail -25 gpurun_out/loop/pytest.log
exit $rc
