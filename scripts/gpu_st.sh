#!/bin/bash
# Star-tree GPU tests + ragged-segment and loopback regression subset.
set -o pipefail
mkdir -p gpurun_out/st
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_ragged.py > gpurun_out/st/pytest.log 2>&1
rc=$?
tail -30 gpurun_out/st/pytest.log
exit $rc
