#!/bin/bash
# GPU parity run: every -m gpu test, one process, per-test timeout; log under gpurun_out/.
set -o pipefail
out=${1:-gpurun_out/pytest_gpu.log}
shift
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" > "$out" 2>&1
rc=$?
tail -5 "$out"
exit $rc
