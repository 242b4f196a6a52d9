#!/bin/bash
# The GPU test suite in parts (each part well inside one gpurun call): scripts/gpu_suite.sh <tag> <files...>
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 1080 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu "$@" > $out/pytest.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $out/pytest.log | tail -12
exit $rc
