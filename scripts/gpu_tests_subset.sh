#!/bin/bash
# A subset of the GPU tests (files given as arguments), then optional extra command.
# Usage: scripts/gpu_tests_subset.sh <tag> <pytest args...>
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" > $out/pytest.log 2>&1
rc=$?
grep -E "passed|failed|error" $out/pytest.log | tail -5
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" $out/pytest.log | head -40; fi
exit $rc
