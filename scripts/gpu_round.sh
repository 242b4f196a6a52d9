#!/bin/bash
# Whole-round GPU validation: the full -m gpu suite, smoke(), then scripts/gpu_bench.sh (config-2 and config-4
# bench lines + rocprofv3 kernel summaries). Usage: scripts/gpu_round.sh <tag>   (outputs under gpurun_out/<tag>/)
set -o pipefail
tag=${1:-round}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
bash scripts/gpu_bench.sh $tag
