#!/bin/bash
# The driver's default bench invocation and smoke() at HEAD.
set -o pipefail
out=gpurun_out/final_bench
mkdir -p $out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
python scripts/show_bench.py $out/bench.json
