#!/bin/bash
# Driver-settings bench (20 steps / 5 warm-ups) twice, config 2 only: the step-time shape after the warm-ups.
set -o pipefail
out=gpurun_out/gap
mkdir -p $out
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-config4 --no-cpu-baseline --no-verify > $out/b$i.json 2> $out/b$i.err || { tail -20 $out/b$i.err; exit 1; }
  python3 scripts/show_bench.py $out/b$i.json
done
