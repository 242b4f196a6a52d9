#!/bin/bash
# Config-4 host phases (debug.host_phases=1) on the counted and the ring plan, 6 steps each.
set -o pipefail
out=gpurun_out/${1:-c4ph}
mkdir -p $out
for cfg in "group.ring=0" "group.ring=1"; do
  name=$(echo "$cfg" | tr '=.' '__')
  timeout -k 10 300 python bench.py --workload config4 --steps 6 --warmup 2 --no-cpu-baseline --engine-config "$cfg;debug.host_phases=1" > $out/$name.json 2> $out/$name.err || { tail -20 $out/$name.err; exit 1; }
  echo "== $cfg"; python scripts/show_bench.py $out/$name.json | head -3; grep pinot_gpu $out/$name.err | tail -12
done
