#!/bin/bash
set -o pipefail
out=gpurun_out/${1:-c4host}
mkdir -p $out
for cfg in "group.ring=0;debug.host_phases=1" "group.ring=1"; do
  name=$(echo "$cfg" | tr '=.;' '___')
  timeout -k 10 200 python scripts/c4_host.py "$cfg" > $out/$name.log 2> $out/$name.err || { tail -20 $out/$name.err; exit 1; }
  echo "== $cfg"; cat $out/$name.log | cut -c1-250; grep "C-ABI\|key space\|host phases" $out/$name.err | tail -6
done
