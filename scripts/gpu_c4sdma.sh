#!/bin/bash
set -o pipefail
out=gpurun_out/${1:-c4sdma}
mkdir -p $out
timeout -k 10 200 python scripts/c4_host.py "group.ring=0" > $out/sdma_on.log 2> $out/sdma_on.err || { tail -20 $out/sdma_on.err; exit 1; }
HSA_ENABLE_SDMA=0 timeout -k 10 200 python scripts/c4_host.py "group.ring=0" > $out/sdma_off.log 2> $out/sdma_off.err || { tail -20 $out/sdma_off.err; exit 1; }
for f in sdma_on sdma_off; do echo "== $f"; python3 -c "
import json,sys
for l in open('$out/$f.log'):
    d=json.loads(l); print('%2d top %7.2f dev %6.2f dt %5.2f free %5.2f' % (d['step'], d['group_by_top_ms'], d['device_ms'], d['datatable_ms'], d['free_ms']))
"; done
