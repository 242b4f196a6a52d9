#!/usr/bin/env python3
"""Per-mode kernel durations of a ring_probe.py run (rocprofv3 --kernel-trace database): probe_split.py <db> <reps>
[<modes>]. k_group_ring<0> = mode 0; k_group_ring<1> = the other modes in order; every mode runs one GB_FILTER,
one ring and one reduce per query."""
import json
import sqlite3
import sys

db, reps = sys.argv[1], int(sys.argv[2])
modes = [int(m) for m in (sys.argv[3] if len(sys.argv) > 3 else "0,4,1,2,3").split(",")]
c = sqlite3.connect(db)
rows = [(n, (e - s) / 1e6) for n, s, e in c.execute("select name, start, end from kernels order by start")]
ring = {0: [d for n, d in rows if "k_group_ring<0>" in n]}
r1 = [d for n, d in rows if "k_group_ring<1>" in n]
red = [d for n, d in rows if "k_ring_reduce" in n]
flt = [d for n, d in rows if "k_group_query<7" in n]
others = [m for m in modes if m != 0]
for i, m in enumerate(others):
    ring[m] = r1[i * reps:(i + 1) * reps]
for i, m in enumerate(modes):
    r = ring.get(m, [])
    print(json.dumps({"debug_ring": m, "ring_ms": [round(x, 4) for x in r],
                      "reduce_ms": [round(x, 4) for x in red[i * reps:(i + 1) * reps]],
                      "filter_ms": [round(x, 4) for x in flt[i * reps:(i + 1) * reps]]}))
