#!/usr/bin/env python3
"""Config-4 ring-plan probe (timing experiments, run under rocprofv3 --kernel-trace): the full-size config-4 group-by
on the engine with each debug.ring mode in turn, R queries per mode, in this order:

    0 production  |  4 instrumented (wait counters)  |  1 decode only  |  2 sink without HBM stores  |  3 claims only

Modes 1-3 give wrong results (timing only). Prints one JSON line per mode: the engine's HIP-event time of the timed
group-by region (filter + ring + reduce) per query and the ring-sink wait counters; the per-kernel split comes from
the rocprof database (k_group_ring<0> launches are mode 0; k_group_ring<1> launches are modes 4, 1, 2, 3 in order)."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "incubator-pinot_amd"))
sys.path.insert(0, REPO)

import bench  # noqa: E402  (COLUMNS, CONFIG4, BASE_SEED)
from pinot_amd import GpuEngine, ServerQueryExecutor  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=4)
ap.add_argument("--segments", type=int, default=8)
ap.add_argument("--docs", type=int, default=125_000_000)
ap.add_argument("--modes", default="0,4,1,2,3")
ap.add_argument("--query", default=bench.CONFIG4)
args = ap.parse_args()

e = GpuEngine(0)
segs = [e.register_synthetic("fact_%d" % s, args.docs, bench.COLUMNS, bench.BASE_SEED + s) for s in range(args.segments)]
e.synchronize()
ex = ServerQueryExecutor(e, num_groups_limit=1_000_000)
q = ex.prepare(args.query)
for mode in [int(m) for m in args.modes.split(",")]:
    e.set_config("debug.ring=%d;timing=1" % mode)
    w0, s0 = e.stat("group.ring_waits"), e.stat("group.ring_sleeps")
    ms = []
    t0 = time.time()
    for _ in range(args.reps):
        res, st = ex.group_by_result(q, segs)
        ms.append(e.last_kernel_ms(1)[0])
        del res
    print(json.dumps({"debug_ring": mode, "region_ms": ms, "wall_s": time.time() - t0,
                      "ring_queries": e.stat("group.ring_queries"), "fallbacks": e.stat("group.ring_fallbacks"),
                      "waits_per_query": (e.stat("group.ring_waits") - w0) / args.reps,
                      "sleeps_per_query": (e.stat("group.ring_sleeps") - s0) / args.reps}), flush=True)
e.set_config("debug.ring=0;timing=0")
e.close()
