#!/usr/bin/env python3
"""Config-4 host time split per step (engine path): prune, group_by_top (C-ABI), DataTable, result free."""
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "incubator-pinot_amd"))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from pinot_amd import GpuEngine, ServerQueryExecutor, _lib  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else ""
e = GpuEngine(0, cfg or None)
segs = [e.register_synthetic("fact_%d" % s, 125_000_000, bench.COLUMNS, bench.BASE_SEED + s) for s in range(8)]
e.synchronize()
ex = ServerQueryExecutor(e, num_groups_limit=1_000_000)
q = ex.prepare(bench.CONFIG4)
import gc  # noqa: E402
gc.disable()
for i in range(10):
    t0 = time.perf_counter()
    kept, total, handles = ex._prune(q.marshal, segs)
    t1 = time.perf_counter()
    res, st = ex.group_by_result(q, kept, top_n=10)
    t2 = time.perf_counter()
    ta = time.perf_counter()
    kept = [res.trimmed_groups(10, i) for i in range(3)]
    tb = time.perf_counter()
    regs = res.hll(2)
    tc = time.perf_counter()
    keys = res.raw_keys()
    td = time.perf_counter()
    dt = res.data_table(q.marshal, st, 10, None)
    t3 = time.perf_counter()
    print(json.dumps({"trim_lists_ms": (tb - ta) * 1e3, "hll_fetch_ms": (tc - tb) * 1e3, "raw_keys_ms": (td - tc) * 1e3}))
    del res
    t4 = time.perf_counter()
    print(json.dumps({"step": i, "prune_ms": (t1 - t0) * 1e3, "group_by_top_ms": (t2 - t1) * 1e3,
                      "abi_host_ms": st.host_ms, "device_ms": st.device_ms, "datatable_ms": (t3 - t2) * 1e3,
                      "free_ms": (t4 - t3) * 1e3, "bytes": len(dt)}), flush=True)
e.close()
