#!/usr/bin/env python3
"""Config-4 host time split per step (engine path, the server's DataTable answer): prune, group_by_top (C-ABI, device
time inside), the trimmed lists, the native DataTable writer, the bytes copy, result free."""
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
from pinot_amd._lib import check  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else ""
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
e = GpuEngine(0, cfg or None)
segs = [e.register_synthetic("fact_%d" % s, 125_000_000, bench.COLUMNS, bench.BASE_SEED + s) for s in range(8)]
e.synchronize()
ex = ServerQueryExecutor(e, num_groups_limit=1_000_000)
q = ex.prepare(bench.CONFIG4)
import gc  # noqa: E402
gc.collect()
gc.disable()
lib = e.lib
for i in range(steps):
    t0 = time.perf_counter()
    kept, total, handles = ex._prune(q.marshal, segs)
    t1 = time.perf_counter()
    res, st = ex.group_by_result(q, kept, top_n=10)
    t2 = time.perf_counter()
    lists = [res.trimmed_groups(10, f) for f in range(3)]
    t3 = time.perf_counter()
    groups = (C.c_void_p * 3)(*[k.ctypes.data_as(C.c_void_p) for k in lists])
    nums = (C.c_int64 * 3)(*[k.shape[0] for k in lists])
    data, size = C.c_void_p(), C.c_uint64()
    check(lib.pinot_datatable_group_by(C.byref(q.marshal.q), res.ptr, groups, nums, C.byref(st), None, C.byref(data),
                                       C.byref(size)))
    t4 = time.perf_counter()
    dt = C.string_at(data, size.value)
    t5 = time.perf_counter()
    del res
    t6 = time.perf_counter()
    print(json.dumps({"step": i, "prune_ms": (t1 - t0) * 1e3, "group_by_top_ms": (t2 - t1) * 1e3,
                      "abi_host_ms": st.host_ms, "device_ms": st.device_ms, "trim_lists_ms": (t3 - t2) * 1e3,
                      "datatable_ms": (t4 - t3) * 1e3, "bytes_copy_ms": (t5 - t4) * 1e3, "free_ms": (t6 - t5) * 1e3,
                      "step_ms": (t6 - t0) * 1e3, "bytes": len(dt)}), flush=True)
e.close()
