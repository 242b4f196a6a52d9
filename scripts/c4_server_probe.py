#!/usr/bin/env python3
"""Where a config-4 server-path step goes (N = 1): the C-ABI group-by call (pinot_gpu_server_group_by_top), the
per-function kept lists and the DataTable writer, each timed over several steps, beside the engine path's."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "incubator-pinot_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

from bench import BASE_SEED, COLUMNS, CONFIG4  # noqa: E402
from pinot_amd import GpuServer, ServerExecutor, ServerQueryExecutor  # noqa: E402
from pinot_amd import _lib  # noqa: E402

docs = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000_000
srv = GpuServer([0], "")
eng = srv.engines[0]
segs = [eng.register_synthetic("fact_%d" % s, docs, COLUMNS, BASE_SEED + s) for s in range(8)]
eng.synchronize()
for name, ex in (("server", ServerExecutor(srv, num_groups_limit=1_000_000)),
                 ("engine", ServerQueryExecutor(eng, num_groups_limit=1_000_000))):
    q = ex.prepare(CONFIG4)
    t = {"call": [], "kept": [], "datatable": [], "free": [], "step": []}
    for it in range(12):
        t0 = time.perf_counter()
        if name == "server":
            res, stats, m = ex._group_by(q, segs, 10)
        else:
            res, st = ex.group_by_result(q, segs, top_n=10)
            m, stats = q.marshal, _lib.ExecStats()
        t1 = time.perf_counter()
        kept = [res.trimmed_groups(10, i) for i in range(3)]
        t2 = time.perf_counter()
        dt = res.data_table(m, stats, 10, None, True)
        t3 = time.perf_counter()
        n = len(dt)
        del dt, res
        t4 = time.perf_counter()
        for k, v in (("call", t1 - t0), ("kept", t2 - t1), ("datatable", t3 - t2), ("free", t4 - t3), ("step", t4 - t0)):
            t[k].append(v * 1e3)
    print(name, "groups kept", [len(k) for k in kept], "datatable bytes", n,
          {k: round(float(np.median(v[2:])), 3) for k, v in t.items()}, flush=True)
srv.close()
