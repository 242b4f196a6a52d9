#!/usr/bin/env python3
"""Debug: GB_LDS lane-owns-quarter path vs group.lw=1 on hand-made segments (aggregated DOUBLE / INT columns)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("incubator-pinot_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))
import pinot_oracle as O  # noqa: E402
from pinot_amd import GpuEngine, ServerQueryExecutor, build_segment  # noqa: E402

rng = np.random.default_rng(5)
for n in (64, 5000):
    for dtype in ("DOUBLE", "INT", "LONG", "FLOAT"):
        vals = np.round(rng.normal(0, 1000, size=n), 3) if dtype in ("DOUBLE", "FLOAT") else rng.integers(-50000, 50000, n)
        if dtype == "FLOAT":
            vals = np.float32(vals).astype(np.float64)
        words = ["a", "bb", "ccc", "P", "t", "zz", "Hello", "we"]
        seg = build_segment("d", {"g": ("INT", rng.integers(0, 5, n).tolist()),
                                  "s": ("STRING", [words[i] for i in rng.integers(0, 8, n)]),
                                  "x": (dtype, vals.tolist()),
                                  "y": ("INT", rng.integers(0, 100, n).tolist())})
        for gcol in ("g", "s"):
            for fn in ("SUM", "MAX", "DISTINCTCOUNTHLL"):
                q = {"aggregations": [{"function": fn, "column": "x"}], "filter": None,
                     "group_by": {"columns": [gcol], "top_n": 10}}
                exp, _ = O.execute_server([seg], q)
                out = []
                for cfg in ("", "group.lw=1"):
                    e = GpuEngine(0, cfg or None)
                    g = e.register(seg)
                    got, _ = ServerQueryExecutor(e).process_query(q, [g], trim=False)
                    bad = 0
                    for k in exp:
                        gv, ev = got[k][0], exp[k][0]
                        if fn == "DISTINCTCOUNTHLL":
                            bad += gv.cardinality() != ev.cardinality()
                        else:
                            bad += abs(gv - ev) > 1e-6 * max(1, abs(ev))
                    out.append("%s:%d/%d" % (cfg or "default", bad, len(exp)))
                    e.close()
                print("n %5d %-7s gcol %s %-16s bits x %s : %s" % (n, dtype, gcol, fn, seg.column("x").bits, "  ".join(out)),
                      flush=True)
