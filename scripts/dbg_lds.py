#!/usr/bin/env python3
"""Debug: the random group-by queries of tests/test_gpu_parity.py::test_random_group_by under engine configs, printing
each mismatch (query, config, function, key)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("incubator-pinot_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))
import pinot_oracle as O  # noqa: E402
from pinot_amd import GpuEngine, ServerQueryExecutor  # noqa: E402
from test_gpu_parity import _random_aggs, _random_segment, _random_tree  # noqa: E402

for seed in (1, 5):
    rng = np.random.default_rng(300 + seed)
    n = int(rng.choice([64, 777, 20000]))
    segs = [_random_segment(rng, n, name="s%d" % i) for i in range(int(rng.integers(1, 3)))]
    gpool = ["i0", "i1", "i2", "s", "srt", "i3"]
    qs = []
    for _ in range(5):
        gcols = list(rng.choice(gpool, size=int(rng.integers(1, 3)), replace=False))
        qs.append({"aggregations": _random_aggs(rng), "filter": _random_tree(rng, segs[0]) if rng.random() < 0.7 else None,
                   "group_by": {"columns": gcols, "top_n": 10}})
    print("seed", seed, "segments", len(segs), [s_.num_docs for s_ in segs], flush=True)
    extra = []
    for q in qs:
        q2 = dict(q)
        q2["filter"] = None
        extra.append(q2)
    qs = qs + extra
    for cfg in ("", "group.lw=1"):
        e = GpuEngine(0, cfg or None)
        gsegs = [e.register(s) for s in segs]
        ex = ServerQueryExecutor(e)
        for qi, q in enumerate(qs):
            got, st = ex.process_query(q, gsegs, trim=False)
            exp, scanned = O.execute_server(segs, q)
            bad = []
            if set(got) != set(exp):
                bad.append("keys: got-exp %s exp-got %s" % (sorted(set(got) - set(exp))[:5], sorted(set(exp) - set(got))[:5]))
            else:
                for key in exp:
                    for a, gv, ev in zip(q["aggregations"], got[key], exp[key]):
                        f = a["function"].upper()
                        if f == "DISTINCTCOUNTHLL":
                            if gv.cardinality() != ev.cardinality():
                                bad.append("%s(%s) key %r card %s vs %s" % (f, a["column"], key, gv.cardinality(), ev.cardinality()))
                        elif f == "AVG":
                            s, c = (ev.sum, ev.count) if hasattr(ev, "sum") else ev
                            if gv.count != c or abs(gv.sum - s) > 1e-6 * max(1, abs(s)):
                                bad.append("AVG(%s) key %r %s/%s vs %s/%s" % (a["column"], key, gv.sum, gv.count, s, c))
                        elif abs(gv - ev) > 1e-6 * max(1, abs(ev)):
                            bad.append("%s(%s) key %r %s vs %s" % (f, a["column"], key, gv, ev))
            print("seed %d n %d cfg %-18s q%d filt %s gcols %s aggs %s: %s" % (
                seed, n, cfg or "default", qi, q["filter"] is not None, q["group_by"]["columns"],
                [(a["function"], a["column"]) for a in q["aggregations"]], "OK" if not bad else "%d bad, e.g. %s" % (len(bad), bad[:3])),
                flush=True)
        e.close()
