"""Aggregation-only queries over segments of very different sizes and dictionaries, on the fused and the unfused
(exec.fused=0: per-segment filter + fold / gather launches, then a fixed-order reduce of the block partials) plans.
Regression: the reduce of a small segment once read the block partials a larger segment's launch had left beyond
its own grid (SUM / COUNT over LONG columns taking the gather route came out wrong for mixed-size segments)."""
import numpy as np
import pytest

import pinot_oracle as O
from pinot_amd import GpuEngine, ServerQueryExecutor, build_segment

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = GpuEngine(0)
    yield e
    e.close()


def _segment(rng, n, name):
    cols = {"a": ("INT", rng.integers(0, 4, n).astype(np.int32)),
            "m": ("INT", rng.integers(-500, 1000, n).astype(np.int32)),
            "x": ("LONG", rng.integers(0, 1 << 30, n).astype(np.int64)),
            "d": ("DOUBLE", rng.integers(-1 << 20, 1 << 20, n).astype(np.float64) / 8.0),
            "h": ("INT", rng.integers(0, 5000, n).astype(np.int32))}
    return build_segment(name, cols, allow_sorted=False)


@pytest.mark.parametrize("fused", ["1", "0"])
def test_ragged_segments(engine, fused):
    rng = np.random.default_rng(2100)
    sizes = [20000, 2000, 50, 70000, 1, 4097]
    segs = [_segment(rng, n, "rg%d" % i) for i, n in enumerate(sizes)]
    gs = [engine.register(s) for s in segs]
    engine.set_config("exec.fused=" + fused)
    try:
        ex = ServerQueryExecutor(engine)
        for order in (list(range(len(segs))), list(reversed(range(len(segs))))):
            ss, gg = [segs[i] for i in order], [gs[i] for i in order]
            for flt in (None, {"operator": "EQUALITY", "column": "a", "values": ["1"]},
                        {"operator": "RANGE", "column": "m", "values": ["[0\t\t500)"]}):
                q = {"aggregations": [{"function": "SUM", "column": "x"}, {"function": "COUNT", "column": "*"},
                                      {"function": "AVG", "column": "m"}, {"function": "MAX", "column": "x"},
                                      {"function": "SUM", "column": "d"}, {"function": "MIN", "column": "d"},
                                      {"function": "DISTINCTCOUNTHLL", "column": "h"}],
                     "filter": flt, "group_by": None}
                got, st = ex.process_query(q, gg)
                exp, scanned = O.execute_server(ss, q)
                assert got[0] == exp[0] and got[1] == exp[1] and got[3] == exp[3] and got[4] == exp[4], (flt, got, exp)
                assert (got[2].sum, got[2].count) == exp[2] and got[5] == exp[5], (flt, got, exp)
                assert got[6].cardinality() == exp[6].cardinality()
                assert st.num_docs_scanned == scanned
    finally:
        engine.set_config("exec.fused=1")
        for g in gs:
            g.release()


def _same_value(f, g, e):
    if f == "AVG":
        assert (g.sum, g.count) == tuple(e)
    elif f == "DISTINCTCOUNTHLL":
        assert g.cardinality() == e.cardinality()
    else:
        assert g == e


@pytest.mark.parametrize("cfg", ["", "exec.fused=0", "group.mode=lds", "group.mode=global", "group.mode=partition",
                                 "group.mode=partition;group.ring=0"])
def test_ragged_segments_group_by(engine, cfg):
    """Group-by over the same ragged segments (per-segment dictionaries -> the union key space and remaps), every
    sink; group columns INT / STRING, aggregations over INT / LONG / DOUBLE."""
    rng = np.random.default_rng(2200)
    sizes = [20000, 2000, 50, 70000, 1, 4097]
    segs = []
    for i, n in enumerate(sizes):
        cols = {"a": ("INT", rng.integers(0, 4 + i, n).astype(np.int32)),
                "b": ("STRING", np.array(["k%d" % v for v in rng.integers(0, 30 + 7 * i, n)], dtype=object)),
                "m": ("INT", rng.integers(-500, 1000, n).astype(np.int32)),
                "x": ("LONG", rng.integers(0, 1 << 30, n).astype(np.int64)),
                "d": ("DOUBLE", rng.integers(-1 << 20, 1 << 20, n).astype(np.float64) / 8.0),
                "h": ("INT", rng.integers(0, 5000, n).astype(np.int32))}
        segs.append(build_segment("rgg%d" % i, cols, allow_sorted=False))
    gs = [engine.register(s) for s in segs]
    if cfg:
        engine.set_config(cfg)
    try:
        ex = ServerQueryExecutor(engine)
        aggs = [{"function": f, "column": c} for f, c in (
            ("COUNT", "*"), ("SUM", "x"), ("AVG", "m"), ("MIN", "d"), ("MAX", "x"), ("SUM", "d"),
            ("DISTINCTCOUNTHLL", "h"))]
        for gcols in (["a"], ["b"], ["b", "a"]):
            for flt in (None, {"operator": "RANGE", "column": "m", "values": ["[0\t\t500)"]}):
                q = {"aggregations": aggs, "filter": flt, "group_by": {"columns": gcols, "top_n": 10}}
                got, st = ex.process_query(q, gs, trim=False)
                exp, scanned = O.execute_server(segs, q)
                assert st.num_docs_scanned == scanned
                assert set(got) == set(exp), (gcols, flt)
                for k in exp:
                    for a, gv, ev in zip(aggs, got[k], exp[k]):
                        _same_value(a["function"], gv, ev)
    finally:
        engine.set_config("exec.fused=1;group.mode=auto")
        for g in gs:
            g.release()


RAGGED_CONFIGS = ["", "exec.fused=0", "group.mode=lds", "group.mode=global", "plan.cache=0;agg.affine=0"]


@pytest.mark.parametrize("cfg", RAGGED_CONFIGS)
@pytest.mark.parametrize("seed", range(3))
def test_random_ragged(engine, cfg, seed):
    """Random filters (nested AND / OR over every predicate kind, sorted / bitmap / scan leaves), aggregations and
    group-bys over 2-4 segments of independent sizes and dictionaries, on each plan, against the oracle."""
    from test_gpu_parity import _assert_same, _random_aggs, _random_segment, _random_tree
    rng = np.random.default_rng(2300 + seed)
    sizes = [int(rng.choice([1, 63, 64, 65, 999, 4097, 40000])) for _ in range(int(rng.integers(2, 5)))]
    segs = [_random_segment(rng, n, name="rr%d" % i) for i, n in enumerate(sizes)]
    gs = [engine.register(s) for s in segs]
    if cfg:
        engine.set_config(cfg)
    try:
        ex = ServerQueryExecutor(engine)
        for it in range(10):
            group = None
            if it % 2:
                gcols = list(rng.choice(["i0", "i1", "i2", "s", "srt", "i3"], size=int(rng.integers(1, 3)), replace=False))
                group = {"columns": gcols, "top_n": 10}
            q = {"aggregations": _random_aggs(rng),
                 "filter": _random_tree(rng, segs[int(rng.integers(0, len(segs)))]) if rng.random() < 0.8 else None,
                 "group_by": group}
            got, st = ex.process_query(q, gs, trim=False) if group else ex.process_query(q, gs)
            exp, scanned = O.execute_server(segs, q)
            assert st.num_docs_scanned == scanned, (sizes, q)
            rows = [(got[k], exp[k]) for k in exp] if group else [(got, exp)]
            if group:
                assert set(got) == set(exp), (sizes, q)
            for gv_row, ev_row in rows:
                for a, gv, ev in zip(q["aggregations"], gv_row, ev_row):
                    _assert_same(a["function"], gv, ev, a["column"] not in ("dbl", "flt", "lng"))
    finally:
        engine.set_config("exec.fused=1;group.mode=auto;plan.cache=1;agg.affine=1")
        for g in gs:
            g.release()


@pytest.mark.parametrize("seed", range(3))
def test_random_ragged_multi_value(engine, seed):
    """The multi-value plans (MV leaves, *MV functions, cartesian-product group keys) over segments of independent
    sizes, entry counts and dictionaries."""
    from test_gpu_mv import _aggs, _check, _tree
    from test_mv import mv_segment
    rng = np.random.default_rng(2400 + seed)
    sizes = [int(rng.choice([1, 7, 64, 65, 999, 20000])) for _ in range(int(rng.integers(2, 5)))]
    segs = [mv_segment(rng, n, name="rm%d" % i) for i, n in enumerate(sizes)]
    gs = [engine.register(s) for s in segs]
    ex = ServerQueryExecutor(engine)
    shapes = [None, ["tags"], ["g"], ["tags_s", "g"], None, ["s", "tagl"]]
    try:
        for it in range(12):
            cols = shapes[it % len(shapes)]
            q = {"aggregations": _aggs(rng),
                 "filter": _tree(rng, segs[int(rng.integers(0, len(segs)))]) if rng.random() < 0.7 else None,
                 "group_by": {"columns": cols, "top_n": 10} if cols else None}
            got, st = ex.process_query(q, gs, trim=False) if cols else ex.process_query(q, gs)
            exp, scanned = O.execute_server(segs, q)
            assert st.num_docs_scanned == scanned, (sizes, q)
            _check(q, got, exp)
    finally:
        for g in gs:
            g.release()


@pytest.mark.parametrize("K", [2, 5])
def test_ragged_loopback_server(K):
    """The multi-GPU merge (server.loopback=1: K engines on device 0) over segments of independent sizes: union
    dictionaries, per-engine partials of ragged segments, the reduce-scatter and gather."""
    from pinot_amd import GpuServer, ServerExecutor, compile_pql
    from test_gpu_loopback import AGG_QUERIES, GROUP_QUERIES, _check_agg, _check_group, _segments
    rng = np.random.default_rng(2500 + K)
    host = []
    for i, n in enumerate([int(rng.choice([1, 65, 999, 4097, 30000])) for _ in range(6)]):
        s = _segments(rng, n, 1, t_base=[1000 * (i % 2)])[0]
        s.name = "rl%d" % i
        host.append(s)
    srv = GpuServer([0] * K, "server.loopback=1")
    try:
        gsegs = [srv.engines[i % K].register(s) for i, s in enumerate(host)]
        ex = ServerExecutor(srv, num_groups_limit=100000)
        for text in GROUP_QUERIES:
            q = compile_pql(text)
            got, st = ex.process_query(q, gsegs, trim=False)
            exp, scanned = O.execute_server(host, q)
            assert st.num_docs_scanned == scanned, text
            _check_group(q, got, exp)
        for text in AGG_QUERIES:
            q = compile_pql(text)
            got, st = ex.process_query(q, gsegs)
            exp, scanned = O.execute_server(host, q)
            assert st.num_docs_scanned == scanned, text
            _check_agg(q, got, exp)
    finally:
        srv.close()


@pytest.mark.parametrize("seed", range(3))
def test_ragged_exact_filter_stats(seed):
    """stats.exact=1 over segments of independent sizes and dictionaries: numEntriesScannedInFilter is the sum of
    each segment's replay of the iterator protocol (oracle/iter_stats.py), for aggregation and group-by plans."""
    import iter_stats
    from test_gpu_parity import _random_aggs, _random_segment, _random_tree
    rng = np.random.default_rng(2600 + seed)
    sizes = [int(rng.choice([1, 64, 777, 5000, 20000])) for _ in range(int(rng.integers(2, 4)))]
    segs = [_random_segment(rng, n, name="rs%d" % i) for i, n in enumerate(sizes)]
    e = GpuEngine(0, "stats.exact=1")
    try:
        gs = [e.register(s) for s in segs]
        ex = ServerQueryExecutor(e)
        for it in range(10):
            tree = _random_tree(rng, segs[int(rng.integers(0, len(segs)))])
            group = {"columns": ["i0"], "top_n": 10} if it % 2 else None
            q = {"aggregations": _random_aggs(rng), "filter": tree, "group_by": group}
            _, st = ex.process_query(q, gs, trim=False) if group else ex.process_query(q, gs)
            want = sum(iter_stats.entries_scanned_in_filter(s, tree) for s in segs)
            assert st.num_entries_scanned_in_filter == want, (sizes, tree)
    finally:
        e.close()

