"""The multi-GPU merge protocol with K > 1 ranks on the box's one GPU (server.loopback=1).

Every rank of the communicator lives in this process on device 0 and the collectives are done by the library's
loopback (an in-library device reduce / copy over the ranks' buffers in place of RCCL), so the code a multi-GPU
server runs — the dictionary exchange and union key space, Gp padding, reduce-scatter slicing, per-rank owner
finalize, the gather of every key range to rank 0, identity partials for ranks without segments, and the agreement
that fails every rank together — executes with K = 2, 3 and 8 ranks and is checked against the oracle's
CombineOperator / CombineGroupByOperator (CombineGroupByOperator.java:104-228, CombineOperator.java:75-196).

Two forms: one server over K engines (pinot_gpu_server_create with device 0 repeated, one thread per engine inside
the library) and K servers of the multi-process form (pinot_gpu_server_create_rank, one Python thread per rank, as
one process per GPU would call it)."""
import threading

import numpy as np
import pytest

import pinot_oracle as O
from pinot_amd import GpuServer, PinotGpuError, ServerExecutor, build_segment, compile_pql

pytestmark = pytest.mark.gpu

WORDS = ["a", "bb", "ccc", "P", "t", "zz", "Hello", "wé", "q%"]


def _segments(rng, n, nseg, t_base=None):
    """Segments whose group-by dictionaries differ (shifted g0 values, string subsets); t: a time-like column with
    min / max metadata (t_base[i] + [0, 1000)) the ColumnValue pruner reads."""
    segs = []
    for i in range(nseg):
        tb = 0 if t_base is None else t_base[i]
        cols = {"g0": ("INT", (rng.integers(0, 300, n) + 7 * i).tolist()),
                "g1": ("STRING", [WORDS[k] for k in rng.integers(0, len(WORDS) - (i % 3), n)]),
                "m": ("INT", rng.integers(-5000, 1000000, n).tolist()),
                "l": ("LONG", rng.integers(-2 ** 40, 2 ** 40, n).tolist()),
                "d": ("DOUBLE", np.round(rng.normal(0, 100, n), 3).tolist()),
                "h": ("INT", rng.integers(0, 5000, n).tolist()),
                "t": ("INT", (rng.integers(0, 1000, n) + tb).tolist()),
                "b": ("INT", rng.integers(0, 2, n).tolist())}
        segs.append(build_segment("seg%d" % i, cols, inverted_columns=("g1",), min_max=True))
    return segs


GROUP_QUERIES = [
    "SELECT COUNT(*), SUM(m), AVG(m), MIN(d), MAX(l), DISTINCTCOUNTHLL(h) FROM t WHERE m > 1000 GROUP BY g0, g1",
    "SELECT SUM(d), MAX(m), COUNT(*) FROM t WHERE g1 IN ('a', 'zz', 'q%') OR h < 100 GROUP BY g1",
    "SELECT COUNT(*), SUM(m), MIN(m), DISTINCTCOUNTHLL(l) FROM t WHERE t < 500 GROUP BY h",
    # a key space smaller than the rank count: ranks with an empty key range
    "SELECT COUNT(*), SUM(m), MAX(d) FROM t GROUP BY b",
]
AGG_QUERIES = [
    "SELECT COUNT(*), SUM(m), AVG(l), MIN(m), MAX(d), SUM(d), DISTINCTCOUNTHLL(g1) FROM t WHERE h BETWEEN 10 AND 4000",
    "SELECT COUNT(*), MIN(d), MAX(l) FROM t WHERE m = 123456789",
    "SELECT COUNT(*), SUM(m), MIN(d) FROM t WHERE t < 500",
]


def _check_group(q, got, exp):
    assert set(got) == set(exp), q
    for k in exp:
        for a, g, e in zip(q["aggregations"], got[k], exp[k]):
            f = a["function"].upper()
            if f == "AVG":
                assert g.count == e[1] and abs(g.sum - e[0]) <= 1e-9 * max(1.0, abs(e[0]))
            elif f == "DISTINCTCOUNTHLL":
                assert g.cardinality() == e.cardinality()
                assert (np.asarray(g.registers, dtype=np.int64) == e.reg).all()
            elif a["column"] == "d":
                assert abs(g - e) <= 1e-9 * max(1.0, abs(e))
            else:
                assert g == e, (k, a)


def _check_agg(q, got, exp):
    for a, g, e in zip(q["aggregations"], got, exp):
        f = a["function"].upper()
        if f == "AVG":
            assert g.count == e[1] and abs(g.sum - e[0]) <= 1e-9 * max(1.0, abs(e[0]))
        elif f == "DISTINCTCOUNTHLL":
            assert g.cardinality() == e.cardinality()
        elif a["column"] == "d":
            assert g == e or abs(g - e) <= 1e-9 * max(1.0, abs(e))
        else:
            assert g == e, a


def _threads(K, fn):
    """fn(r) on K threads (ctypes releases the GIL in library calls); per rank (result, exception)."""
    out = [None] * K
    err = [None] * K

    def run(r):
        try:
            out[r] = fn(r)
        except BaseException as ex:  # noqa: BLE001 - reported per rank
            err[r] = ex

    th = [threading.Thread(target=run, args=(r,)) for r in range(K)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a rank is still blocked in the merge"
    return out, err


def _rank_servers(K, host_by_rank, config="server.loopback=1"):
    uid = GpuServer.unique_id()
    servers = [GpuServer.rank(0, K, r, uid, config) for r in range(K)]
    segs = [[servers[r].engines[0].register(s) for s in host_by_rank[r]] for r in range(K)]
    return servers, segs


@pytest.mark.parametrize("K", [2, 3, 8])
def test_loopback_one_server_k_engines(K):
    """One server, K engines on device 0 (segment i -> engine i mod K; with 5 segments and K = 8 three engines hold
    none), union dictionaries, pruned segments, a key space smaller than K."""
    rng = np.random.default_rng(100 + K)
    host = _segments(rng, 9000, 5, t_base=[0, 1000, 0, 1000, 0])
    srv = GpuServer([0] * K, "server.loopback=1")
    gsegs = [srv.engines[i % K].register(s) for i, s in enumerate(host)]
    ex = ServerExecutor(srv, num_groups_limit=100000)
    for text in GROUP_QUERIES:
        q = compile_pql(text)
        got, st = ex.process_query(q, gsegs, trim=False)
        exp, scanned = O.execute_server(host, q)
        assert st.num_docs_scanned == scanned and st.num_total_raw_docs == 5 * 9000
        _check_group(q, got, exp)
    for text in AGG_QUERIES:
        q = compile_pql(text)
        got, st = ex.process_query(q, gsegs)
        exp, scanned = O.execute_server(host, q)
        assert st.num_docs_scanned == scanned and st.num_total_raw_docs == 5 * 9000
        _check_agg(q, got, exp)
    srv.close()


@pytest.mark.parametrize("K", [2, 3, 8])
def test_loopback_rank_form(K):
    """K servers of the multi-process form, one thread per rank: rank 0 returns the whole merged group-by result,
    the others an empty one; aggregations are complete on every rank. Rank 1 holds only segments the `t < 500`
    queries prune; with K = 8 some ranks hold no segment at all."""
    rng = np.random.default_rng(200 + K)
    nseg = 6
    host = _segments(rng, 8000, nseg, t_base=[0, 1000, 0, 1000, 0, 0])
    by_rank = [[] for _ in range(K)]
    by_rank[1] = [host[1], host[3]]  # every segment of rank 1 is pruned by t < 500
    rest = [host[i] for i in (0, 2, 4, 5)]
    for i, s in enumerate(rest):
        by_rank[(0 if K == 2 else 2 + i % (K - 2)) if K > 2 else 0].append(s)
    servers, segs = _rank_servers(K, by_rank)
    execs = [ServerExecutor(s, num_groups_limit=100000) for s in servers]
    for text in GROUP_QUERIES:
        q = compile_pql(text)
        exp, scanned = O.execute_server(host, q)
        out, err = _threads(K, lambda r: execs[r].process_query(q, segs[r], trim=False))
        assert not any(err), err
        got, st = out[0]
        assert st.num_docs_scanned == scanned and st.num_total_raw_docs == nseg * 8000, text
        _check_group(q, got, exp)
        for r in range(1, K):
            assert out[r][0] == {} and out[r][1].num_docs_scanned == scanned
    for text in AGG_QUERIES:
        q = compile_pql(text)
        exp, scanned = O.execute_server(host, q)
        out, err = _threads(K, lambda r: execs[r].process_query(q, segs[r]))
        assert not any(err), err
        for r in range(K):
            got, st = out[r]
            assert st.num_docs_scanned == scanned and st.num_total_raw_docs == nseg * 8000
            _check_agg(q, got, exp)
    for s in servers:
        s.close()


def _wide_segments(rng, n, nseg):
    """Segments of n docs over a ~1M-key space (g0, g1 ~1000 values each, g0 shifted per segment: dictionaries
    differ): tens of thousands of distinct keys per segment, so the 2 x num.groups.limit inter-segment cap binds."""
    segs = []
    for i in range(nseg):
        cols = {"g0": ("INT", (rng.integers(0, 990, n) + 3 * i).tolist()),
                "g1": ("INT", rng.integers(0, 1000, n).tolist()),
                "m": ("INT", rng.integers(-5000, 1000000, n).tolist()),
                "d": ("DOUBLE", np.round(rng.normal(0, 100, n), 3).tolist()),
                "h": ("INT", rng.integers(0, 5000, n).tolist()),
                "f": ("INT", rng.integers(0, 10, n).tolist())}
        segs.append(build_segment("wide%d" % i, cols))
    return segs


@pytest.mark.parametrize("K,limit", [(2, 100_000), (3, 100_000), (8, 100_000), (3, 20_000)])
def test_loopback_num_groups_limit_across_ranks(K, limit):
    """num.groups.limit across GPUs: each rank applies its segments' first-appearance holder rule
    (DictionaryBasedGroupKeyGenerator.java:293-302; at limit 20,000 it binds inside every segment), then the 2 x limit
    inter-segment cap (CombineGroupByOperator.java:80,147) over every rank's segments in rank order, then each rank's
    own segment order: the admitted key set and every group's values equal the oracle's one-server combine over the
    segments in that order (more than 200,000 possible keys)."""
    rng = np.random.default_rng(400 + K + limit)
    nseg = 7
    host = _wide_segments(rng, 60_000, nseg)
    srv = GpuServer([0] * K, "server.loopback=1")
    gsegs = [srv.engines[i % K].register(s) for i, s in enumerate(host)]
    ordered = [host[i] for r in range(K) for i in range(nseg) if i % K == r]  # rank order, then each rank's order
    ex = ServerExecutor(srv, num_groups_limit=limit)
    q = compile_pql("SELECT COUNT(*), SUM(m), MAX(d), DISTINCTCOUNTHLL(h) FROM t WHERE f < 9 GROUP BY g0, g1")
    exp = O.execute_group_by_arrays(ordered, q, num_groups_limit=limit)
    assert exp["keys"].shape[0] == 2 * limit  # the cap bound
    res, st = ex.process_query(q, gsegs, as_result=True)
    assert st.num_docs_scanned == exp["scanned"]
    keys = res.raw_keys()
    assert keys.shape == exp["keys"].shape and (keys == exp["keys"]).all()
    c, v = res.function_values(1)
    assert (c == exp["fns"][1]["count"]).all() and (v == exp["fns"][1]["sum"]).all()
    _, v = res.function_values(2)
    assert (v == exp["fns"][2]["max"]).all()
    regs, cards = res.hll(3)
    assert (cards == exp["fns"][3]["card"]).all() and (regs == exp["fns"][3]["hll"]).all()
    del res
    srv.close()


def test_loopback_key_ranges_without_gather():
    """server.gather=0: every rank returns its own key range; the ranges are disjoint, ascend with the rank and
    together are the oracle's result."""
    K = 3
    rng = np.random.default_rng(300)
    host = _segments(rng, 7000, 4)
    by_rank = [[host[0], host[3]], [host[1]], [host[2]]]
    servers, segs = _rank_servers(K, by_rank, "server.loopback=1;server.gather=0")
    q = compile_pql(GROUP_QUERIES[0])
    exp, _ = O.execute_server(host, q)
    from pinot_amd.executor import GroupByResult  # noqa: F401
    out, err = _threads(K, lambda r: ServerExecutor(servers[r]).process_query(q, segs[r], trim=False, as_result=True))
    assert not any(err), err
    merged = {}
    last = -1
    for r in range(K):
        res = out[r][0]
        keys = res.raw_keys()
        if len(keys):
            assert keys[0] > last and (np.diff(keys) > 0).all()
            last = keys[-1]
        m = res.to_map()
        assert not set(m) & set(merged)
        merged.update(m)
    _check_group(q, merged, exp)
    for s in servers:
        s.close()


def test_loopback_failure_on_one_rank_fails_every_rank():
    """A failure on one rank only — its segments lack a filter column (no pruning: unknown column, BAD_QUERY), or its
    query budget is already spent (TIMEOUT) — fails EVERY rank with that status, and nobody hangs."""
    K = 3
    rng = np.random.default_rng(400)
    host = _segments(rng, 5000, 3)
    odd = build_segment("odd", {"g0": ("INT", rng.integers(0, 50, 5000).tolist()),
                                "m": ("INT", rng.integers(0, 100, 5000).tolist())})
    servers, segs = _rank_servers(K, [[host[0]], [odd], [host[1], host[2]]])
    for text in ("SELECT COUNT(*), SUM(m) FROM t WHERE h < 100 GROUP BY g0", "SELECT COUNT(*), SUM(m) FROM t WHERE h < 100"):
        q = compile_pql(text)
        out, err = _threads(K, lambda r: ServerExecutor(servers[r], pruners=0).process_query(q, segs[r]))
        assert all(isinstance(e, PinotGpuError) and e.status == 5 for e in err), err
    q = compile_pql("SELECT COUNT(*), SUM(m) FROM t GROUP BY g0")
    out, err = _threads(K, lambda r: ServerExecutor(servers[r], timeout_ms=(-1 if r == 2 else 0))
                        .process_query(q, [segs[r][0]] if r != 1 else []))
    assert all(isinstance(e, PinotGpuError) and e.status == 6 for e in err), err
    # the communicator is still usable after a failed query (every rank left it together)
    out, err = _threads(K, lambda r: ServerExecutor(servers[r]).process_query(q, segs[r] if r != 1 else []))
    assert not any(err), err
    exp, _ = O.execute_server([host[0], host[1], host[2]], q)
    _check_group(q, out[0][0], exp)
    for s in servers:
        s.close()


def test_loopback_no_rank_holds_a_segment():
    """Every segment on every rank pruned: all ranks return the empty result (identities / no group) with totalDocs
    over every segment."""
    K = 2
    rng = np.random.default_rng(500)
    host = _segments(rng, 4000, 2, t_base=[1000, 2000])
    servers, segs = _rank_servers(K, [[host[0]], [host[1]]])
    q = compile_pql("SELECT COUNT(*), SUM(m) FROM t WHERE t < 500 GROUP BY g0")
    out, err = _threads(K, lambda r: ServerExecutor(servers[r]).process_query(q, segs[r]))
    assert not any(err), err
    assert out[0][0] == {} and out[0][1].num_total_raw_docs == 8000 and out[0][1].num_segments_processed == 0
    q = compile_pql("SELECT COUNT(*), SUM(m), MIN(d), MAX(d) FROM t WHERE t < 500")
    out, err = _threads(K, lambda r: ServerExecutor(servers[r]).process_query(q, segs[r]))
    assert not any(err), err
    assert out[1][0] == [0, 0.0, float("inf"), float("-inf")] and out[1][1].num_total_raw_docs == 8000
    for s in servers:
        s.close()


def test_loopback_mv_and_star_tree_aggregations():
    """Aggregation-only queries over multi-value columns (the MV functions merge as their single-value forms across
    ranks) and over star-tree segments, with K = 3 loopback ranks, against the oracle."""
    import startree as S
    from startree_writer import build_star_tree
    from test_mv import mv_segment
    from test_startree import DIMS, PAIRS, st_segment
    rng = np.random.default_rng(4242)
    host = [mv_segment(rng, 3000, name="mv%d" % i) for i in range(4)]
    srv = GpuServer([0] * 3, "server.loopback=1")
    gsegs = [srv.engines[i % 3].register(s) for i, s in enumerate(host)]
    ex = ServerExecutor(srv, pruners=0)
    q = {"aggregations": [{"function": f, "column": c} for f, c in (
        ("COUNTMV", "tags"), ("SUMMV", "tags"), ("MINMV", "tagl"), ("MAXMV", "tags"), ("AVGMV", "tags"),
        ("DISTINCTCOUNTHLLMV", "tags_s"), ("COUNT", "*"))],
         "filter": {"operator": "NOT_IN", "column": "tags_s", "values": ["t01\t\tt03"]}, "group_by": None}
    got, st = ex.process_query(q, gsegs)
    exp, scanned = O.execute_server(host, q)
    assert st.num_docs_scanned == scanned
    assert got[0] == exp[0] and got[1] == exp[1] and got[2] == exp[2] and got[3] == exp[3] and got[6] == exp[6]
    assert (got[4].sum, got[4].count) == exp[4]
    assert got[5].cardinality() == exp[5].cardinality()
    srv.close()
    # star-tree segments on every rank
    sts_host = [st_segment(rng, 2000, name="st%d" % i) for i in range(3)]
    trees = [build_star_tree(s, DIMS, PAIRS, max_leaf_records=10) for s in sts_host]
    srv = GpuServer([0] * 3, "server.loopback=1")
    gsegs = []
    for i, (s, t) in enumerate(zip(sts_host, trees)):
        g = srv.engines[i % 3].register(s)
        g.attach_star_tree(s, t.tree_bytes, t.dimensions, t.dims, t.metrics)
        gsegs.append(g)
    ex = ServerExecutor(srv, pruners=0)
    q = {"aggregations": [{"function": "COUNT", "column": "*"}, {"function": "SUM", "column": "m"},
                          {"function": "MAX", "column": "x"}, {"function": "AVG", "column": "m"}],
         "filter": {"operator": "IN", "column": "c", "values": ["3\t\t9\t\t30"]}, "group_by": None}
    got, st = ex.process_query(q, gsegs)
    exp, scanned = S.execute_server(sts_host, trees, q)
    assert got[:3] == exp[:3] and (got[3].sum, got[3].count) == exp[3] and st.num_docs_scanned == scanned
    srv.close()


@pytest.mark.parametrize("K", [2, 3])
def test_loopback_mv_group_by(K):
    """Group-by over multi-value group columns and with *MV functions across K loopback ranks: each rank's
    k_group_by_mv partial over the union key space (AvgMV's entry count in a hidden CountMV array through the
    reduce-scatter), then, with a binding num.groups.limit, each segment's first-appearance holder (getIntRawKeys
    order) and the 2 x limit cap over every rank's segments in rank order, then each rank's segment order
    (DictionaryBasedGroupKeyGenerator.java:282-302, CombineGroupByOperator.java:80,147)."""
    from test_gpu_mv import _check
    from test_mv import mv_segment
    rng = np.random.default_rng(4600 + K)
    nseg = 5
    host = [mv_segment(rng, int(rng.choice([800, 2500])), name="lm%d" % i) for i in range(nseg)]
    srv = GpuServer([0] * K, "server.loopback=1")
    gsegs = [srv.engines[i % K].register(s) for i, s in enumerate(host)]
    ordered = [host[i] for r in range(K) for i in range(nseg) if i % K == r]
    aggs = [{"function": "COUNT", "column": "*"}, {"function": "SUM", "column": "m"},
            {"function": "MAXMV", "column": "tags"}, {"function": "AVGMV", "column": "tagl"},
            {"function": "COUNTMV", "column": "tags_s"}, {"function": "DISTINCTCOUNTHLLMV", "column": "tagd"}]
    for cols, limit, thr in ((["tags", "g"], 100_000, 10_000), (["tags_s", "g"], 100_000, 10_000),
                             (["g"], 100_000, 10_000), (["tags", "tags_s"], 60, 10), (["tagl", "tags"], 150, 40)):
        q = {"aggregations": aggs, "filter": {"operator": "RANGE", "column": "m", "values": ["[-900\t\t*)"]},
             "group_by": {"columns": cols, "top_n": 10}}
        ex = ServerExecutor(srv, num_groups_limit=limit, max_init_group_holder_capacity=thr, pruners=0)
        got, st = ex.process_query(q, gsegs, trim=False)
        exp, scanned = O.execute_server(ordered, q, num_groups_limit=limit, array_threshold=thr)
        assert st.num_docs_scanned == scanned
        if limit < 1000:
            assert len(exp) == 2 * limit  # the cap binds
        _check(q, got, exp)
    srv.close()


def _trim_segments(rng, n, nseg):
    """Segments of ~60,000 group keys (more than 4 x trimSize at TOP 10): the server trim binds."""
    return [build_segment("wide%d" % i, {
        "k": ("INT", rng.integers(0, 60_000, n).tolist()),
        "j": ("INT", rng.integers(0, 3, n).tolist()),
        "m": ("INT", rng.integers(-5000, 1_000_000, n).tolist()),
        "h": ("INT", rng.integers(0, 50, n).tolist())}) for i in range(nseg)]


@pytest.mark.parametrize("K", [2, 3, 8])
def test_loopback_trimmed_server_answer(K):
    """pinot_gpu_server_group_by_top: each rank trims its own key range (its trimSize best groups per function) before
    the gather, rank 0 picks each function's trimSize best among them. The DataTable equals the one-engine device-trimmed
    answer over the same segments (itself checked against the host trim), every kept value equals the oracle's merged
    map, and below 4 x trimSize groups nothing is trimmed."""
    import datatable as D
    from pinot_amd import GpuEngine, ServerQueryExecutor
    rng = np.random.default_rng(500 + K)
    host = _trim_segments(rng, 60_000, 5)
    srv = GpuServer([0] * K, "server.loopback=1")
    gsegs = [srv.engines[i % K].register(s) for i, s in enumerate(host)]
    ex = ServerExecutor(srv, num_groups_limit=1_000_000)
    eng = GpuEngine(0)
    esegs = [eng.register(s) for s in host]
    ee = ServerQueryExecutor(eng, num_groups_limit=1_000_000)
    for text, trimmed in (("SELECT COUNT(*), SUM(m), MIN(m), AVG(m), DISTINCTCOUNTHLL(h) FROM t GROUP BY k TOP 10", True),
                          ("SELECT MAX(m), COUNT(*) FROM t WHERE h < 10 GROUP BY k, j TOP 20", True),
                          ("SELECT SUM(m), COUNT(*) FROM t WHERE k < 15000 GROUP BY k TOP 10", False)):
        q = compile_pql(text)
        data, st = ex.process_query_datatable(q, gsegs, trim=True)
        ref, _ = ee.process_query_datatable(q, esegs, trim=True)
        d, r = D.decode(data), D.decode(ref)
        assert d["cells"] == r["cells"], text
        md = dict(d["metadata"])
        assert md.get("numGroupsLimitReached") == dict(r["metadata"]).get("numGroupsLimitReached")
        exp, _ = O.execute_server(host, q, num_groups_limit=1_000_000)
        T = max(5 * q["group_by"].get("top_n", 10), 5000)
        for i, (a, row) in enumerate(zip(q["aggregations"], d["cells"])):
            got = row[1]
            assert len(got) == (T if trimmed else len(exp)), (text, i)
            f = a["function"].upper()
            for k, v in list(got.items())[:300]:
                e = exp[k][i]
                if f == "AVG":
                    assert v[1] == e[1] and abs(v[0] - e[0]) <= 1e-9 * max(1.0, abs(e[0]))
                elif f == "DISTINCTCOUNTHLL":
                    assert v == [int(x) for x in e.reg]  # the registers (HyperLogLog.getBytes decoded)
                else:
                    assert v == e, (text, k, f)
        # the untrimmed merged result still holds every group; the trimmed one only the kept union (rank 0 got no more)
        res, _ = ex.group_by_result(q, gsegs)
        assert res.num_groups() == len(exp)
        del res
        top = q["group_by"].get("top_n", 10)
        res, _ = ex.group_by_result(q, gsegs, top_n=top)
        n_aggs = len(q["aggregations"])
        if trimmed:  # at most every rank's per-function candidates reached rank 0; each function keeps T of them
            assert res.num_groups() <= min(len(exp), K * n_aggs * T)
            assert all(len(res.trimmed_groups(top, i)) == T for i in range(n_aggs))
        else:
            assert res.num_groups() == len(exp)
        del res
    srv.close()
    eng.close()


@pytest.mark.parametrize("K", [2, 3, 8])
def test_loopback_hashed_key_space(K):
    """Group-bys over key spaces past the dense limit (LONG_MAP / ARRAY_MAP holders; MV and SV group columns) across K
    ranks: each rank runs its segments' group-bys (each segment's holder admission applied locally), rank 0 merges
    the segments' groups by key string in rank then segment order (CombineGroupByOperator.java:142-161) with the
    2 x num.groups.limit cap — equal to the oracle over the segments in that order, with and without the cap
    binding (DictionaryBasedGroupKeyGenerator.java:459-470)."""
    from test_gpu_mv import hashed_mv_segment, _check as _check_mv
    rng = np.random.default_rng(900 + K)
    host = [hashed_mv_segment(rng, 12000, "hk%d" % i) for i in range(4)]
    srv = GpuServer([0] * K, "server.loopback=1")
    gsegs = [srv.engines[i % K].register(s) for i, s in enumerate(host)]
    order = [host[i] for r in range(K) for i in range(len(host)) if i % K == r]  # the server's merge order
    aggs = [{"function": "COUNT", "column": "*"}, {"function": "SUMMV", "column": "tags"},
            {"function": "AVGMV", "column": "tags"}, {"function": "SUM", "column": "m"},
            {"function": "DISTINCTCOUNTHLLMV", "column": "tags"}, {"function": "MIN", "column": "m"}]
    for cols, limit, thr in ((["hv", "hs"], None, None), (["hs", "m", "g"], None, None), (["hv", "hs"], 500, 10)):
        q = {"aggregations": aggs, "filter": {"operator": "RANGE", "column": "m", "values": ["[-500\t\t900)"]},
             "group_by": {"columns": cols, "top_n": 10}}
        ex = ServerExecutor(srv, num_groups_limit=limit or 100000, max_init_group_holder_capacity=thr or 10000)
        got, st = ex.process_query(q, gsegs, trim=False)
        okw = {} if limit is None else {"num_groups_limit": limit, "array_threshold": thr}
        exp, scanned = O.execute_server(order, q, **okw)
        assert st.num_docs_scanned == scanned and st.num_total_raw_docs == 4 * 12000
        assert len(exp) > (2 * limit if limit else 10000) // 2
        _check_mv(q, got, exp)
        # the trimmed answer (TOP 10 -> 5,000 per function when more than 20,000 groups) keeps each function's best
        data, _ = ex.process_query_datatable(q, gsegs, trim=True)
        assert b"sumMV_tags" in data
    srv.close()
