"""GPU parity for the paths the BASELINE configs run at full size, at sizes the oracle finishes in seconds:

* every fixed-bit width 1..32 through the fused scan (RANGE / 64-entry LUT / membership-LUT leaves, Σ dictId,
  Σ dictionary value, min/max folds), the stepwise-pipelined kernel and the unfused launches, and the one-doc-per-lane
  group-key decode (PinotDataBitSet.readInt, PinotDataBitSet.java:79-100; FixedBitSingleValueReader.java:36-51);
* config 2's ten-column table (d8 at 20 bits) from the HBM generator;
* config 4's 1M-key GROUP BY d6, d7 with SUM / AVG (20-bit d8) and DISTINCTCOUNTHLL (16-bit d5) at
  num.groups.limit = 1,000,000 (dense partitioned plan) and at the reference default 100,000 (first-appearance
  admission per segment + the 2 x limit inter-segment cap; DictionaryBasedGroupKeyGenerator.java:261-335,
  CombineGroupByOperator.java:61,147).
Integer results bit-exact; whole group maps compared as arrays against the vectorised oracle."""
import numpy as np
import pytest

import pinot_oracle as O
import synth
from pinot_amd import GpuEngine, ServerQueryExecutor, build_segment, compile_pql

pytestmark = pytest.mark.gpu

WIDTH_MODES = ("", "exec.nt=0", "exec.pipe=1", "exec.fused=0")


@pytest.fixture(scope="module")
def engines():
    es = {m: GpuEngine(0, m or None) for m in WIDTH_MODES}
    yield es
    for e in es.values():
        e.close()


def _width_segment(b):
    """Columns at bitsPerElement b: w (affine dictionary 5*id - 1000, Σ dictId fold), x (non-affine dictionary,
    int32 gathers), f (card 16 filter column). b <= 16: minimal width; 17..20: minimal width with the top dictId bit
    used (card 2^(b-1) + 3); > 20: card 2^16 + 3 written at a wider metadata width (ColumnMetadata.java:98)."""
    rng = np.random.default_rng(1000 + b)
    if b <= 16:
        card = 1 << b
        n = max(70001 + 17 * b, card + 5000)
    elif b <= 20:
        card = (1 << (b - 1)) + 3
        n = card + 50001
    else:
        card = (1 << 16) + 3
        n = card + 30001
    def ids():
        v = np.concatenate([rng.permutation(card), rng.integers(0, card, n - card)])
        return v[rng.permutation(n)] if b % 2 else v
    iw, ix = ids(), ids()
    xd = 3 * np.arange(card, dtype=np.int64) + (np.arange(card, dtype=np.int64) ** 2) // card
    cols = {"w": ("INT", (5 * iw - 1000).tolist()), "x": ("INT", xd[ix].tolist()),
            "f": ("INT", rng.integers(0, 16, n).tolist())}
    seg = build_segment("width%d" % b, cols, bits={"w": b, "x": b}, allow_sorted=False)
    assert seg.column("w").bits == b and seg.column("x").bits == b
    return seg, card, xd


def _agg_equal(q, got, exp):
    for a, g, e in zip(q["aggregations"], got, exp):
        f = a["function"].upper()
        if f == "AVG":
            assert (g.sum, g.count) == e
        elif f == "DISTINCTCOUNTHLL":
            assert g.cardinality() == e.cardinality()
            assert (np.asarray(g.registers, dtype=np.int64) == e.reg).all()
        else:
            assert g == e, (a, g, e)


def _assert_group_arrays(res, exp, q):
    """GroupByResult (device) against execute_group_by_arrays, every group."""
    keys = res.raw_keys()
    assert keys.shape == exp["keys"].shape
    assert (keys == exp["keys"]).all()
    for i, (a, r) in enumerate(zip(q["aggregations"], exp["fns"])):
        f = a["function"].upper()
        if f == "DISTINCTCOUNTHLL":
            regs, cards = res.hll(i)
            assert (cards == r["card"]).all()
            assert (regs == r["hll"]).all()
            continue
        counts, vals = res.function_values(i)
        assert (counts == r["count"]).all()
        if f in ("SUM", "AVG"):
            assert (vals == r["sum"]).all()
        elif f == "MIN":
            assert (vals == r["min"]).all()
        elif f == "MAX":
            assert (vals == r["max"]).all()
    rng = np.random.default_rng(0)
    for g in rng.choice(keys.shape[0], size=min(200, keys.shape[0]), replace=False):
        assert res.lib.pinot_groupby_key(res.ptr, int(g)).decode() == O.key_string(exp, int(keys[g]))


@pytest.mark.parametrize("b", range(1, 33))
def test_fused_width_sweep(engines, b):
    seg, card, xd = _width_segment(b)
    vals_w = 5 * np.arange(card) - 1000
    lo, hi = int(vals_w[card // 5]), int(vals_w[(3 * card) // 4])
    xin = ", ".join(str(int(xd[min(card - 1, i)])) for i in sorted({0, card - 1, card // 3, card // 2 + 1,
                                                                       (7 * card) // 9}))
    queries = [
        "SELECT COUNT(*), SUM(w), MIN(w), MAX(w), SUM(x), MAX(x), MIN(x) FROM t WHERE w BETWEEN %d AND %d "
        "AND f IN (1, 3, 5, 7)" % (lo, hi),
        "SELECT COUNT(*), SUM(w), AVG(x), MIN(w) FROM t WHERE x IN (%s)" % xin,
        "SELECT COUNT(*), MAX(w), SUM(x) FROM t WHERE w NOT IN (%d, %d) AND x > %d" % (
            int(vals_w[1]), int(vals_w[card - 1]), int(xd[card // 7])),
        "SELECT COUNT(*), SUM(x), DISTINCTCOUNTHLL(w) FROM t WHERE f <> 4",
        # RANGE + LUT leaves with Σ dictId and min/max folds only; an OR of two leaves
        "SELECT COUNT(*), SUM(w), MIN(w), MAX(w) FROM t WHERE w BETWEEN %d AND %d AND f IN (1, 3, 5, 7)" % (lo, hi),
        "SELECT COUNT(*), MAX(w) FROM t WHERE f IN (2, 9) OR w < %d" % lo,
    ]
    gq = compile_pql("SELECT COUNT(*), SUM(x), MAX(x) FROM t WHERE f < 9 GROUP BY w")
    gexp = O.execute_group_by_arrays([seg], gq, num_groups_limit=1 << 22)
    for mode, e in engines.items():
        g = e.register(seg)
        ex = ServerQueryExecutor(e)
        for text in queries:
            q = compile_pql(text)
            got, st = ex.process_query(q, [g])
            exp, scanned = O.execute_server([seg], q)
            assert st.num_docs_scanned == scanned, (mode, text)
            _agg_equal(q, got, exp)
        res, st = ServerQueryExecutor(e, num_groups_limit=1 << 22).group_by_result(gq, [g])
        assert st.num_docs_scanned == gexp["scanned"]
        _assert_group_arrays(res, gexp, gq)
        del res
        g.release()


# ------------------------------------------------------------------ BASELINE config 2 / 4 tables (HBM generator)
CONFIG_COLUMNS = [("d0", 16), ("d1", 100), ("d2", 1000), ("d3", 4096), ("d4", 10000), ("d5", 65536), ("d6", 1000),
                  ("d7", 1000), ("d8", 1 << 20), ("d9", 1000)]
BASE_SEED = 0x5EED0000


def _synthetic(engine, nseg, docs):
    gsegs = [engine.register_synthetic("fact_%d" % s, docs, CONFIG_COLUMNS, BASE_SEED + s) for s in range(nseg)]
    host = [synth.make_segment("fact_%d" % s, docs, CONFIG_COLUMNS, BASE_SEED + s) for s in range(nseg)]
    return gsegs, host


def test_config2_ten_column_table():
    """Config 2's table (10 columns, d8 = 2^20 values at 20 bits) and query at 2 x 2M docs, plus variants that
    filter and fold the 20- and 16-bit columns; the HBM generator against its host restatement + the oracle."""
    e = GpuEngine(0)
    gsegs, host = _synthetic(e, 2, 2_000_003)
    ex = ServerQueryExecutor(e)
    for text in ("SELECT COUNT(*), SUM(d8) FROM fact WHERE d2 BETWEEN 100 AND 599 AND d0 IN (1, 3, 5, 7)",
                 "SELECT COUNT(*), SUM(d8), MIN(d8), MAX(d5), AVG(d3) FROM fact WHERE d8 < 524288 AND d5 >= 1000",
                 "SELECT SUM(d4), MAX(d8), DISTINCTCOUNTHLL(d5), COUNT(*) FROM fact WHERE d1 IN (3, 50, 99) OR d9 = 7",
                 "SELECT COUNT(*), SUM(d8), SUM(d7) FROM fact WHERE d8 NOT IN (0, 1048575) AND d6 BETWEEN 10 AND 20"):
        q = compile_pql(text)
        got, st = ex.process_query(q, gsegs)
        exp, scanned = O.execute_server(host, q)
        assert st.num_docs_scanned == scanned
        _agg_equal(q, got, exp)
    e.close()


CONFIG4 = ("SELECT SUM(d8), AVG(d8), DISTINCTCOUNTHLL(d5) FROM fact WHERE d2 < 800 GROUP BY d6, d7 TOP 10")


@pytest.mark.parametrize("mode,limit,nseg,docs", [
    ("", 1_000_000, 2, 2_000_000),                       # 1M keys, ring-partitioned plan (default)
    ("group.ring=0", 1_000_000, 2, 2_000_000),           # 1M keys, counted partitioned plan
    ("group.mode=global", 1_000_000, 2, 2_000_000),      # HBM-atomic sink
    ("", 100_000, 3, 1_500_000),                         # reference default limit: admission + inter-segment cap
    ("exec.fused=0", 100_000, 3, 1_500_000),             # the same on the bitset path
])
def test_config4_shape(mode, limit, nseg, docs):
    e = GpuEngine(0, mode or None)
    gsegs, host = _synthetic(e, nseg, docs)
    q = compile_pql(CONFIG4)
    exp = O.execute_group_by_arrays(host, q, num_groups_limit=limit)
    res, st = ServerQueryExecutor(e, num_groups_limit=limit).group_by_result(q, gsegs)
    assert st.num_docs_scanned == exp["scanned"]
    if limit < 1_000_000:
        assert exp["keys"].shape[0] == 2 * limit  # the inter-segment cap bound
    _assert_group_arrays(res, exp, q)
    del res
    e.close()


# ------------------------------------------------------------------ trimming, bulk export, query budget
def _oracle_trim(exp, q, fn, top_n):
    """AggregationGroupByTrimmingService.trimIntermediateResultsMap on the oracle arrays for one function (ties: lower
    raw key first, the engine's documented tie rule)."""
    f = q["aggregations"][fn]["function"].upper()
    r = exp["fns"][fn]
    n = exp["keys"].shape[0]
    trim_size = max(5 * top_n, 5000)
    if n <= 4 * trim_size:
        return np.arange(n)
    v = {"COUNT": lambda: r["count"].astype(np.float64), "SUM": lambda: r["sum"], "MIN": lambda: r["min"],
         "MAX": lambda: r["max"], "AVG": lambda: r["sum"] / r["count"],
         "DISTINCTCOUNTHLL": lambda: r["card"].astype(np.float64)}[f]()
    order = np.lexsort((np.arange(n), v if f == "MIN" else -v))
    return np.sort(order[:trim_size])


def test_server_trim_and_bulk_export_1m_groups():
    """More than 20,000 groups (4 x max(5 * topN, 5000)): the native trim keeps each function's own top 5000
    (MIN ascending, HLL by cardinality), the broker top-N over two servers equals the oracle's, and the bulk
    C-ABI export of the ~1M-group result (keys + values + cardinalities) is one call each."""
    import time
    from pinot_amd import BrokerReduce
    e = GpuEngine(0)
    gsegs, host = _synthetic(e, 2, 2_000_000)
    q = compile_pql("SELECT COUNT(*), SUM(d8), MIN(d4), MAX(d3), AVG(d9), DISTINCTCOUNTHLL(d5) FROM fact "
                    "WHERE d2 < 800 GROUP BY d6, d7 TOP 10")
    exp = O.execute_group_by_arrays(host, q, num_groups_limit=1_000_000)
    ex = ServerQueryExecutor(e, num_groups_limit=1_000_000)
    res, _ = ex.group_by_result(q, gsegs)
    n = res.num_groups()
    assert n == exp["keys"].shape[0] and n > 20000
    for fn in range(len(q["aggregations"])):
        kept = res.trimmed_groups(10, fn)
        assert kept.shape[0] == 5000
        assert (kept == _oracle_trim(exp, q, fn, 10)).all(), q["aggregations"][fn]
    t0 = time.perf_counter()
    buf, offs = res.key_bytes()
    for fn in range(len(q["aggregations"])):
        if q["aggregations"][fn]["function"] == "DISTINCTCOUNTHLL":
            continue
        res.function_values(fn)
    t_abi = time.perf_counter() - t0
    print("bulk C-ABI export of %d groups: %.1f ms" % (n, t_abi * 1e3))
    assert offs[-1] == len(buf) and t_abi < 0.5
    # broker top-N over two servers holding the same segments: per-function trimmed maps (65,536 groups), merged
    # per function, equal the top-N of the untrimmed maps
    qb = compile_pql("SELECT COUNT(*), SUM(d8), MIN(d4), AVG(d9), DISTINCTCOUNTHLL(d5) FROM fact WHERE d2 < 800 "
                     "GROUP BY d3, d0 TOP 10")
    server, _ = ex.process_query(qb, gsegs)
    assert len(server) < 65536
    got = BrokerReduce.reduce(qb, [server, server])
    full, _ = ex.process_query(qb, gsegs, trim=False)
    ref = BrokerReduce.reduce(qb, [full, full])
    for g, r in zip(got, ref):
        assert [v for _, v in g] == [v for _, v in r]
    del res
    e.close()


def test_device_trim_equals_host_trim():
    """pinot_gpu_group_by_top (CombineGroupByOperator's trim on the device, AggregationGroupByTrimmingService
    :71-116): each function's kept groups equal the oracle's trim of the full arrays, the result holds only their
    union, and the server's DataTable bytes equal the host-trimmed DataTable of the untrimmed result."""
    e = GpuEngine(0)
    gsegs, host = _synthetic(e, 2, 2_000_000)
    q = compile_pql("SELECT COUNT(*), SUM(d8), MIN(d4), MAX(d3), AVG(d9), DISTINCTCOUNTHLL(d5) FROM fact "
                    "WHERE d2 < 800 GROUP BY d6, d7 TOP 10")
    exp = O.execute_group_by_arrays(host, q, num_groups_limit=1_000_000)
    ex = ServerQueryExecutor(e, num_groups_limit=1_000_000)
    top, st = ex.group_by_result(q, gsegs, top_n=10)
    assert st.num_docs_scanned == exp["scanned"]
    ukeys = top.raw_keys()
    union = set()
    for fn in range(len(q["aggregations"])):
        kept = top.trimmed_groups(10, fn)
        want = exp["keys"][_oracle_trim(exp, q, fn, 10)]
        assert kept.shape[0] == 5000 and (ukeys[kept] == want).all(), q["aggregations"][fn]
        union |= set(want.tolist())
    assert sorted(union) == ukeys.tolist()
    # the kept groups' values are the full result's
    pos = np.searchsorted(exp["keys"], ukeys)
    c, v = top.function_values(1)
    assert (c == exp["fns"][1]["count"][pos]).all() and (v == exp["fns"][1]["sum"][pos]).all()
    regs, cards = top.hll(5)
    assert (cards == exp["fns"][5]["card"][pos]).all() and (regs == exp["fns"][5]["hll"][pos]).all()
    # DataTable: device trim == host trim of the untrimmed result
    got, _ = ex.process_query_datatable(q, gsegs, trim=True)
    full, st2 = ex.group_by_result(q, gsegs)
    m = ex.prepare(q).marshal
    ref = full.data_table(m, st2, 10)
    assert got == ref
    del top, full
    e.close()


def test_query_timeout_status():
    """pinot_query.timeout_ms: a budget already spent returns PINOT_ERR_TIMEOUT before any device work
    (ServerQueryExecutorV1Impl.java:116-126); a budget shorter than the device work times out in the wait
    (CombineGroupByOperator.java:174-181); the engine keeps serving queries afterwards."""
    from pinot_amd import PinotGpuError
    e = GpuEngine(0)
    gsegs, host = _synthetic(e, 2, 2_000_000)
    q = compile_pql(CONFIG4)
    for budget in (-1, 1):
        with pytest.raises(PinotGpuError) as ei:
            ServerQueryExecutor(e, num_groups_limit=1_000_000, timeout_ms=budget).group_by_result(q, gsegs)
        assert ei.value.status == 6
    q2 = compile_pql("SELECT COUNT(*), SUM(d8) FROM fact WHERE d2 BETWEEN 100 AND 599 AND d0 IN (1, 3, 5, 7)")
    got, _ = ServerQueryExecutor(e, timeout_ms=60000).process_query(q2, gsegs)
    exp, _ = O.execute_server(host, q2)
    assert got[0] == exp[0] and got[1] == exp[1]
    e.close()


# ------------------------------------------------------------------ the LDS-privatised group-by (bench `lds_group_by`)
LDS_QUERIES = [
    # the bench's lds_group_by query: 1,600 keys, COUNT + SUM / AVG of the 20-bit d8 (count packed beside the dictId
    # sum); 3 read columns -> the <= 3-column lane-owns-quarter GB_LDS instance (k_group_query<GB_LDS, 4, 512, 4>)
    ("SELECT COUNT(*), SUM(d8), AVG(d8) FROM fact WHERE d2 < 800 GROUP BY d0, d1 TOP 10", 1 * 10000 + 4 * 1000 + 512),
    # group.lds_qfilter=1: a one-leaf filter evaluated per quarter from its own loads (k_group_query<GB_LDS, 5, 512, 4>;
    # measured slower, off by default); two leaves stay staged (PATH 4); no filter: the `pre` words only (PATH 5)
    ("SELECT COUNT(*), SUM(d8), AVG(d8) FROM fact WHERE d2 < 800 GROUP BY d0, d1 TOP 10 |group.lds_qfilter=1",
     1 * 10000 + 5 * 1000 + 512),
    ("SELECT COUNT(*), SUM(d8) FROM fact WHERE d2 < 800 AND d3 > 100 GROUP BY d0, d1 TOP 10 |group.lds_qfilter=1",
     1 * 10000 + 4 * 1000 + 512),
    ("SELECT COUNT(*), SUM(d8) FROM fact GROUP BY d0, d1 TOP 10 |group.lds_qfilter=1", 1 * 10000 + 5 * 1000 + 512),
    ("SELECT COUNT(*), MAX(d8) FROM fact WHERE d0 IN (1, 4, 9) GROUP BY d1, d0 TOP 10 |group.lds_qfilter=1",
     1 * 10000 + 5 * 1000 + 512),
    # MIN / MAX: 4 read columns -> the general lane-owns-quarter instance (k_group_query<GB_LDS, 3, 512, 4>)
    ("SELECT MIN(d8), MAX(d3), COUNT(*) FROM fact WHERE d2 < 800 GROUP BY d0, d1 TOP 10", 1 * 10000 + 3 * 1000 + 512),
    ("SELECT MAX(d3), SUM(d8), AVG(d8) FROM fact WHERE d2 < 800 GROUP BY d0, d1 TOP 10", 1 * 10000 + 3 * 1000 + 512),
    # DISTINCTCOUNTHLL: 1,600 keys x 1 KiB of LDS registers do not fit 60 KiB -> another sink (group-level parity only)
    ("SELECT COUNT(*), SUM(d8), DISTINCTCOUNTHLL(d5) FROM fact WHERE d2 < 800 GROUP BY d0, d1 TOP 10", None),
]


@pytest.mark.parametrize("text,instance", LDS_QUERIES)
def test_lds_shape(text, instance):
    """The bench's LDS group-by workload (config 2's table, GROUP BY d0, d1: 16 x 100 keys) at 2 x 2M docs in the
    default engine mode: every group's count, integer sum, MIN / MAX and HLL registers against the oracle's arrays,
    and the kernel instance that ran (group.last_instance)."""
    text, _, cfg = text.partition(" |")
    e = GpuEngine(0, cfg or None)
    gsegs, host = _synthetic(e, 2, 2_000_000)
    q = compile_pql(text)
    exp = O.execute_group_by_arrays(host, q, num_groups_limit=1_000_000)
    res, st = ServerQueryExecutor(e, num_groups_limit=1_000_000).group_by_result(q, gsegs)
    assert st.num_docs_scanned == exp["scanned"]
    assert exp["keys"].shape[0] == (300 if "IN (1, 4, 9)" in text else 1600)
    _assert_group_arrays(res, exp, q)
    if instance is not None:
        assert e.stat("group.last_instance") == instance
    del res
    e.close()


def test_compact_readback_after_device_trim():
    """d2h.compact=1 (key bitmap + u32 read-back) with a TOP large enough that the device trim's kept union holds more
    than 65,536 groups: the result is the trimmed union (not a bitmap of every group), equal to the oracle's trim."""
    e = GpuEngine(0, "d2h.compact=1")
    gsegs, host = _synthetic(e, 2, 2_000_000)
    q = compile_pql("SELECT SUM(d8), AVG(d8), DISTINCTCOUNTHLL(d5) FROM fact WHERE d2 < 800 GROUP BY d6, d7 TOP 20000")
    exp = O.execute_group_by_arrays(host, q, num_groups_limit=1_000_000)
    top, st = ServerQueryExecutor(e, num_groups_limit=1_000_000).group_by_result(q, gsegs, top_n=20000)
    ukeys = top.raw_keys()
    union = set()
    for fn in range(len(q["aggregations"])):
        kept = top.trimmed_groups(20000, fn)
        want = exp["keys"][_oracle_trim(exp, q, fn, 20000)]
        assert (ukeys[kept] == want).all(), q["aggregations"][fn]
        union |= set(want.tolist())
    assert len(union) >= 65536
    assert sorted(union) == ukeys.tolist()
    pos = np.searchsorted(exp["keys"], ukeys)
    c, v = top.function_values(0)
    assert (c == exp["fns"][0]["count"][pos]).all() and (v == exp["fns"][0]["sum"][pos]).all()
    regs, cards = top.hll(2)
    assert (cards == exp["fns"][2]["card"][pos]).all() and (regs == exp["fns"][2]["hll"][pos]).all()
    del top
    e.close()


def test_diagnostic_keys_rejected():
    """The product library has no wrong-result diagnostic modes: the former debug.emit / debug.ring keys are unknown
    configuration keys (PINOT_ERR_BAD_ARG)."""
    from pinot_amd import PinotGpuError
    e = GpuEngine(0)
    for key in ("debug.emit=4", "debug.ring=1"):
        with pytest.raises(PinotGpuError) as ei:
            e.set_config(key)
        assert ei.value.status == 1
    e.close()
