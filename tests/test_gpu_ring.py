"""GPU parity of the ring-partitioned group-by plan (group_ring.hip: [GB_FILTER ->] k_group_ring -> k_ring_reduce), the
plan config 4's 1M-key GROUP BY runs on: every group's count, integer sum, ordered MIN / MAX, double sum and HLL
registers bit-exact against the oracle (DictionaryBasedGroupKeyGenerator.java:195-302,
DefaultGroupByExecutor.java:70-168), including
* the HLL registers whose rank exceeds the reduce's 4-bit nibbles (the exception list);
* the filter evaluated inside k_group_ring on each quarter (a conjunction of <= 2 scan leaves: RANGE, IN / NOT IN
  tables, no filter at all) and every other filter shape through GB_FILTER's words (OR terms, sorted-index leaves, more
  leaves);
* chunk windows from a sorted-index leaf, where a few blocks get all the matching docs;
* per-segment dictionaries of the group columns (dictId -> global id remaps) and ragged segment sizes;
* skewed keys that overflow a region: the counted plan answers instead (group.ring_fallbacks), same results."""
import numpy as np
import pytest

import pinot_oracle as O
import synth
from pinot_amd import GpuEngine, ServerQueryExecutor, build_segment, compile_pql

pytestmark = pytest.mark.gpu

CONFIG_COLUMNS = [("d0", 16), ("d1", 100), ("d2", 1000), ("d3", 4096), ("d4", 10000), ("d5", 65536), ("d6", 1000),
                  ("d7", 1000), ("d8", 1 << 20), ("d9", 1000)]
BASE_SEED = 0x5EED0000
CONFIG4 = "SELECT SUM(d8), AVG(d8), DISTINCTCOUNTHLL(d5) FROM fact WHERE d2 < 800 GROUP BY d6, d7 TOP 10"


def _assert_group_arrays(res, exp, q):
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
            if np.issubdtype(np.asarray(r["sum"]).dtype, np.floating) and not (vals == r["sum"]).all():
                np.testing.assert_allclose(vals, r["sum"], rtol=1e-9)  # double sums: 1e-9 relative (north star)
            else:
                assert (vals == r["sum"]).all()
        elif f == "MIN":
            assert (vals == r["min"]).all()
        elif f == "MAX":
            assert (vals == r["max"]).all()


def _run(e, q, gsegs, host, limit=1 << 22, qfilter=None):
    """Runs q, checks it against the oracle; returns (ring-plan launches, fallbacks). qfilter: whether the ring kernel
    must have evaluated the filter itself (True) or taken GB_FILTER's words (False)."""
    exp = O.execute_group_by_arrays(host, q, num_groups_limit=limit)
    before = e.stat("group.ring_queries"), e.stat("group.ring_fallbacks"), e.stat("group.ring_qfilter_queries")
    res, st = ServerQueryExecutor(e, num_groups_limit=limit).group_by_result(q, gsegs)
    assert st.num_docs_scanned == exp["scanned"]
    _assert_group_arrays(res, exp, q)
    del res
    if qfilter is not None:
        assert (e.stat("group.ring_qfilter_queries") - before[2]) == (1 if qfilter else 0)
    return e.stat("group.ring_queries") - before[0], e.stat("group.ring_fallbacks") - before[1]


@pytest.mark.parametrize("hll,rec6", [(1, 0), (0, 0), (1, 1), (0, 1)])
def test_ring_config4_shape(hll, rec6):
    """Config 4's query and table at 2 x 2M docs: 1M keys in 977 partitions of 1024, SUM / AVG over the 20-bit d8
    (count packed beside the dictId sum), HLL over the 16-bit d5 (~120 ranks > 15 across the groups). hll: the
    scatter computes d5's HLL (register, rank) field (else the reduce hashes d5's dictId); rec6: 6-byte records (the
    10-bit local key + 20-bit d8 + 13-bit HLL field or 16-bit d5 dictId fit 48 bits)."""
    e = GpuEngine(0, "group.ring=1;group.ring_hll=%d;group.ring_rec6=%d" % (hll, rec6))
    gsegs = [e.register_synthetic("fact_%d" % s, 2_000_000, CONFIG_COLUMNS, BASE_SEED + s) for s in range(2)]
    host = [synth.make_segment("fact_%d" % s, 2_000_000, CONFIG_COLUMNS, BASE_SEED + s) for s in range(2)]
    ran, fell = _run(e, compile_pql(CONFIG4), gsegs, host, limit=1_000_000, qfilter=True)
    assert (ran, fell) == (1, 0), "ring status %d" % e.stat("group.ring_last_status")
    assert e.stat("group.ring_rec_bytes") == (6 if rec6 else 8)
    assert e.stat("group.ring_hll_slot") == hll
    # the same query with the filter as GB_FILTER's words
    e.set_config("group.ring_qfilter=0")
    ran, fell = _run(e, compile_pql(CONFIG4), gsegs, host, limit=1_000_000, qfilter=False)
    assert (ran, fell) == (1, 0)
    e.set_config("group.ring_qfilter=1")
    # the counted plan on the same engine (group.ring=0) gives the same arrays
    e.set_config("group.ring=0")
    ran, fell = _run(e, compile_pql(CONFIG4), gsegs, host, limit=1_000_000)
    assert (ran, fell) == (0, 0)
    e.close()


def test_ring_one_rank_server_answer():
    """The multi-GPU server with one rank on config 4's query at 2 x 2M docs (server.cpp): its partial runs the ring
    plan and keeps the packed HLL register sums in the partial arrays, the owner finalize reads the cardinalities from
    them, and the trimmed answer's key ids and serialized HLLs are made on the device. The untrimmed server arrays equal
    the oracle's; the trimmed DataTable's cells equal the engine path's."""
    import datatable as D
    from pinot_amd import GpuServer, ServerExecutor
    host = [synth.make_segment("fact_%d" % s, 2_000_000, CONFIG_COLUMNS, BASE_SEED + s) for s in range(2)]
    srv = GpuServer([0], "group.ring=1")
    e0 = srv.engines[0]
    gsegs = [e0.register_synthetic("fact_%d" % s, 2_000_000, CONFIG_COLUMNS, BASE_SEED + s) for s in range(2)]
    ex = ServerExecutor(srv, num_groups_limit=1_000_000)
    q = compile_pql(CONFIG4)
    exp = O.execute_group_by_arrays(host, q, num_groups_limit=1_000_000)
    before = e0.stat("group.ring_queries"), e0.stat("group.ring_fallbacks")
    res, st = ex.group_by_result(q, gsegs)
    assert (e0.stat("group.ring_queries") - before[0], e0.stat("group.ring_fallbacks") - before[1]) == (1, 0)
    assert e0.stat("group.ring_hll_slot") == 1
    _assert_group_arrays(res, exp, q)
    del res
    data, _ = ex.process_query_datatable(q, gsegs, trim=True)
    e = GpuEngine(0, "group.ring=1")
    esegs = [e.register_synthetic("fact_%d" % s, 2_000_000, CONFIG_COLUMNS, BASE_SEED + s) for s in range(2)]
    ref, _ = ServerQueryExecutor(e, num_groups_limit=1_000_000).process_query_datatable(q, esegs, trim=True)
    d, r = D.decode(data), D.decode(ref)
    assert d["cells"] == r["cells"]
    assert all(len(row[1]) == 5000 for row in d["cells"])
    e.close()
    srv.close()


_POOL = np.random.default_rng(77)
LV_POOL = _POOL.integers(-(1 << 40), 1 << 40, 3000) * 7
DV_POOL = (_POOL.standard_normal(2000) * 1e6).round(3)
H_POOL = np.arange(0, 50000, 7)


def _from_pool(rng, pool, n):
    """n values from pool, every pool value present (the partitioned plans carry dictIds: the aggregated columns'
    dictionaries must be identical on every segment)."""
    v = np.concatenate([pool, rng.choice(pool, n - pool.shape[0])])
    return v[rng.permutation(n)]


def _mixed_segment(name, n, seed, k1_vals, k2_vals, sorted_ts=False):
    rng = np.random.default_rng(seed)
    cols = {
        "k1": ("INT", rng.choice(k1_vals, n).tolist()),
        "k2": ("STRING", ["s%04d" % v for v in rng.choice(k2_vals, n)]),
        "f": ("INT", rng.integers(0, 100, n).tolist()),
        "lv": ("LONG", _from_pool(rng, LV_POOL, n).tolist()),
        "dv": ("DOUBLE", _from_pool(rng, DV_POOL, n).tolist()),
        "h": ("INT", _from_pool(rng, H_POOL, n).tolist()),
    }
    if sorted_ts:
        cols["ts"] = ("INT", (np.arange(n) // 997).tolist())
    return build_segment(name, cols)


@pytest.mark.parametrize("text", [
    "SELECT MIN(dv), MAX(lv) FROM t WHERE f < 70 GROUP BY k1, k2",
    "SELECT SUM(dv), COUNT(*) FROM t WHERE f >= 10 GROUP BY k2, k1",
    "SELECT SUM(lv), DISTINCTCOUNTHLL(h) FROM t WHERE f <> 5 GROUP BY k1, k2",
    "SELECT DISTINCTCOUNTHLL(h), COUNT(*) FROM t WHERE f > 3 GROUP BY k2, k1",
    "SELECT DISTINCTCOUNTHLL(h), MAX(h) FROM t GROUP BY k1, k2",
])
def test_ring_remap_ragged_kinds(text):
    """Three segments of different sizes whose group dictionaries differ (remapped to the union key space), every
    accumulator kind the ring reduce folds: ordered MIN / MAX, double and int64 sums, counts, HLL."""
    segs = [_mixed_segment("r0", 70_001, 1, np.arange(0, 90), np.arange(0, 80)),
            _mixed_segment("r1", 33_333, 2, np.arange(20, 120), np.arange(10, 95)),
            _mixed_segment("r2", 120_017, 3, np.arange(5, 100), np.arange(0, 90))]
    e = GpuEngine(0, "group.mode=partition;group.ring=1")
    gsegs = [e.register(s) for s in segs]
    ran, fell = _run(e, compile_pql(text), gsegs, segs)
    assert (ran, fell) == (1, 0)
    e.close()


def test_ring_sorted_window_busiest_block():
    """A sorted-index leaf bounds each segment's chunk window: the blocks split the windows' chunks only (the sorted
    leaf's ranges are not a quarter-form leaf: GB_FILTER's words)."""
    segs = [_mixed_segment("w0", 400_000, 11, np.arange(0, 100), np.arange(0, 100), sorted_ts=True),
            _mixed_segment("w1", 250_000, 12, np.arange(0, 100), np.arange(0, 100), sorted_ts=True)]
    e = GpuEngine(0, "group.mode=partition;group.ring=1")
    gsegs = [e.register(s) for s in segs]
    q = compile_pql("SELECT SUM(lv), MAX(dv) FROM t WHERE ts BETWEEN 40 AND 90 AND f < 95 GROUP BY k1, k2")
    ran, fell = _run(e, q, gsegs, segs, qfilter=False)
    assert (ran, fell) == (1, 0)
    e.close()


@pytest.mark.parametrize("qfilter", [1, 0])
@pytest.mark.parametrize("text,qf", [
    ("SELECT SUM(lv), COUNT(*) FROM t GROUP BY k1, k2", True),                              # no filter
    ("SELECT SUM(lv), MAX(dv) FROM t WHERE k1 IN (3, 5, 7, 60, 61) GROUP BY k1, k2", True),  # IN: membership LUT
    ("SELECT SUM(lv) FROM t WHERE f NOT IN (1, 2, 3) AND h > 20000 GROUP BY k2, k1", True),  # two leaves, negated
    ("SELECT SUM(lv) FROM t WHERE f < 30 AND h > 20000 AND k1 <> 4 GROUP BY k1, k2", None),  # three leaves
    ("SELECT SUM(lv), DISTINCTCOUNTHLL(h) FROM t WHERE f < 10 OR h < 9000 GROUP BY k1, k2", None),  # OR term
])
def test_ring_filter_forms(text, qf, qfilter):
    """The filter shapes the ring kernel evaluates on each quarter (the planner may also hand it a `pre` bitset of
    the terms it does not fuse: qf None), and every shape through GB_FILTER's words (group.ring_qfilter=0), over ragged
    segments whose last chunk is partial (tail docs masked)."""
    segs = [_mixed_segment("q0", 90_001, 21, np.arange(0, 90), np.arange(0, 80)),
            _mixed_segment("q1", 41_000, 22, np.arange(10, 100), np.arange(5, 85))]
    e = GpuEngine(0, "group.mode=partition;group.ring=1;group.ring_qfilter=%d" % qfilter)
    gsegs = [e.register(s) for s in segs]
    ran, fell = _run(e, compile_pql(text), gsegs, segs, qfilter=(qf if qfilter else False))
    assert (ran, fell) == (1, 0)
    e.close()


def test_ring_skewed_keys_fall_back():
    """90 % of the docs on one key: its partition's records overflow every block's region; the query is re-answered
    on the counted plan with identical results."""
    n = 600_000
    rng = np.random.default_rng(5)
    k1 = np.where(rng.random(n) < 0.9, 3, rng.integers(0, 100, n))
    k2 = np.where(k1 == 3, 7, rng.integers(0, 100, n))
    seg = build_segment("skew", {"k1": ("INT", k1.tolist()), "k2": ("INT", k2.tolist()),
                                 "x": ("INT", rng.integers(0, 1000, n).tolist()),
                                 "f": ("INT", rng.integers(0, 10, n).tolist())})
    e = GpuEngine(0, "group.mode=partition;group.ring=1")
    g = e.register(seg)
    q = compile_pql("SELECT SUM(x), MAX(x) FROM t WHERE f < 8 GROUP BY k1, k2")
    ran, fell = _run(e, q, [g], [seg])
    assert (ran, fell) == (1, 1)
    e.close()


def test_ring_sparse_query_after_wide_records():
    """A sparse query after a dense one on the same engine: the record buffer's slots beyond each region's streamed
    range still hold the first query's records (another field layout), and the reduce's dictionary / HLL-LUT gathers
    must not index by them (non-affine LONG dictionary: the HLL reads its LUT)."""
    segs = [_mixed_segment("s0", 200_000, 31, np.arange(0, 100), np.arange(0, 100)),
            _mixed_segment("s1", 150_000, 32, np.arange(0, 100), np.arange(0, 100))]
    e = GpuEngine(0, "group.mode=partition;group.ring=1")
    gsegs = [e.register(s) for s in segs]
    for text in ("SELECT SUM(dv), MAX(lv) FROM t GROUP BY k1, k2",
                 "SELECT DISTINCTCOUNTHLL(lv), SUM(lv) FROM t WHERE f < 1 AND h > 30000 GROUP BY k2, k1",
                 "SELECT DISTINCTCOUNTHLL(lv) FROM t WHERE f = 3 OR h < 70 GROUP BY k1, k2"):
        ran, fell = _run(e, compile_pql(text), gsegs, segs)
        assert (ran, fell) == (1, 0)
    e.close()


def test_ring_record_forms():
    """The record width (group.ring_rec6=1) and the flushers' HLL field by shape (1M keys: 10-bit local keys): two 20-bit aggregated
    columns beside the local key exceed 48 bits (8-byte records), an HLL over an affine dictionary with values >= 2^32 keeps its dictId (the reduce
    hashes the 64-bit value), an HLL beside a SUM of the same column keeps its dictId."""
    n = 600_000
    rng = np.random.default_rng(41)
    cols = {"k1": ("INT", rng.integers(0, 1000, n).tolist()), "k2": ("INT", rng.integers(0, 1000, n).tolist()),
            "x": ("INT", rng.permutation(1 << 20)[:n].tolist()),   # 600,000 distinct values: 20-bit dictIds
            "y": ("INT", rng.permutation(1 << 20)[:n].tolist()),
            "big": ("LONG", ((1 << 33) + 5 * rng.integers(0, 4000, n)).tolist()),
            "h": ("INT", (3 * rng.integers(0, 9000, n)).tolist()),
            "f": ("INT", rng.integers(0, 10, n).tolist())}
    segs = [build_segment("rf0", cols)]
    e = GpuEngine(0, "group.mode=partition;group.ring=1;group.ring_rec6=1")  # 6-byte records where they fit
    gsegs = [e.register(s) for s in segs]
    for text, rb, hs in (("SELECT SUM(x), MAX(y) FROM t WHERE f < 8 GROUP BY k1, k2", 8, 0),
                         ("SELECT SUM(x), DISTINCTCOUNTHLL(h) FROM t WHERE f < 8 GROUP BY k1, k2", 6, 1),
                         ("SELECT DISTINCTCOUNTHLL(big), COUNT(*) FROM t WHERE f < 9 GROUP BY k1, k2", 6, 0),
                         ("SELECT DISTINCTCOUNTHLL(h), SUM(h) FROM t GROUP BY k2, k1", 6, 0)):
        ran, fell = _run(e, compile_pql(text), gsegs, segs)
        assert (ran, fell) == (1, 0), text
        assert (e.stat("group.ring_rec_bytes"), e.stat("group.ring_hll_slot")) == (rb, hs), text
    e.close()
