"""Raw (no-dictionary) numeric columns on the GPU: registered with PINOT_ENCODING_RAW (the values themselves) and
transcoded once to the dictionary form. Filters are checked against the oracle's raw-value evaluators
(pinot_oracle.raw_leaf_mask: RawValueBased*PredicateEvaluator semantics), aggregations and group-by against the
oracle over the same values, and a raw registration against the dictionary registration of the same data."""
import numpy as np
import pytest

import pinot_oracle as O
from pinot_amd import GpuEngine, ServerQueryExecutor, build_segment, compile_pql
from test_gpu_parity import _assert_same, _random_aggs, _random_columns, _random_tree

pytestmark = pytest.mark.gpu
RAW = ("big", "lng", "dbl", "flt", "i0", "s")  # "s": a var-byte STRING column


@pytest.fixture(scope="module")
def engine():
    e = GpuEngine(0)
    yield e
    e.close()


def _norm(v):
    if hasattr(v, "registers"):  # HyperLogLog
        return ("hll", bytes(v.registers), v.cardinality())
    if hasattr(v, "count") and hasattr(v, "sum"):  # AvgPair
        return ("avg", v.sum, v.count)
    if isinstance(v, tuple) and len(v) == 2:  # the oracle's AvgPair (sum, count)
        return ("avg", v[0], v[1])
    return v


def _segments(rng, n, k):
    out = []
    for i in range(k):
        cols, inv = _random_columns(rng, n)
        out.append(build_segment("raw%d" % i, cols, inverted_columns=tuple(x for x in inv if x not in RAW),
                                 raw_columns=RAW))
    return out


@pytest.mark.parametrize("seed", range(3))
def test_raw_filter_bitsets(engine, seed):
    rng = np.random.default_rng(700 + seed)
    n = int(rng.choice([1, 65, 1000, 30001]))
    seg = _segments(rng, n, 1)[0]
    g = engine.register(seg)
    for _ in range(16):
        tree = _random_tree(rng, seg)
        exp = O.filter_mask(seg, tree)
        bits, cnt = engine.filter(g, tree)
        got = np.unpackbits(bits.view(np.uint8), bitorder="little")[:n].astype(bool)
        assert cnt == int(exp.sum()), tree
        assert (got == exp).all(), tree
    g.release()


@pytest.mark.parametrize("seed", range(3))
def test_raw_aggregations_and_group_by(engine, seed):
    rng = np.random.default_rng(800 + seed)
    n = int(rng.choice([64, 999, 20000]))
    segs = _segments(rng, n, int(rng.integers(1, 3)))
    gsegs = [engine.register(s) for s in segs]
    ex = ServerQueryExecutor(engine)
    for it in range(10):
        q = {"aggregations": _random_aggs(rng), "filter": _random_tree(rng, segs[0]) if rng.random() < 0.8 else None,
             "group_by": {"columns": list(rng.choice(["i0", "big", "i1", "s"], size=int(rng.integers(1, 3)),
                                                     replace=False)), "top_n": 10} if it % 2 else None}
        got, st = ex.process_query(q, gsegs, trim=False)
        exp, scanned = O.execute_server(segs, q)
        assert st.num_docs_scanned == scanned
        if q["group_by"]:
            assert set(got) == set(exp)
            pairs = [(got[k], exp[k]) for k in exp]
        else:
            pairs = [(got, exp)]
        for gv_row, ev_row in pairs:
            for a, gv, ev in zip(q["aggregations"], gv_row, ev_row):
                _assert_same(a["function"], gv, ev, a["column"] not in ("dbl", "flt", "lng"))
    for g in gsegs:
        g.release()


def test_raw_matches_dictionary_registration(engine):
    rng = np.random.default_rng(900)
    n = 5000
    cols, _ = _random_columns(rng, n)
    raw = build_segment("raw", cols, raw_columns=RAW)
    dic = build_segment("dic", cols)
    gr, gd = engine.register(raw), engine.register(dic)
    ex = ServerQueryExecutor(engine)
    for text in ("SELECT COUNT(*), SUM(big), MIN(lng), MAX(dbl), AVG(flt), DISTINCTCOUNTHLL(big) FROM t "
                 "WHERE big > 0 AND lng BETWEEN -1000000000 AND 1000000000000",
                 "SELECT SUM(lng), MAX(big) FROM t WHERE i0 IN (%s) OR dbl < 0" % ", ".join(
                     str(int(x)) for x in raw.columns["i0"].dict_values()[:3]),
                 "SELECT COUNT(*), SUM(i1) FROM t GROUP BY i0, s"):
        q = compile_pql(text)
        a, _ = ex.process_query(q, [gr], trim=False)
        b, _ = ex.process_query(q, [gd], trim=False)
        if q.get("group_by"):
            assert set(a) == set(b), text
            pairs = [(a[k], b[k]) for k in a]
        else:
            pairs = [(a, b)]
        for x, y in pairs:
            assert [_norm(v) for v in x] == [_norm(v) for v in y], text
    # MIN / MAX without a filter: the dictionary plan reads a dictionary column's ends (no scan); a raw column is
    # scanned (InstancePlanMakerImplV2.isFitForDictionaryBasedPlan needs a dictionary)
    q = compile_pql("SELECT MIN(big), MAX(lng) FROM t")
    a, sa = ex.process_query(q, [gr])
    b, sb = ex.process_query(q, [gd])
    assert a == b and a[0] == float(min(cols["big"][1])) and a[1] == float(max(cols["lng"][1]))
    assert sb.num_entries_scanned_post_filter == 0 and sa.num_entries_scanned_post_filter == 2 * n
    gr.release()
    gd.release()


def test_var_byte_fixture_on_gpu(engine, tmp_path):
    """The reference's data/varByteStrings.v1 as a raw STRING column's forward index (1009 docs cycling "abcde",
    "fgh", "ijklmn", "12345"): loaded from a segment directory, grouped, filtered."""
    import os
    from segdir_writer import write_segment_dir
    fixture = open(os.path.join(os.path.dirname(__file__), "golden", "var_byte_strings.v1"), "rb").read()
    expected = ["abcde", "fgh", "ijklmn", "12345"]
    vals = [expected[i % 4] for i in range(1009)]
    seg = build_segment("vb", {"s": ("STRING", np.array(vals, dtype=object)),
                               "i": ("INT", np.arange(1009, dtype=np.int32))}, raw_columns=("s",))
    seg.columns["s"].raw_file = fixture
    g = engine.load(write_segment_dir(seg, str(tmp_path / "vb"), version="v3"))
    ex = ServerQueryExecutor(engine)
    got, _ = ex.process_query(compile_pql("SELECT COUNT(*), SUM(i) FROM t GROUP BY s"), [g], trim=False)
    assert got == {v: [len(range(k, 1009, 4)), float(sum(range(k, 1009, 4)))] for k, v in enumerate(expected)}
    got, st = ex.process_query(compile_pql("SELECT COUNT(*) FROM t WHERE s BETWEEN 'abcde' AND 'fgh'"), [g])
    assert got == [505] and st.num_docs_scanned == 505
    g.release()


def test_fixed_byte_fixture_on_gpu(engine, tmp_path):
    """The reference's data/fixedByteSVRDoubles.v1 (version 1, Snappy; doc i = (double) i for 10,009 docs) as a raw
    DOUBLE column loaded from a segment directory: every doc's value through a range filter, aggregations and a
    group-by, against the oracle over the same values."""
    import os
    from segdir_writer import write_segment_dir
    fixture = open(os.path.join(os.path.dirname(__file__), "golden", "fixed_byte_svr_doubles.v1"), "rb").read()
    n = 10009
    cols = {"d": ("DOUBLE", np.arange(n, dtype=np.float64)), "k": ("INT", (np.arange(n) % 7).astype(np.int32))}
    seg = build_segment("fb", cols, raw_columns=("d",))
    seg.columns["d"].raw_file = fixture
    g = engine.load(write_segment_dir(seg, str(tmp_path / "fb"), version="v3"))
    ex = ServerQueryExecutor(engine)
    for text in ("SELECT COUNT(*), SUM(d), MIN(d), MAX(d), AVG(d) FROM t",
                 "SELECT COUNT(*), SUM(d), MAX(d) FROM t WHERE d BETWEEN 100.5 AND 5000",
                 "SELECT COUNT(*), MIN(d) FROM t WHERE d > 9000 OR d < 3",
                 "SELECT SUM(d), MAX(d) FROM t WHERE d >= 17 GROUP BY k"):
        q = compile_pql(text)
        got, st = ex.process_query(q, [g], trim=False)
        exp, scanned = O.execute_server([seg], q)
        assert st.num_docs_scanned == scanned, text
        if isinstance(exp, dict):
            assert {k: [_norm(v) for v in x] for k, x in got.items()} == \
                   {k: [_norm(v) for v in x] for k, x in exp.items()}, text
        else:
            assert [_norm(v) for v in got] == [_norm(v) for v in exp], text
    # every doc's value: d == i exactly (a per-doc equality filter over a sample of docs)
    for i in (0, 1, 4095, 4096, 8191, 10008):
        got, _ = ex.process_query(compile_pql("SELECT COUNT(*), SUM(d) FROM t WHERE d = %d" % i), [g])
        assert got == [1, float(i)], i
    g.release()


def test_raw_fp_primitive_comparisons(engine):
    """Raw FLOAT / DOUBLE predicates compare primitives (RawValueBased evaluators): -0.0 == 0.0, NaN (literal or
    value) never compares true — unlike the transcoded dictionary's Double.compare order. Checked against the
    oracle's raw-value evaluators (numpy IEEE comparisons)."""
    import pinot_oracle as O
    vals = [float("nan"), -0.0, 0.0, 1.5, -2.25, 0.0, -0.0, float("nan"), 7.0, -1.0] * 50
    seg = build_segment("fp", {"d": ("DOUBLE", vals), "f": ("FLOAT", np.array(vals, dtype=np.float32)),
                               "i": ("INT", np.arange(len(vals), dtype=np.int32))}, raw_columns=("d", "f"))
    g = engine.register(seg)
    lits = ["NaN", "0.0", "-0.0", "1.5", "-1.0"]
    for col in ("d", "f"):
        trees = []
        for l in lits:
            trees += [{"operator": op, "column": col, "values": [l]} for op in ("EQUALITY", "NOT")]
            trees += [{"operator": op, "column": col, "values": [l + "\t\t7.0"]} for op in ("IN", "NOT_IN")]
            trees += [{"operator": "RANGE", "column": col, "values": [r]} for r in (
                "[%s\t\t*)" % l, "(%s\t\t*)" % l, "(*\t\t%s]" % l, "(*\t\t%s)" % l, "[-0.0\t\t%s]" % l)]
        trees.append({"operator": "RANGE", "column": col, "values": ["(*\t\t*)"]})
        for tree in trees:
            exp = O.filter_mask(seg, tree)
            bits, cnt = engine.filter(g, tree)
            got = np.unpackbits(bits.view(np.uint8), bitorder="little")[:len(vals)].astype(bool)
            assert cnt == int(exp.sum()) and (got == exp).all(), tree
    g.release()


def test_large_raw_columns_threaded_transcode(engine):
    """3 M-doc raw columns: registration transcodes them on several host threads (segment_parse.cpp); the result
    answers exactly as the dictionary registration of the same values."""
    rng = np.random.default_rng(950)
    n = 3_000_000
    words = np.array(["w%03d" % i for i in range(300)], dtype=object)
    cols = {"big": ("INT", rng.integers(-2 ** 31, 2 ** 31, n).astype(np.int32)),
            "lng": ("LONG", rng.integers(0, 1000, n).astype(np.int64) * 1_000_003 - 7),
            "dbl": ("DOUBLE", np.where(rng.random(n) < 0.01, -0.0, np.round(rng.normal(0, 50, n), 2))),
            "s": ("STRING", words[rng.integers(0, words.shape[0], n)]),
            "k": ("INT", rng.integers(0, 40, n).astype(np.int32))}
    raw = build_segment("rawbig", cols, raw_columns=("big", "lng", "dbl", "s"), allow_sorted=False)
    dic = build_segment("dicbig", cols, allow_sorted=False)
    gr, gd = engine.register(raw), engine.register(dic)
    try:
        ex = ServerQueryExecutor(engine)
        for text in ("SELECT COUNT(*), SUM(lng), MIN(big), MAX(dbl), DISTINCTCOUNTHLL(s) FROM t WHERE big > 0 AND "
                     "lng BETWEEN 1000003 AND 500000000 AND s IN ('w001', 'w150', 'w299', 'zz')",
                     "SELECT SUM(dbl), MAX(lng), COUNT(*) FROM t WHERE s >= 'w100' OR k = 3",
                     "SELECT COUNT(*), SUM(lng), MIN(dbl) FROM t WHERE big < 0 GROUP BY s, k"):
            q = compile_pql(text)
            a, sa = ex.process_query(q, [gr], trim=False)
            b, sb = ex.process_query(q, [gd], trim=False)
            assert sa.num_docs_scanned == sb.num_docs_scanned, text
            if q.get("group_by"):
                assert set(a) == set(b), text
                pairs = [(a[k], b[k]) for k in a]
            else:
                pairs = [(a, b)]
            for x, y in pairs:
                assert [_norm(v) for v in x] == [_norm(v) for v in y], text
    finally:
        gr.release()
        gd.release()


@pytest.mark.parametrize("n", [1, 2, 777, 65537, 2_000_000])
def test_device_transcode_matches_host(engine, n):
    """Registration's device transcode of raw numeric columns (transcode.hip: radix sort of value keys, distinct count,
    MSB-first packing) gives the host path's bytes exactly: dictionary, cardinality, bit width, forward index — for
    INT / LONG / FLOAT / DOUBLE with negative values, -0.0 beside 0.0, NaN and infinities, single-value and
    all-distinct columns."""
    rng = np.random.default_rng(990 + n)
    dbl = np.round(rng.normal(0, 1e3, n), 1)
    dbl[rng.random(n) < 0.01] = -0.0
    dbl[rng.random(n) < 0.005] = np.nan
    dbl[rng.random(n) < 0.005] = np.inf
    flt = rng.normal(0, 10, n).astype(np.float32)
    flt[rng.random(n) < 0.01] = np.float32(-np.inf)
    cols = {"i": ("INT", rng.integers(-2 ** 31, 2 ** 31, n).astype(np.int32)),
            "l": ("LONG", rng.integers(-5, 5, n).astype(np.int64) * 10 ** 15),
            "f": ("FLOAT", flt),
            "d": ("DOUBLE", dbl),
            "one": ("INT", np.full(n, 7, np.int32)),
            "all": ("LONG", np.arange(n, dtype=np.int64) * 3 - n)}
    seg = build_segment("tc", cols, raw_columns=tuple(cols), allow_sorted=False)
    before = engine.stat("raw.device_columns")
    for c in cols:
        dev = engine.transcode_raw(seg, c, on_device=True)
        host = engine.transcode_raw(seg, c, on_device=False)
        assert dev[:2] == host[:2], c
        assert dev[2] == host[2], c
        assert dev[3] == host[3], c
    assert engine.stat("raw.device_columns") == before + 2 * len(cols)  # the wrapper's length call transcodes too
