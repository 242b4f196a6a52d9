"""GPU parity: the HIP path (through the C-ABI) against the reference's known answers and the CPU oracle.

Integer results (doc sets, counts, integer sums, dictIds, group keys, HLL registers) must be bit-exact;
double sums of floating-point columns within 1e-9 relative (BASELINE.json north_star)."""
import math

import numpy as np
import pytest

import pinot_oracle as O
from pinot_amd import (AvgPair, BrokerReduce, GpuEngine, HyperLogLog, ServerQueryExecutor, build_segment,
                       compile_pql)
from pinot_amd.segment import build_column, Segment

pytestmark = pytest.mark.gpu
REL = 1e-9
# engine configurations: default (fused single-launch path, pipelined whole-chunk staging where a chunk
# fits), forced scan / forced index leaves, the stepwise fused kernel, the non-temporal DMA policy, and
# the unfused per-segment launch sequence
ENGINE_MODES = ("", "filter.force=scan", "filter.force=index", "exec.nt=0", "exec.pipe=1", "exec.nt=0;exec.pipe=1",
                "exec.fused=0")


@pytest.fixture(scope="module", params=ENGINE_MODES)
def engine(request):
    e = GpuEngine(0, request.param or None)
    e.mode_cfg = request.param
    yield e
    e.close()


@pytest.fixture(scope="module")
def sv_gpu(engine, sv_segment):
    return engine.register(sv_segment)


def _close(a, b):
    if isinstance(a, float) and isinstance(b, float) and (math.isinf(a) or math.isinf(b)):
        return a == b
    return abs(a - b) <= REL * max(1.0, abs(a), abs(b))


def _assert_same(f, got, exp, exact=True):
    f = f.upper()
    if f == "COUNT":
        assert got == exp
    elif f == "AVG":
        s, c = (exp.sum, exp.count) if isinstance(exp, AvgPair) else exp
        assert got.count == c
        assert (got.sum == s) if exact else _close(got.sum, s)
    elif f == "DISTINCTCOUNTHLL":
        assert got.cardinality() == exp.cardinality()
        assert (np.asarray(got.registers, dtype=np.int64) == np.asarray(exp.reg, dtype=np.int64)).all()
    else:
        assert (got == exp) if exact else _close(got, exp)


# ------------------------------------------------------------------ reference known answers
def test_kat_inner_aggregation(engine, sv_gpu, kats):
    k = kats["inner_aggregation"]
    ex = ServerQueryExecutor(engine)
    for case, where in (("unfiltered", ""), ("filtered", kats["filter"])):
        res, st = ex.process_query(k["query"] + where, [sv_gpu])
        exp = k[case]["result"]
        assert [res[0], int(res[1]), int(res[2]), int(res[3]), int(res[4].sum), res[4].count] == exp
        assert st.num_docs_scanned == k[case]["stats"][0]
        assert st.num_entries_scanned_post_filter == k[case]["stats"][2]
        assert st.num_total_raw_docs == k[case]["stats"][3]


@pytest.mark.parametrize("idx", range(8))
def test_kat_inner_group_by(engine, sv_gpu, kats, idx):
    k = kats["inner_group_by"]
    case = k["cases"][idx]
    if case["holder"] in ("LONG_MAP_BASED", "ARRAY_MAP_BASED") and engine.mode_cfg == "exec.fused=0":
        pytest.skip("hashed key spaces (LONG_MAP / ARRAY_MAP) run on the fused group-by only")
    text = "SELECT" + k["aggregation"] + " FROM testTable" + (kats["filter"] if case["filtered"] else "") + \
        case["group_by"]
    res, st = ServerQueryExecutor(engine).process_query(text, [sv_gpu], trim=False)
    v = res[case["key"]]
    assert [v[0], int(v[1]), int(v[2]), int(v[3]), int(v[4].sum), v[4].count] == case["result"]
    assert st.num_docs_scanned == case["stats"][0]
    assert st.num_entries_scanned_post_filter == case["stats"][2]


def test_kat_inter_segment(engine, sv_gpu, kats):
    k = kats["inter_segment"]
    ex = ServerQueryExecutor(engine)
    for case in k["cases"]:
        for variant, where, gb in (("unfiltered", "", ""), ("filtered", kats["filter"], ""),
                                   ("unfiltered_group_by", "", k["group_by"]),
                                   ("filtered_group_by", kats["filter"], k["group_by"])):
            q = compile_pql(case["query"] + where + gb)
            server, st = ex.process_query(q, [sv_gpu, sv_gpu])
            got = BrokerReduce.reduce(q, [server, server])
            if q.get("group_by"):
                got = [g[0][1] for g in got]
            assert got == case[variant], (case["query"], variant)
            # 2 servers x 2 segments: the broker sums the servers' statistics. numEntriesScannedInFilter is the
            # iterator-protocol count (SVScanDocIdIterator.java:77-131) and is not modelled.
            stats = [2 * st.num_docs_scanned, 2 * st.num_entries_scanned_post_filter, 2 * st.num_total_raw_docs]
            exp = case["stats"][variant]
            assert stats == [exp[0], exp[2], exp[3]], (case["query"], variant, stats)


def test_kat_query_executor(engine, simple_segments, kats):
    segs = [engine.register(s) for s in simple_segments]
    ex = ServerQueryExecutor(engine)
    for case in kats["query_executor"]["cases"]:
        res, _ = ex.process_query(case["query"], segs)
        assert float(res[0]) == float(case["expected"])


def _membership_segment(lists, n=40, inverted=True):
    cols = {"k%d" % i: ("INT", [1 if d in set(lst) else 0 for d in range(n)]) for i, lst in enumerate(lists)}
    return build_segment("fake", cols, inverted_columns=tuple(cols) if inverted else ())


def _tree_to_filter(tree, lists):
    op, kids = tree
    out = []
    for kid in kids:
        if isinstance(kid[0], str):
            out.append(_tree_to_filter(kid, lists))
        else:
            idx = lists.index(kid)
            out.append({"operator": "EQUALITY", "column": "k%d" % idx, "values": ["1"]})
    return {"operator": op, "children": out}


def _flatten_lists(tree, acc):
    for kid in tree[1]:
        if isinstance(kid[0], str):
            _flatten_lists(kid, acc)
        elif kid not in acc:
            acc.append(kid)
    return acc


@pytest.mark.parametrize("inverted", [True, False])
def test_kat_and_or_filter_operators(engine, kats, inverted):
    for case in kats["and_filter_operator"]["cases"]:
        lists = _flatten_lists(case["tree"], [])
        seg = _membership_segment(lists, inverted=inverted)
        g = engine.register(seg)
        bits, cnt = engine.filter(g, _tree_to_filter(case["tree"], lists))
        docs = np.nonzero(np.unpackbits(bits.view(np.uint8), bitorder="little")[:seg.num_docs])[0].tolist()
        assert docs == case["expected"], case["_line"]
        assert cnt == len(case["expected"])
        g.release()


# ------------------------------------------------------------------ randomized parity vs the oracle
def _random_segment(rng, n, name="seg", n_int=5, with_strings=True, sorted_col=True, double_col=True):
    cols, inv = _random_columns(rng, n, n_int, with_strings, sorted_col, double_col)
    return build_segment(name, cols, inverted_columns=tuple(inv))


def _random_columns(rng, n, n_int=5, with_strings=True, sorted_col=True, double_col=True):
    cols = {}
    inv = []
    for i in range(n_int):
        card = int(rng.choice([1, 2, 3, 17, 64, 65, 100, 1000, 5000]))
        card = max(1, min(card, n))
        vals = rng.integers(-50000, 50000, size=card)
        vals = np.unique(vals)
        pick = rng.integers(0, vals.shape[0], size=n)
        cols["i%d" % i] = ("INT", vals[pick].astype(np.int64).tolist())
        if rng.random() < 0.5:
            inv.append("i%d" % i)
    cols["big"] = ("INT", rng.integers(-2 ** 31, 2 ** 31, size=n).tolist())
    cols["lng"] = ("LONG", (rng.integers(-2 ** 40, 2 ** 40, size=n)).tolist())
    if double_col:
        cols["dbl"] = ("DOUBLE", np.round(rng.normal(0, 1000, size=n), 3).tolist())
        cols["flt"] = ("FLOAT", np.float32(rng.normal(0, 10, size=n)).astype(np.float64).tolist())
    if with_strings:
        words = ["a", "bb", "ccc", "P", "t", "zz", "Hello", "wé"]
        cols["s"] = ("STRING", [words[i] for i in rng.integers(0, len(words), size=n)])
        inv.append("s")
    if sorted_col:
        cols["srt"] = ("INT", np.sort(rng.integers(0, max(2, n // 50), size=n)).tolist())
    return cols, inv


def _random_leaf(rng, seg):
    names = [c for c in seg.columns]
    c = seg.column(names[int(rng.integers(0, len(names)))])
    vals = c.dict_values()
    pick = lambda: vals[int(rng.integers(0, len(vals)))]  # noqa: E731
    def lit(v):
        if c.data_type in ("INT", "LONG"):
            return str(int(v))
        if c.data_type in ("FLOAT", "DOUBLE"):
            return repr(float(v))
        return str(v)
    kind = rng.choice(["EQUALITY", "NOT", "IN", "NOT_IN", "RANGE", "RANGE", "EQ_MISSING"])
    if kind == "EQ_MISSING":
        v = "zzzz_missing" if c.data_type == "STRING" else ("123456789" if c.data_type in ("INT", "LONG") else "1.25")
        return {"operator": "EQUALITY", "column": c.name, "values": [v]}
    if kind in ("EQUALITY", "NOT"):
        return {"operator": kind, "column": c.name, "values": [lit(pick())]}
    if kind in ("IN", "NOT_IN"):
        k = int(rng.integers(1, 6))
        return {"operator": kind, "column": c.name, "values": ["\t\t".join(lit(pick()) for _ in range(k))]}
    a, b = sorted([pick(), pick()], key=lambda x: x.encode() if isinstance(x, str) else x)
    lo = "*" if rng.random() < 0.2 else lit(a)
    hi = "*" if rng.random() < 0.2 else lit(b)
    return {"operator": "RANGE", "column": c.name,
            "values": ["%s%s\t\t%s%s" % (rng.choice(["(", "["]), lo, hi, rng.choice([")", "]"]))]}


def _random_tree(rng, seg, depth=0):
    if depth >= 2 or rng.random() < 0.4:
        return _random_leaf(rng, seg)
    k = int(rng.integers(2, 4))
    return {"operator": rng.choice(["AND", "OR"]), "children": [_random_tree(rng, seg, depth + 1) for _ in range(k)]}


def _random_aggs(rng):
    pool = [("COUNT", "*"), ("SUM", "big"), ("SUM", "i0"), ("MIN", "i1"), ("MAX", "big"), ("AVG", "i2"),
            ("SUM", "lng"), ("MAX", "lng"), ("SUM", "dbl"), ("MIN", "dbl"), ("AVG", "flt"),
            ("DISTINCTCOUNTHLL", "big"), ("DISTINCTCOUNTHLL", "s"), ("DISTINCTCOUNTHLL", "dbl"), ("SUM", "srt")]
    idx = rng.choice(len(pool), size=int(rng.integers(1, 6)), replace=False)
    return [{"function": pool[i][0], "column": pool[i][1]} for i in idx]


@pytest.mark.parametrize("seed", range(6))
def test_random_filter_bitsets(engine, seed):
    rng = np.random.default_rng(100 + seed)
    n = int(rng.choice([1, 63, 64, 65, 1000, 70001]))
    seg = _random_segment(rng, n)
    g = engine.register(seg)
    for _ in range(12):
        tree = _random_tree(rng, seg)
        exp = O.filter_mask(seg, tree)
        bits, cnt = engine.filter(g, tree)
        got = np.unpackbits(bits.view(np.uint8), bitorder="little")[:n].astype(bool)
        assert cnt == int(exp.sum())
        assert (got == exp).all()
        if bits.shape[0] and n % 64:
            assert int(bits[-1]) >> (n % 64) == 0  # tail bits beyond numDocs stay clear
    g.release()


def _small_leaf(rng, seg):
    """A leaf the fused kernel evaluates in registers: EQ / NOT / IN / NOT_IN of a few literals (scan, sorted or
    bitmap leaf by the planner's cost model) or a RANGE."""
    while True:
        leaf = _random_leaf(rng, seg)
        if leaf["operator"] != "RANGE" or leaf["column"] not in ("s",) and not leaf["column"].startswith("i"):
            return leaf


def _deep_tree(rng, seg, depth=0, max_depth=4):
    """AND / OR levels alternating down to max_depth (every level nests: FilterOperatorUtils builds one operator per
    level, FilterOperatorUtils.java:74-122)."""
    if depth >= max_depth or (depth >= 2 and rng.random() < 0.3):
        return _small_leaf(rng, seg)
    op = ("AND", "OR")[(depth + int(rng.integers(0, 2)) * (depth == 0)) % 2]
    k = int(rng.integers(2, 4))
    return {"operator": op, "children": [_deep_tree(rng, seg, depth + 1, max_depth) for _ in range(k)]}


@pytest.mark.parametrize("seed", range(4))
def test_deep_filter_trees_in_registers(seed):
    """Filter trees nested four levels deep (alternating AND / OR) run inside the fused kernel's register program
    (postfix terms over its register stack): no segment's filter goes through the dense-bitset launch sequence
    (exec.last_pre_segments == 0), and the aggregations equal the oracle's."""
    rng = np.random.default_rng(2100 + seed)
    n = int(rng.choice([1000, 70001]))
    segs = [_random_segment(rng, n, name="d%d" % i) for i in range(2)]
    e = GpuEngine(0)
    gsegs = [e.register(s) for s in segs]
    ex = ServerQueryExecutor(e)
    for _ in range(10):
        tree = _deep_tree(rng, segs[0])
        q = {"aggregations": [{"function": "COUNT", "column": "*"}, {"function": "SUM", "column": "big"},
                              {"function": "MAX", "column": "lng"}], "filter": tree, "group_by": None}
        got, st = ex.process_query(q, gsegs)
        exp, scanned = O.execute_server(segs, q)
        assert st.num_docs_scanned == scanned, tree
        for a, gv, ev in zip(q["aggregations"], got, exp):
            _assert_same(a["function"], gv, ev, True)
        assert e.stat("exec.last_pre_segments") == 0, tree
        # the same tree through the filter API (the dense-bitset launch path) agrees doc for doc
        bits, cnt = e.filter(gsegs[0], tree)
        m = O.filter_mask(segs[0], tree)
        assert cnt == int(m.sum())
    e.close()


def test_wide_bitmap_leaf_in_registers():
    """A bitmap-indexed leaf over 200 dictIds (a config-3 variant: b4 IN (200 values)) is evaluated from the roaring
    containers inside the fused kernel, one launch with no `pre` bitset, equal to the oracle and to the forced-scan
    plan."""
    rng = np.random.default_rng(2200)
    n = 300_000
    cols = {"s0": ("INT", np.sort(rng.integers(0, 400, n)).tolist()),
            "b4": ("INT", rng.integers(0, 1000, n).tolist()),
            "b1": ("INT", rng.integers(0, 50, n).tolist()),
            "m": ("INT", rng.integers(-1000, 100000, n).tolist())}
    seg = build_segment("cfg3", cols, inverted_columns=("b4", "b1"))
    e = GpuEngine(0, "filter.force=index")
    g = e.register(seg)
    ex = ServerQueryExecutor(e)
    vals = "\t\t".join(str(v) for v in sorted(rng.choice(1000, 200, replace=False)))
    for tree in ({"operator": "IN", "column": "b4", "values": [vals]},
                 {"operator": "AND", "children": [
                     {"operator": "RANGE", "column": "s0", "values": ["[10\t\t300)"]},
                     {"operator": "OR", "children": [{"operator": "IN", "column": "b4", "values": [vals]},
                                                     {"operator": "EQUALITY", "column": "b1", "values": ["3"]}]}]},
                 {"operator": "NOT_IN", "column": "b4", "values": [vals]}):
        q = {"aggregations": [{"function": "COUNT", "column": "*"}, {"function": "SUM", "column": "m"},
                              {"function": "MAX", "column": "m"}], "filter": tree, "group_by": None}
        got, st = ex.process_query(q, [g])
        exp, scanned = O.execute_server([seg], q)
        assert st.num_docs_scanned == scanned and got == exp, tree
        assert e.stat("exec.last_pre_segments") == 0, tree
    e.close()


def _leaf(col, op, vals):
    return {"operator": op, "column": col, "values": vals}


def test_depth5_tree_with_1000_id_bitmap_leaf_fused():
    """A filter nested five levels deep (AND / OR alternating, a bushy level among them) with a 1,000-dictId IN on a
    bitmap-indexed column at the bottom: the planner starts each term with its deepest child, and the wide bitmap leaf
    ORs its containers listed per roaring key inside the launch — no segment takes the dense-bitset launch sequence
    (exec.last_pre_segments == 0) — for the aggregation kernel and the group-by kernel, equal to the oracle
    (FilterOperatorUtils.java:74-122, BitmapBasedFilterOperator.java:69-84)."""
    rng = np.random.default_rng(2300)
    segs = []
    for i, n in enumerate((200_000, 131_073)):
        segs.append(build_segment("deep%d" % i, {
            "b": ("INT", rng.integers(0, 4000, n).tolist()),
            "a": ("INT", rng.integers(0, 100, n).tolist()),
            "c": ("INT", rng.integers(0, 50, n).tolist()),
            "d": ("INT", rng.integers(0, 10, n).tolist()),
            "f": ("INT", rng.integers(0, 30, n).tolist()),
            "g": ("INT", rng.integers(0, 7, n).tolist()),
            "m": ("INT", rng.integers(-1000, 100000, n).tolist())}, inverted_columns=("b",)))
    ids = "\t\t".join(str(v) for v in sorted(rng.choice(4000, 1000, replace=False)))
    wide = _leaf("b", "IN", [ids])
    deep = {"operator": "AND", "children": [
        _leaf("a", "RANGE", ["[5\t\t95)"]),
        {"operator": "OR", "children": [
            _leaf("c", "RANGE", ["[0\t\t3)"]),
            {"operator": "AND", "children": [
                _leaf("d", "NOT_IN", ["9"]),
                {"operator": "OR", "children": [
                    {"operator": "AND", "children": [_leaf("g", "IN", ["1\t\t2"]), _leaf("f", "RANGE", ["[0\t\t20)"])]},
                    {"operator": "AND", "children": [
                        _leaf("f", "RANGE", ["[10\t\t30)"]),
                        {"operator": "OR", "children": [wide, _leaf("g", "EQUALITY", ["5"])]}]}]}]}]}]}
    bushy = {"operator": "OR", "children": [  # every level holds two composite children (needs the register stack)
        {"operator": "AND", "children": [
            {"operator": "OR", "children": [_leaf("a", "RANGE", ["[0\t\t10)"]), _leaf("c", "EQUALITY", ["4"])]},
            {"operator": "OR", "children": [_leaf("d", "IN", ["1\t\t2"]), wide]}]},
        {"operator": "AND", "children": [
            {"operator": "OR", "children": [_leaf("f", "RANGE", ["[0\t\t5)"]), _leaf("g", "EQUALITY", ["3"])]},
            {"operator": "OR", "children": [_leaf("a", "RANGE", ["[50\t\t60)"]), _leaf("d", "NOT_IN", ["0\t\t1"])]}]}]}
    e = GpuEngine(0, "filter.force=index")
    gsegs = [e.register(s) for s in segs]
    ex = ServerQueryExecutor(e)
    for tree in (deep, bushy, {"operator": "AND", "children": [wide, _leaf("a", "RANGE", ["[0\t\t50)"])]}):
        q = {"aggregations": [{"function": "COUNT", "column": "*"}, {"function": "SUM", "column": "m"},
                              {"function": "MAX", "column": "m"}], "filter": tree, "group_by": None}
        got, st = ex.process_query(q, gsegs)
        exp, scanned = O.execute_server(segs, q)
        assert st.num_docs_scanned == scanned and got == exp, tree
        assert e.stat("exec.last_pre_segments") == 0, tree
        qg = dict(q, group_by={"columns": ["g"], "top_n": 10})
        gotg, stg = ex.process_query(qg, gsegs, trim=False)
        expg, scg = O.execute_server(segs, qg)
        assert stg.num_docs_scanned == scg and set(gotg) == set(expg)
        for k in expg:
            assert gotg[k][0] == expg[k][0] and gotg[k][1] == expg[k][1] and gotg[k][2] == expg[k][2], k
        assert e.stat("exec.last_pre_segments") == 0, tree
    e.close()


@pytest.mark.parametrize("seed", range(6))
def test_random_aggregations(engine, seed):
    rng = np.random.default_rng(200 + seed)
    n = int(rng.choice([5, 64, 999, 40000]))
    segs = [_random_segment(rng, n, name="s%d" % i) for i in range(int(rng.integers(1, 3)))]
    gsegs = [engine.register(s) for s in segs]
    ex = ServerQueryExecutor(engine)
    for _ in range(8):
        q = {"aggregations": _random_aggs(rng), "filter": _random_tree(rng, segs[0]) if rng.random() < 0.8 else None,
             "group_by": None}
        got, st = ex.process_query(q, gsegs)
        exp, scanned = O.execute_server(segs, q)
        assert st.num_docs_scanned == scanned
        for a, gv, ev in zip(q["aggregations"], got, exp):
            exact = a["column"] not in ("dbl", "flt", "lng")
            _assert_same(a["function"], gv, ev, exact)
    for g in gsegs:
        g.release()


@pytest.mark.parametrize("seed", range(6))
def test_random_group_by(engine, seed):
    rng = np.random.default_rng(300 + seed)
    n = int(rng.choice([64, 777, 20000]))
    segs = [_random_segment(rng, n, name="s%d" % i) for i in range(int(rng.integers(1, 3)))]
    gsegs = [engine.register(s) for s in segs]
    ex = ServerQueryExecutor(engine)
    gpool = ["i0", "i1", "i2", "s", "srt", "i3"]
    for _ in range(5):
        gcols = list(rng.choice(gpool, size=int(rng.integers(1, 3)), replace=False))
        q = {"aggregations": _random_aggs(rng), "filter": _random_tree(rng, segs[0]) if rng.random() < 0.7 else None,
             "group_by": {"columns": gcols, "top_n": 10}}
        got, st = ex.process_query(q, gsegs, trim=False)
        exp, scanned = O.execute_server(segs, q)
        assert st.num_docs_scanned == scanned
        assert set(got) == set(exp)
        for key in exp:
            for a, gv, ev in zip(q["aggregations"], got[key], exp[key]):
                exact = a["column"] not in ("dbl", "flt", "lng")
                _assert_same(a["function"], gv, ev, exact)
    for g in gsegs:
        g.release()


DOUBLE_KEYS = [1.0, 0.1, 100.0, 1e7, 9999999.0, 0.001, 1e-4, 123456789.0, -12.5, 0.1 + 0.2, 2.0 ** 63, 1e21, 5e-324,
               1.7976931348623157e308, -3.25e-9, 65536.0, 1234567.125]
FLOAT_KEYS = [0.1, 1e10, 3.4028235e38, 1.4e-45, 1.0 / 3.0, 16777216.0, 1e-5, -2.5, 0.001, 1e7, 7.0e-4]


@pytest.mark.parametrize("gcols", [["dbl"], ["flt"], ["flt", "i0"], ["i0", "dbl"]])
def test_group_by_floating_point_keys(engine, gcols):
    """FLOAT / DOUBLE group keys are Float.toString / Double.toString of the dictionary values
    (DoubleDictionary.getStringValue, PC/segment/index/readers/DoubleDictionary.java:73-75): plain decimals in
    [1e-3, 1e7), computerized scientific notation outside, shortest distinguishing digits."""
    rng = np.random.default_rng(77)
    n = 5000
    cols = {"dbl": ("DOUBLE", [DOUBLE_KEYS[i] for i in rng.integers(0, len(DOUBLE_KEYS), n)]),
            "flt": ("FLOAT", np.float32([FLOAT_KEYS[i] for i in rng.integers(0, len(FLOAT_KEYS), n)]).astype(np.float64).tolist()),
            "i0": ("INT", rng.integers(0, 3, n).tolist()),
            "v": ("INT", rng.integers(0, 1000, n).tolist())}
    seg = build_segment("fp", cols)
    g = engine.register(seg)
    q = {"aggregations": [{"function": "COUNT", "column": "*"}, {"function": "SUM", "column": "v"}],
         "filter": None, "group_by": {"columns": gcols, "top_n": 100}}
    got, _ = ServerQueryExecutor(engine).process_query(q, [g], trim=False)
    exp, _ = O.execute_server([seg], q)
    assert set(got) == set(exp)
    for key in exp:
        assert got[key][0] == exp[key][0] and got[key][1] == exp[key][1]
    if gcols == ["dbl"]:
        assert {"1.0E7", "1.0E-4", "1.23456789E8", "4.9E-324", "0.30000000000000004", "9999999.0"} <= set(got)
    if gcols == ["flt"]:
        assert {"0.1", "1.0E10", "3.4028235E38", "1.4E-45", "0.33333334", "1.6777216E7"} <= set(got)
    g.release()


GROUP_SINKS = ("group.mode=lds", "group.mode=global", "group.mode=partition", "group.mode=partition;group.ring=0",
               # two-level partitioned plan: many 4-key partitions, EMIT into coarse runs of 4 / 256 partitions
               "group.mode=partition;group.pshift=2;group.split=2",
               "group.mode=partition;group.pshift=0;group.split=8",
               "group.mode=partition;group.pshift=1")


@pytest.mark.parametrize("mode", GROUP_SINKS)
@pytest.mark.parametrize("seed", range(3))
def test_group_by_sinks(mode, seed):
    """Each fused group-by sink (LDS-private, HBM atomics, partitioned COUNT/EMIT/reduce) against the oracle,
    over two segments with identical dictionaries (rows permuted) so the partitioned plan applies."""
    rng = np.random.default_rng(400 + seed)
    n = int(rng.choice([777, 20000]))
    cols, inv = _random_columns(rng, n, sorted_col=False)
    perm = rng.permutation(n)
    segs = [build_segment("p0", cols, inverted_columns=tuple(inv)),
            build_segment("p1", {k: (t, [v[i] for i in perm]) for k, (t, v) in cols.items()},
                          inverted_columns=tuple(inv))]
    e = GpuEngine(0, mode)
    gsegs = [e.register(x) for x in segs]
    ex = ServerQueryExecutor(e)
    gpool = ["i0", "i1", "i2", "s", "i3"]
    # repeated (accumulator kind, column) pairs share one device accumulator (SUM + AVG, HLL twice, MIN twice)
    dup = [{"function": f, "column": c} for f, c in (("SUM", "i0"), ("AVG", "i0"), ("COUNT", "*"),
                                                     ("DISTINCTCOUNTHLL", "i1"), ("DISTINCTCOUNTHLL", "i1"),
                                                     ("MIN", "big"), ("MIN", "big"), ("AVG", "i0"))]
    for it in range(5):
        gcols = list(rng.choice(gpool, size=int(rng.integers(1, 3)), replace=False))
        aggs = [x for x in _random_aggs(rng) if x["column"] != "srt"] or [{"function": "COUNT", "column": "*"}]
        if it == 0:
            aggs = dup
        q = {"aggregations": aggs, "filter": _random_tree(rng, segs[0]) if rng.random() < 0.7 else None,
             "group_by": {"columns": gcols, "top_n": 10}}
        got, st = ex.process_query(q, gsegs, trim=False)
        exp, scanned = O.execute_server(segs, q)
        assert st.num_docs_scanned == scanned
        assert set(got) == set(exp)
        for key in exp:
            for a, gv, ev in zip(q["aggregations"], got[key], exp[key]):
                exact = a["column"] not in ("dbl", "flt", "lng")
                _assert_same(a["function"], gv, ev, exact)
    e.close()


def test_group_by_num_groups_limit(sv_segment):
    """num.groups.limit: first-appearance groups only (IntMapBasedHolder.getGroupId :293-302)."""
    e = GpuEngine(0)
    g = e.register(sv_segment)
    ex = ServerQueryExecutor(e, num_groups_limit=50, max_init_group_holder_capacity=10)
    q = compile_pql("SELECT COUNT(*), SUM(column1) FROM testTable GROUP BY column9, column11")
    got, _ = ex.process_query(q, [g], trim=False)
    exp = O.group_by_segment(sv_segment, q, O.filter_mask(sv_segment, None), num_groups_limit=50,
                             array_threshold=10)
    assert set(got) == set(exp) and len(got) == 50
    for k in exp:
        assert got[k][0] == exp[k][0] and got[k][1] == exp[k][1]
    e.close()


def test_empty_result_defaults(engine, sv_gpu):
    q = "SELECT COUNT(*), SUM(column1), MIN(column3), MAX(column3), AVG(column7) FROM testTable WHERE column1 = 7"
    res, st = ServerQueryExecutor(engine).process_query(q, [sv_gpu])
    assert res[0] == 0 and res[1] == 0.0
    assert res[2] == math.inf and res[3] == -math.inf  # Min/MaxAggregationFunction DEFAULT_VALUE
    assert res[4].sum == 0.0 and res[4].count == 0
    assert st.num_docs_scanned == 0


def test_bad_literal_is_bad_query(engine, sv_gpu):
    from pinot_amd import PinotGpuError
    with pytest.raises(PinotGpuError) as ei:
        ServerQueryExecutor(engine).process_query("SELECT COUNT(*) FROM t WHERE column1 = 'abc'", [sv_gpu])
    assert ei.value.status == 5


def test_fused_and_unfused_agree_on_selective_index_filters(sv_segment):
    """Sorted/bitmap `pre` bitsets + scan leaves in one launch; early chunk exit on empty masks."""
    qs = ["SELECT COUNT(*), SUM(column1), MIN(column3), MAX(column6), AVG(column7), DISTINCTCOUNTHLL(column1) "
          "FROM t WHERE column5 = 'gFuH' AND column1 > 100000000",
          "SELECT COUNT(*), SUM(column3) FROM t WHERE daysSinceEpoch IN (126164076, 167572854) AND column9 < 5000000",
          "SELECT COUNT(*), MAX(column1) FROM t WHERE (column6 = 1689277 OR column11 = 'P') AND column3 > 5"]
    e1, e0 = GpuEngine(0), GpuEngine(0, "exec.fused=0")
    g1, g0 = e1.register(sv_segment), e0.register(sv_segment)
    for text in qs:
        r1, s1 = ServerQueryExecutor(e1).process_query(text, [g1, g1])
        r0, s0 = ServerQueryExecutor(e0).process_query(text, [g0, g0])
        exp, scanned = O.execute_server([sv_segment, sv_segment], compile_pql(text))
        assert s1.num_docs_scanned == s0.num_docs_scanned == scanned
        q = compile_pql(text)
        for a, x, y, z in zip(q["aggregations"], r1, r0, exp):
            _assert_same(a["function"], x, z)
            _assert_same(a["function"], y, z)
    e1.close()
    e0.close()


@pytest.mark.parametrize("cfg", [None, "exec.fused=0", "group.mode=lds", "group.mode=global",
                                 "group.mode=partition;group.pshift=2;group.split=2"])
def test_distributed_group_by_single_rank(sv_segment, cfg):
    """pinot_gpu_group_by_partial -> (no peers) -> finalize equals the one-call group-by, through the fused
    sinks (stopped before compaction) and the bitset path."""
    from pinot_amd.combine import distributed_group_by
    e = GpuEngine(0, cfg)
    g = e.register(sv_segment)
    ex = ServerQueryExecutor(e)
    q = compile_pql("SELECT COUNT(*), SUM(column1), MIN(column3), MAX(column6), AVG(column7), "
                    "DISTINCTCOUNTHLL(column1) FROM t WHERE column1 > 100000000 GROUP BY column9, column11")
    got, st = distributed_group_by(ex, q, [g, g])
    exp, scanned = O.execute_server([sv_segment, sv_segment], q)
    assert st.num_docs_scanned == scanned
    assert set(got) == set(exp)
    for k in exp:
        for a, gv, ev in zip(q["aggregations"], got[k], exp[k]):
            _assert_same(a["function"], gv, ev)
    e.close()


CONFIG3_COLUMNS = [("s0", 1000, "sorted"), ("b1", 10, "inverted"), ("b2", 100, "inverted"), ("b3", 1000, "inverted"),
                   ("b4", 10000, "inverted"), ("d8", 1 << 17, "random"), ("m1", 1024, "random")]
CONFIG3_QUERY = ("SELECT SUM(d8), MAX(m1), COUNT(*) FROM t WHERE s0 IN (10,11,12,13,14,15,16,17,18,19) "
                 "AND (b1 = 3 OR b2 IN (5, 6, 7)) AND b3 <> 0")


def test_synthetic_index_columns_match_host_builder(engine):
    """Synthetic sorted / bitmap-inverted columns (config 3 table) == the host format builder + oracle."""
    import synth
    n = 200003
    seg = engine.register_synthetic("syn3", n, CONFIG3_COLUMNS, seed=0x5EED0011)
    host = synth.make_segment_kinds("syn3", n, CONFIG3_COLUMNS, seed=0x5EED0011)
    ex = ServerQueryExecutor(engine)
    for text in (CONFIG3_QUERY, "SELECT COUNT(*), SUM(d8) FROM t WHERE b4 IN (1, 77, 9999) OR s0 = 999",
                 "SELECT COUNT(*), MIN(m1) FROM t WHERE b2 NOT IN (1, 2) AND s0 BETWEEN 5 AND 500 GROUP BY b1"):
        q = compile_pql(text)
        got, st = ex.process_query(q, [seg], trim=False)
        exp, scanned = O.execute_server([host], q)
        assert st.num_docs_scanned == scanned
        if q.get("group_by"):
            assert set(got) == set(exp)
            for k in exp:
                for a, gv, ev in zip(q["aggregations"], got[k], exp[k]):
                    _assert_same(a["function"], gv, ev)
        else:
            for a, gv, ev in zip(q["aggregations"], got, exp):
                _assert_same(a["function"], gv, ev)
    seg.release()


def test_synthetic_segment_matches_host_generator(engine):
    """The HBM synthetic generator == the oracle's host restatement (bench data parity)."""
    import synth
    n = 200003
    cols = [("d0", 16), ("d2", 1000), ("d8", 1 << 17)]
    seg = engine.register_synthetic("syn", n, cols, seed=0x5EED0007)
    q = compile_pql("SELECT COUNT(*), SUM(d8), MIN(d8), MAX(d2) FROM t WHERE d2 BETWEEN 100 AND 599 AND d0 IN (1,3,5,7)")
    got, _ = ServerQueryExecutor(engine).process_query(q, [seg])
    host = synth.make_segment("syn", n, cols, seed=0x5EED0007)
    exp, _ = O.execute_server([host], q)
    assert got[0] == exp[0] and got[1] == exp[1] and got[2] == exp[2] and got[3] == exp[3]
    seg.release()


# ------------------------------------------------------------------ config 1: the quick-start query shape
def _assert_group_maps(q, got, exp):
    assert set(got) == set(exp)
    for k in exp:
        for a, gv, ev in zip(q["aggregations"], got[k], exp[k]):
            _assert_same(a["function"], gv, ev)


def test_config1_airline_stats_real_data(engine):
    """Config-1 query shape on real reference data: pinot-tools' airlineStats sample (tests/golden/airline_stats.npz,
    9746 rows; ArrDelay nulls = Integer.MIN_VALUE, the default INT dimension null)."""
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "airline_stats.npz"))
    seg = build_segment("airlineStats_OFFLINE_16071_16101_0", {
        "Carrier": ("STRING", z["Carrier"].tolist()), "ArrDelay": ("INT", z["ArrDelay"].tolist()),
        "DaysSinceEpoch": ("INT", z["DaysSinceEpoch"].tolist())})
    g = engine.register(seg)
    med = int(np.median(z["DaysSinceEpoch"]))
    ex = ServerQueryExecutor(engine)
    for text in ("SELECT COUNT(*), SUM(ArrDelay) FROM airlineStats WHERE DaysSinceEpoch > %d GROUP BY Carrier" % med,
                 "SELECT COUNT(*), MAX(ArrDelay), MIN(ArrDelay), AVG(ArrDelay) FROM airlineStats "
                 "WHERE Carrier IN ('AA', 'DL') AND ArrDelay > -100 GROUP BY DaysSinceEpoch"):
        q = compile_pql(text)
        got, st = ex.process_query(q, [g], trim=False)
        exp, scanned = O.execute_server([seg], q)
        assert st.num_docs_scanned == scanned
        _assert_group_maps(q, got, exp)
    g.release()


def test_config1_baseball_synthetic(engine):
    """BASELINE config 1 (quick-start baseballStats; the CSV is absent, so a synthetic segment of the schema's
    shape): SELECT COUNT(*), SUM(runs) WHERE yearID > 2000 GROUP BY teamID, inverted indexes on
    playerID and teamID (baseballStats_offline_table_config.json)."""
    rng = np.random.default_rng(1871)
    n = 97889
    teams = ["T%03d" % i for i in range(149)]
    players = ["p%05d" % i for i in range(18000)]
    runs = np.where(rng.random(n) < 0.45, 0, rng.integers(0, 193, n))
    seg = build_segment("baseballStats_OFFLINE_0", {
        "playerID": ("STRING", [players[i] for i in rng.integers(0, len(players), n)]),
        "yearID": ("INT", rng.integers(1871, 2014, n).tolist()),
        "teamID": ("STRING", [teams[i] for i in rng.integers(0, len(teams), n)]),
        "runs": ("INT", runs.tolist())}, inverted_columns=("playerID", "teamID"))
    g = engine.register(seg)
    q = compile_pql("SELECT COUNT(*), SUM(runs) FROM baseballStats WHERE yearID > 2000 GROUP BY teamID")
    got, st = ServerQueryExecutor(engine).process_query(q, [g], trim=False)
    exp, scanned = O.execute_server([seg], q)
    assert st.num_docs_scanned == scanned
    _assert_group_maps(q, got, exp)
    g.release()


@pytest.mark.parametrize("mode", ["group.mode=partition;group.pshift=3", "group.mode=partition;group.pshift=3;agg.affine=0",
                                  "group.mode=partition;group.pshift=2;group.split=0", "group.mode=partition",
                                  "group.mode=partition;group.ring=0"])
def test_group_by_partitioned_affine(mode):
    """Partitioned plan over arithmetic-progression dictionaries (k_partition_reduce sums dictIds and hashes
    value = base + step * dictId on the device) against the oracle: SUM / AVG / MAX and DISTINCTCOUNTHLL of INT
    and LONG columns, negative bases, over two segments with identical dictionaries."""
    rng = np.random.default_rng(77)
    n = 30000

    def ap(card, base, step):
        ids = np.concatenate([np.arange(card), rng.integers(0, card, n - card)])  # every value present
        return (base + step * ids).astype(np.int64).tolist()

    cols = {"g0": ("INT", ap(40, 0, 1)), "g1": ("INT", ap(30, -7, 3)), "m": ("INT", ap(1000, -123456, 77)),
            "h": ("INT", ap(5000, -2 ** 31 + 5, 1)), "l": ("LONG", ap(300, -2 ** 40, 12345))}
    perm = rng.permutation(n)
    segs = [build_segment("a0", cols),
            build_segment("a1", {k: (t, [v[i] for i in perm]) for k, (t, v) in cols.items()})]
    e = GpuEngine(0, mode)
    gsegs = [e.register(x) for x in segs]
    ex = ServerQueryExecutor(e)
    for pql in ("SELECT COUNT(*), SUM(m), AVG(m), MAX(m), DISTINCTCOUNTHLL(h), DISTINCTCOUNTHLL(l) FROM t "
                "WHERE m > -100000 GROUP BY g0, g1",
                "SELECT SUM(m), DISTINCTCOUNTHLL(m), MIN(l) FROM t GROUP BY g1, g0"):
        q = compile_pql(pql)
        got, st = ex.process_query(q, gsegs, trim=False)
        exp, scanned = O.execute_server(segs, q)
        assert st.num_docs_scanned == scanned
        assert set(got) == set(exp)
        for key in exp:
            for a, gv, ev in zip(q["aggregations"], got[key], exp[key]):
                _assert_same(a["function"], gv, ev, True)
    e.close()
