"""Multi-value columns on the GPU against the oracle: MV scan leaves (applyMV any / every) and MV inverted-index
leaves, the *MV aggregation functions beside single-value ones, group-by over MV group columns (cartesian product
with duplicates) and MV aggregations under single-value group keys, multi-segment combines, segment directories
holding <col>.mv.fwd, and the DataTable column names of MV functions."""
import numpy as np
import pytest

import pinot_oracle as O
from pinot_amd import GpuEngine, ServerQueryExecutor
from pinot_amd._lib import PinotGpuError
from segdir_writer import write_segment_dir
from test_gpu_parity import _assert_same, _random_leaf
from test_mv import mv_rows, mv_segment
from pinot_amd import build_segment

pytestmark = pytest.mark.gpu
MV_COLS = ("tags", "tagl", "tagd", "tags_s")
FP_COLS = ("tagd", "tagl")  # double sums (LONG sums beyond 2^53 round differently in another order)


@pytest.fixture(scope="module")
def engine():
    e = GpuEngine(0)
    yield e
    e.close()


def _tree(rng, seg, depth=0):
    if depth >= 2 or rng.random() < 0.45:
        return _random_leaf(rng, seg)
    return {"operator": rng.choice(["AND", "OR"]),
            "children": [_tree(rng, seg, depth + 1) for _ in range(int(rng.integers(2, 4)))]}


def _aggs(rng):
    pool = [("COUNT", "*"), ("COUNTMV", "tags"), ("SUMMV", "tags"), ("MINMV", "tagl"), ("MAXMV", "tags"),
            ("AVGMV", "tagl"), ("SUMMV", "tagd"), ("MINMV", "tagd"), ("AVGMV", "tags"), ("DISTINCTCOUNTHLLMV", "tags"),
            ("DISTINCTCOUNTHLLMV", "tags_s"), ("COUNTMV", "tags_s"), ("SUM", "m"), ("MAX", "m"), ("AVG", "m")]
    idx = rng.choice(len(pool), size=int(rng.integers(1, 6)), replace=False)
    return [{"function": pool[i][0], "column": pool[i][1]} for i in idx]


def _check(q, got, exp):
    if q["group_by"]:
        assert set(got) == set(exp), q
        pairs = [(got[k], exp[k]) for k in exp]
    else:
        pairs = [(got, exp)]
    for gv_row, ev_row in pairs:
        for a, gv, ev in zip(q["aggregations"], gv_row, ev_row):
            f = O.sv(a["function"])
            _assert_same(f, gv, ev, a["column"] not in FP_COLS)


@pytest.mark.parametrize("seed", range(4))
def test_mv_filter_bitsets(engine, seed):
    rng = np.random.default_rng(900 + seed)
    n = int(rng.choice([1, 63, 64, 65, 1000, 30001]))
    seg = mv_segment(rng, n)
    g = engine.register(seg)
    for mode in ("", "filter.force=scan", "filter.force=index"):
        engine.set_config(mode)
        for _ in range(10):
            tree = _tree(rng, seg)
            exp = O.filter_mask(seg, tree)
            bits, cnt = engine.filter(g, tree)
            got = np.unpackbits(bits.view(np.uint8), bitorder="little")[:n].astype(bool)
            assert cnt == int(exp.sum()), (mode, tree)
            assert (got == exp).all(), (mode, tree)
    engine.set_config("")
    g.release()


@pytest.mark.parametrize("seed", range(4))
def test_mv_aggregations(engine, seed):
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.choice([5, 64, 999, 40000]))
    segs = [mv_segment(rng, n, name="m%d" % i) for i in range(int(rng.integers(1, 4)))]
    gsegs = [engine.register(s) for s in segs]
    ex = ServerQueryExecutor(engine)
    for _ in range(10):
        q = {"aggregations": _aggs(rng), "filter": _tree(rng, segs[0]) if rng.random() < 0.7 else None,
             "group_by": None}
        got, st = ex.process_query(q, gsegs)
        exp, scanned = O.execute_server(segs, q)
        assert st.num_docs_scanned == scanned
        _check(q, got, exp)
    for g in gsegs:
        g.release()


@pytest.mark.parametrize("seed", range(4))
def test_mv_group_by(engine, seed):
    rng = np.random.default_rng(1100 + seed)
    n = int(rng.choice([7, 500, 20000]))
    segs = [mv_segment(rng, n, name="g%d" % i) for i in range(int(rng.integers(1, 3)))]
    gsegs = [engine.register(s) for s in segs]
    ex = ServerQueryExecutor(engine)
    shapes = [["tags"], ["g"], ["tags_s", "g"], ["tags", "tags_s"], ["s", "tagl"], ["tagd"]]
    for it in range(12):
        cols = shapes[it % len(shapes)]
        aggs = _aggs(rng) if it % 3 else [{"function": "COUNT", "column": "*"}, {"function": "SUM", "column": "m"}]
        q = {"aggregations": aggs, "filter": _tree(rng, segs[0]) if rng.random() < 0.6 else None,
             "group_by": {"columns": cols, "top_n": 10}}
        got, st = ex.process_query(q, gsegs, trim=False)
        exp, scanned = O.execute_server(segs, q)
        assert st.num_docs_scanned == scanned
        _check(q, got, exp)
    for g in gsegs:
        g.release()


@pytest.mark.parametrize("seed", range(3))
def test_mv_group_by_admission(engine, seed):
    """MV group-by beyond num.groups.limit: each segment's holder admits keys at first appearance (doc order, each
    doc's keys in getIntRawKeys order) up to min(product, limit), then the 2 x limit inter-segment cap in segment order
    (DictionaryBasedGroupKeyGenerator.java:282-302, CombineGroupByOperator.java:80,147); small limits and holder
    thresholds (max.init.group.holder.capacity) make both rules bind on small segments."""
    rng = np.random.default_rng(1500 + seed)
    segs = [mv_segment(rng, int(rng.choice([600, 3000])), name="a%d" % i) for i in range(int(rng.integers(2, 4)))]
    gsegs = [engine.register(s) for s in segs]
    shapes = [["tags", "tags_s"], ["tags", "g"], ["tags_s", "tagl"], ["g", "tags"]]
    for it, cols in enumerate(shapes):
        limit, thr = [(40, 10), (120, 60), (25, 5), (300, 10)][it]
        aggs = [{"function": "COUNT", "column": "*"}, {"function": "SUM", "column": "m"},
                {"function": "MAXMV", "column": "tags"}, {"function": "AVGMV", "column": "tagl"}]
        q = {"aggregations": aggs, "filter": _tree(rng, segs[0]) if it % 2 else None,
             "group_by": {"columns": cols, "top_n": 10}}
        ex = ServerQueryExecutor(engine, num_groups_limit=limit, max_init_group_holder_capacity=thr)
        got, st = ex.process_query(q, gsegs, trim=False)
        exp, scanned = O.execute_server(segs, q, num_groups_limit=limit, array_threshold=thr)
        assert st.num_docs_scanned == scanned
        assert len(exp) <= 2 * limit
        _check(q, got, exp)
    for g in gsegs:
        g.release()


def hashed_mv_segment(rng, n, name):
    """Group columns whose cardinality product is beyond the dense key limit (2^27): an MV INT column of ~2n values
    and a single-value LONG of ~n values (the LONG_MAP / ARRAY_MAP holder shapes, DictionaryBasedGroupKeyGenerator
    .java:79-126), beside an MV aggregation column."""
    cols = {
        "hv": ("INT", [[int(v) for v in r] for r in mv_rows(rng, n, 4 * n, 3)]),
        "hs": ("LONG", rng.integers(0, 10 ** 12, n).astype(np.int64)),
        "tags": ("INT", [[int(v) * 7 - 100 for v in r] for r in mv_rows(rng, n, 40, 4)]),
        "g": ("INT", rng.integers(0, 6, n).astype(np.int32)),
        "m": ("INT", rng.integers(-1000, 1000, n).astype(np.int32)),
    }
    return build_segment(name, cols, inverted_columns=(), mv_columns=("hv", "tags"), allow_sorted=False)


@pytest.mark.parametrize("seed", range(2))
def test_mv_group_by_hashed_key_space(engine, seed):
    """MV group-by over a key space past the dense limit: keys are fingerprint-table slots (mv_hash.h), the result's
    groups carry their global-id tuples; with and without the num.groups.limit admission binding."""
    rng = np.random.default_rng(1700 + seed)
    segs = [hashed_mv_segment(rng, 12000, "h%d" % i) for i in range(2)]
    gsegs = [engine.register(s) for s in segs]
    cases = [(["hv", "hs"], None, None), (["hs", "hv", "g"], None, None), (["hv", "hs"], 500, 10)]
    for cols, limit, thr in cases:
        aggs = [{"function": "COUNT", "column": "*"}, {"function": "SUMMV", "column": "tags"},
                {"function": "SUM", "column": "m"}, {"function": "DISTINCTCOUNTHLLMV", "column": "tags"}]
        q = {"aggregations": aggs, "filter": {"operator": "RANGE", "column": "m", "values": ["[-500\t\t900)"]},
             "group_by": {"columns": cols, "top_n": 10}}
        kw = {} if limit is None else {"num_groups_limit": limit, "max_init_group_holder_capacity": thr}
        ex = ServerQueryExecutor(engine, **kw)
        got, st = ex.process_query(q, gsegs, trim=False)
        okw = {} if limit is None else {"num_groups_limit": limit, "array_threshold": thr}
        exp, scanned = O.execute_server(segs, q, **okw)
        assert st.num_docs_scanned == scanned
        assert len(exp) > (2 * limit if limit else 10000) // 2
        _check(q, got, exp)
        dt, _ = ex.process_query_datatable(q, gsegs)
        assert b"sumMV_tags" in dt
    for g in gsegs:
        g.release()


def test_mv_segment_dir_and_datatable(engine, tmp_path):
    rng = np.random.default_rng(1200)
    seg = mv_segment(rng, 5000)
    d = write_segment_dir(seg, str(tmp_path / "s"), version="v3")
    g = engine.load(d)
    ex = ServerQueryExecutor(engine)
    q = {"aggregations": [{"function": "COUNTMV", "column": "tags"}, {"function": "AVGMV", "column": "tagl"},
                          {"function": "DISTINCTCOUNTHLLMV", "column": "tags_s"}],
         "filter": {"operator": "IN", "column": "tags", "values": ["-100\t\t-93\t\t-86"]},
         "group_by": {"columns": ["tags_s"], "top_n": 10}}
    got, _ = ex.process_query(q, [g], trim=False)
    exp, _ = O.execute_server([seg], q)
    _check(q, got, exp)
    dt, _ = ex.process_query_datatable(q, [g])
    for name in (b"countMV_tags", b"avgMV_tagl", b"distinctCountHLLMV_tags_s"):
        assert name in dt
    qa = dict(q, group_by=None)
    dt, _ = ex.process_query_datatable(qa, [g])
    assert b"countMV_tags" in dt and b"avgMV_tagl" in dt
    g.release()


def test_mv_errors(engine):
    rng = np.random.default_rng(1300)
    seg = mv_segment(rng, 200)
    g = engine.register(seg)
    ex = ServerQueryExecutor(engine)
    with pytest.raises(PinotGpuError):  # a single-value function over an MV column
        ex.process_query({"aggregations": [{"function": "SUM", "column": "tags"}], "filter": None,
                          "group_by": None}, [g])
    with pytest.raises(PinotGpuError):  # an MV function over a single-value column
        ex.process_query({"aggregations": [{"function": "SUMMV", "column": "m"}], "filter": None,
                          "group_by": None}, [g])
    g.release()
