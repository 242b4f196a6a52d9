"""Star-tree v2 plans on the GPU (pinot_gpu_segment_attach_star_tree): queries the tree fits run on the star docs —
host traversal, device aggregation / group-by over the pair columns — and equal the oracle's star-tree plan
(results and numDocsScanned) and the scan plan; startree.use=0 and non-fitting queries take the regular plan."""
import numpy as np
import pytest

import pinot_oracle as O
import startree as S
from pinot_amd import GpuEngine, ServerQueryExecutor
from startree_writer import build_star_tree
from test_startree import DIMS, PAIRS, _same, random_query, st_segment

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = GpuEngine(0)
    yield e
    e.close()


def _attach(engine, seg, leaf=10, skip=()):
    st = build_star_tree(seg, DIMS, PAIRS, max_leaf_records=leaf, skip_star=skip)
    g = engine.register(seg)
    g.attach_star_tree(seg, st.tree_bytes, st.dimensions, st.dims, st.metrics)
    return g, st


@pytest.mark.parametrize("seed", range(4))
def test_star_tree_plans(engine, seed):
    rng = np.random.default_rng(1600 + seed)
    segs = [st_segment(rng, int(rng.choice([50, 2000, 20000])), name="st%d" % i) for i in range(1 + seed % 2)]
    attached = [_attach(engine, s, leaf=[1, 10, 100, 5000][seed]) for s in segs]
    gs, sts = [a[0] for a in attached], [a[1] for a in attached]
    ex = ServerQueryExecutor(engine)
    for it in range(16):
        group = [None, ["a"], ["b", "c"], ["c", "a", "b"]][it % 4]
        q = random_query(rng, segs[0], group)
        got, st = ex.process_query(q, gs, trim=False)
        exp, scanned = S.execute_server(segs, sts, q)
        _same(q, got, exp)
        assert st.num_docs_scanned == scanned, q
        scan, _ = O.execute_server(segs, q)
        _same(q, got, scan)
    engine.set_config("startree.use=0")
    try:
        q = random_query(rng, segs[0], ["a"])
        got, st = ex.process_query(q, gs, trim=False)
        exp, scanned = O.execute_server(segs, q)
        _same(q, got, exp)
        assert st.num_docs_scanned == scanned
    finally:
        engine.set_config("startree.use=1")
    # a function without a pair (AVG over x) runs the regular plan
    q = {"aggregations": [{"function": "AVG", "column": "x"}, {"function": "COUNT", "column": "*"}],
         "filter": {"operator": "EQUALITY", "column": "a", "values": ["1"]}, "group_by": None}
    got, st = ex.process_query(q, gs)
    exp, scanned = O.execute_server(segs, q)
    assert got[1] == exp[1] and got[0].count == exp[0][1] and st.num_docs_scanned == scanned
    for g in gs:
        g.release()


def test_star_tree_attach_checks(engine):
    from pinot_amd import PinotGpuError
    rng = np.random.default_rng(1700)
    seg = st_segment(rng, 300)
    st = build_star_tree(seg, DIMS, PAIRS, max_leaf_records=5)
    g = engine.register(seg)
    bad = bytearray(st.tree_bytes)
    bad[0] ^= 0xFF
    with pytest.raises(PinotGpuError, match="magic"):
        g.attach_star_tree(seg, bytes(bad), st.dimensions, st.dims, st.metrics)
    with pytest.raises(PinotGpuError, match="size"):
        g.attach_star_tree(seg, st.tree_bytes[:-4], st.dimensions, st.dims, st.metrics)
    g.attach_star_tree(seg, st.tree_bytes, st.dimensions, st.dims, st.metrics)
    with pytest.raises(PinotGpuError, match="already"):
        g.attach_star_tree(seg, st.tree_bytes, st.dimensions, st.dims, st.metrics)
    g.release()


@pytest.mark.parametrize("version", ["v1", "v3"])
def test_star_tree_from_segment_directory(engine, tmp_path, version):
    """star_tree_index + star_tree_index_map + startree.v2.* metadata (StarTreeLoaderUtils) read by
    pinot_gpu_segment_load: fitting queries run on the loaded tree."""
    from segdir_writer import write_segment_dir
    rng = np.random.default_rng(1800)
    seg = st_segment(rng, 4000, name="stdir")
    st = build_star_tree(seg, DIMS, PAIRS, max_leaf_records=20)
    g = engine.load(write_segment_dir(seg, str(tmp_path / "s"), version=version, star_tree=st))
    ex = ServerQueryExecutor(engine)
    for it in range(8):
        q = random_query(rng, seg, [None, ["b"]][it % 2])
        got, stt = ex.process_query(q, [g], trim=False)
        exp, scanned = S.execute_server([seg], [st], q)
        _same(q, got, exp)
        assert stt.num_docs_scanned == scanned
    g.release()


def test_star_tree_mixed_segments(engine):
    """Segments plan one by one (AggregationPlanNode per segment): a segment with a fitting tree runs the star-tree
    plan, one without runs the scan plan, and the two blocks merge — numDocsScanned adds the star docs of the first
    to the matching docs of the second; group-bys likewise fold both kinds of segment into one key space."""
    rng = np.random.default_rng(1900)
    segs = [st_segment(rng, 3000, name="mx%d" % i) for i in range(3)]
    g0, st0 = _attach(engine, segs[0], leaf=10)
    g2, st2 = _attach(engine, segs[2], leaf=100)
    g1 = engine.register(segs[1])
    gs, trees = [g0, g1, g2], [st0, None, st2]
    ex = ServerQueryExecutor(engine)
    for it in range(12):
        q = random_query(rng, segs[0], None)
        got, st = ex.process_query(q, gs)
        exp, scanned = S.execute_server(segs, trees, q)
        _same(q, got, exp)
        assert st.num_docs_scanned == scanned, q
    for it in range(12):
        q = random_query(rng, segs[0], [["b"], ["a", "c"], ["c"]][it % 3])
        got, st = ex.process_query(q, gs, trim=False)
        exp, scanned = S.execute_server(segs, trees, q)
        _same(q, got, exp)
        assert st.num_docs_scanned == scanned, q
        scan, _ = O.execute_server(segs, q)
        _same(q, got, scan)
    for g in gs:
        g.release()


def test_star_tree_hll_after_other_plans(engine):
    """A star-tree DISTINCTCOUNTHLL right after scan-plan and star-tree HLL queries that filled the shared register
    block: the star plan starts from cleared registers (a narrower filter, and one matching nothing, equal the oracle
    rather than the earlier queries' registers)."""
    rng = np.random.default_rng(1700)
    seg = st_segment(rng, 20000, name="sth")
    g, st = _attach(engine, seg, leaf=10)
    ex = ServerQueryExecutor(engine)
    wide = {"aggregations": [{"function": "DISTINCTCOUNTHLL", "column": "m"}], "filter": None, "group_by": None}
    got, _ = ex.process_query(wide, [g])  # m has no HLL pair: the regular (scan) plan
    assert got[0].cardinality() == O.execute_server([seg], wide)[0][0].cardinality()
    for flt in (None, {"operator": "EQUALITY", "column": "a", "values": ["1"]},
                {"operator": "EQUALITY", "column": "a", "values": ["123456789"]}):
        q = {"aggregations": [{"function": "DISTINCTCOUNTHLL", "column": "c"}, {"function": "COUNT", "column": "*"}],
             "filter": flt, "group_by": None}
        got, stats = ex.process_query(q, [g])
        exp, scanned = S.execute_server([seg], [st], q)
        assert got[1] == exp[1] and stats.num_docs_scanned == scanned, flt
        assert got[0].cardinality() == exp[0].cardinality(), flt
        assert (np.asarray(got[0].registers, dtype=np.int64) == np.asarray(exp[0].reg, dtype=np.int64)).all(), flt
    g.release()
