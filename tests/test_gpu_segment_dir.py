"""Segments loaded from disk straight into HBM (pinot_gpu_segment_load: the engine's C++ v1/v3 reader) answer
queries exactly like the oracle over the same directories (oracle/segment_dir.py): the reference's Java-written
padding segments (LoaderTest.java:144-206) and v1 / v3 directories with sorted and bitmap-indexed columns."""
import os

import numpy as np
import pytest

import pinot_oracle as O
from pinot_amd import GpuEngine, ServerQueryExecutor, build_segment
from segment_dir import read_segment_dir
from segdir_writer import write_segment_dir
from test_gpu_parity import _assert_same

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
SEGS = os.path.join(HERE, "golden", "segments")


@pytest.fixture(scope="module")
def engine():
    e = GpuEngine(0)
    yield e
    e.close()


def _check(engine, dirs, q):
    gsegs = [engine.load(d) for d in dirs]
    osegs = [read_segment_dir(d) for d in dirs]
    got, st = ServerQueryExecutor(engine).process_query(q, gsegs, trim=False)
    exp, scanned = O.execute_server(osegs, q)
    assert st.num_docs_scanned == scanned
    if q.get("group_by"):
        assert set(got) == set(exp)
        for k in exp:
            for a, g, e in zip(q["aggregations"], got[k], exp[k]):
                _assert_same(a["function"], g, e, exact=a["column"] != "percent")
    else:
        for a, g, e in zip(q["aggregations"], got, exp):
            _assert_same(a["function"], g, e, exact=a["column"] != "percent")
    for g in gsegs:
        g.release()
    return got


@pytest.mark.parametrize("name", ["paddingNull", "paddingOld", "paddingPercent"])
def test_java_segments_group_by_name(engine, name):
    q = {"aggregations": [{"function": "COUNT", "column": "*"}, {"function": "SUM", "column": "age"},
                          {"function": "MAX", "column": "outgoingName1"}],
         "filter": None, "group_by": {"columns": ["name"], "top_n": 10}}
    got = _check(engine, [os.path.join(SEGS, name)], q)
    assert set(got) == {"lynda", "lynda 2.0"}


@pytest.mark.parametrize("name", ["paddingOld", "paddingPercent"])
def test_percent_padded_predicates(engine, name):
    """'lynda%' and 'lynda%%' pad to the stored 'lynda%%%%' (LoaderTest.java:164-165): they match 'lynda'."""
    d = os.path.join(SEGS, name)
    for lit in ("lynda%", "lynda%%", "lynda", "lynda 2.0"):
        q = {"aggregations": [{"function": "COUNT", "column": "*"}],
             "filter": {"operator": "EQUALITY", "column": "name", "values": [lit]}, "group_by": None}
        _check(engine, [d], q)


def test_null_padded_predicates(engine):
    d = os.path.join(SEGS, "paddingNull")
    for lit in ("lynda", "lynda 2.0", "lynda%"):
        q = {"aggregations": [{"function": "COUNT", "column": "*"}, {"function": "SUM", "column": "percent"}],
             "filter": {"operator": "EQUALITY", "column": "name", "values": [lit]}, "group_by": None}
        _check(engine, [d], q)


def _random_segment(seed, n):
    rng = np.random.default_rng(seed)
    cols = {
        "i": ("INT", rng.integers(-500, 500, n).astype(np.int32)),
        "l": ("LONG", rng.integers(0, 1 << 40, n).astype(np.int64)),
        "s": ("STRING", np.array(["v%d" % v for v in rng.integers(0, 40, n)], dtype=object)),
        "srt": ("INT", np.sort(rng.integers(0, 100, n)).astype(np.int32)),
        "m": ("INT", rng.integers(0, 1 << 20, n).astype(np.int32)),
    }
    return build_segment("seg%d" % seed, cols, inverted_columns=("i", "s"))


@pytest.mark.parametrize("version", ["v1", "v3"])
def test_written_segments_match_registered_and_oracle(engine, tmp_path, version):
    dirs = [write_segment_dir(_random_segment(20 + k, 70001), str(tmp_path / ("s%d" % k)), version=version)
            for k in range(2)]
    queries = [
        {"aggregations": [{"function": "COUNT", "column": "*"}, {"function": "SUM", "column": "m"},
                          {"function": "MIN", "column": "l"}],
         "filter": {"operator": "AND", "children": [
             {"operator": "IN", "column": "s", "values": ["v1\t\tv7\t\tv30"]},
             {"operator": "RANGE", "column": "srt", "values": ["[10\t\t60)"]}]}, "group_by": None},
        {"aggregations": [{"function": "COUNT", "column": "*"}, {"function": "SUM", "column": "m"},
                          {"function": "DISTINCTCOUNTHLL", "column": "i"}],
         "filter": {"operator": "EQUALITY", "column": "i", "values": ["17"]}, "group_by": None},
        {"aggregations": [{"function": "COUNT", "column": "*"}, {"function": "MAX", "column": "m"}],
         "filter": {"operator": "NOT", "column": "srt", "values": ["3"]},
         "group_by": {"columns": ["s", "srt"], "top_n": 10}},
    ]
    for q in queries:
        _check(engine, dirs, q)


def test_raw_columns_loaded_from_disk(engine, tmp_path):
    """Raw (no-dictionary) columns read from their chunked .sv.raw.fwd (Snappy and PASS_THROUGH chunks), transcoded
    at registration, answer like the oracle over the in-memory raw columns (raw-value predicate semantics)."""
    from pinot_amd import compile_pql
    from segdir_writer import raw_chunk_file
    rng = np.random.default_rng(12)
    n = 7000
    cols = {"a": ("INT", rng.integers(-300, 300, n).astype(np.int32)), "m": ("LONG", rng.integers(-10 ** 6, 10 ** 6, n)),
            "f": ("FLOAT", (rng.integers(-20, 20, n) * 0.5).astype(np.float32)),
            "d": ("DOUBLE", np.round(rng.normal(5, 3, n), 2) + 0.001), "g": ("INT", rng.integers(0, 6, n).astype(np.int32))}
    segs, dirs = [], []
    for i, (version, comp) in enumerate((("v1", 1), ("v3", 0))):
        seg = build_segment("raw%d" % i, cols, raw_columns=("a", "m", "f", "d"))
        for c in ("a", "m", "f", "d"):
            col = seg.columns[c]
            col.raw_file = raw_chunk_file(col.fwd, 4 if col.data_type in ("INT", "FLOAT") else 8, n,
                                          docs_per_chunk=1000, compression=comp)
        dirs.append(write_segment_dir(seg, str(tmp_path / ("r%d" % i)), version=version))
        segs.append(seg)
    gsegs = [engine.load(d) for d in dirs]
    ex = ServerQueryExecutor(engine)
    for text in ("SELECT COUNT(*), SUM(a), MIN(m), MAX(d), AVG(f), DISTINCTCOUNTHLL(a) FROM t WHERE a > 10 AND f <= 3",
                 "SELECT SUM(m), MIN(d) FROM t WHERE m BETWEEN -1000 AND 400000 OR d < 2.5",
                 "SELECT MIN(a), MAX(m) FROM t",
                 "SELECT COUNT(*), SUM(m) FROM t WHERE f IN (1.5, 2.0, -3.5) GROUP BY g, a TOP 5"):
        q = compile_pql(text)
        got, st = ex.process_query(q, gsegs, trim=False)
        exp, scanned = O.execute_server(segs, q)
        assert st.num_docs_scanned == scanned, text
        if q.get("group_by"):
            assert set(got) == set(exp), text
            pairs = [(got[k], exp[k]) for k in exp]
        else:
            pairs = [(got, exp)]
        for gr, er in pairs:
            for a, g, e in zip(q["aggregations"], gr, er):
                _assert_same(a["function"], g, e, exact=a["column"] not in ("d", "f"))
    for g in gsegs:
        g.release()


@pytest.mark.parametrize("version", ["v1", "v3"])
def test_segment_cache_by_name_and_crc(tmp_path, version):
    """pinot_gpu_segment_acquire: the same name + creation.meta CRC is the cached device copy; acquires are
    reference-counted (SegmentDataManager reference counts): a new CRC replaces the cache entry while the old copy
    stays valid for its holders until the last release; no creation.meta is never cached."""
    from pinot_amd import PinotGpuError
    e = GpuEngine(0)
    try:
        seg = _random_segment(40, 5000)
        d1 = write_segment_dir(seg, str(tmp_path / "a"), version=version, crc=1234567890123)
        g1, hit = e.acquire(d1)
        assert not hit
        g2, hit = e.acquire(d1)
        assert hit and g2.handle == g1.handle
        ex = ServerQueryExecutor(e)
        q = {"aggregations": [{"function": "COUNT", "column": "*"}, {"function": "SUM", "column": "m"}],
             "filter": {"operator": "RANGE", "column": "i", "values": ["[0\t\t*)"]}, "group_by": None}
        exp, _ = O.execute_server([seg], q)
        got, _ = ex.process_query(q, [g2])
        assert got == exp
        # a new build of the segment (another CRC): reloaded and cached; the old copy serves its two holders
        seg_b = _random_segment(41, 6000)
        seg_b.name = seg.name
        d2 = write_segment_dir(seg_b, str(tmp_path / "b"), version=version, crc=-5)
        g3, hit = e.acquire(d2)
        assert not hit and g3.handle != g1.handle
        got, _ = ex.process_query(q, [g1])
        assert got == exp
        old = g1.handle
        g1.release()
        got, _ = ex.process_query(q, [g2])
        assert got == exp
        g2.release()  # last reference of the replaced copy: dropped
        g1.handle = old
        with pytest.raises(PinotGpuError):
            ex.process_query(q, [g1])
        g1.handle = None
        got, _ = ex.process_query(q, [g3])
        assert got == O.execute_server([seg_b], q)[0]
        g4, hit = e.acquire(d2)
        assert hit and g4.handle == g3.handle
        g3.release()  # g4 still holds it: cached, valid
        got, _ = ex.process_query(q, [g4])
        assert got == O.execute_server([seg_b], q)[0]
        g5, hit = e.acquire(d2)
        assert hit and g5.handle == g4.handle
        g4.release()
        g5.release()  # the last reference: the next acquire loads again
        g6, hit = e.acquire(d2)
        assert not hit
        g6.release()
        # no creation.meta: loaded every time
        d3 = write_segment_dir(seg, str(tmp_path / "c"), version=version)
        h1, hit1 = e.acquire(d3)
        h2, hit2 = e.acquire(d3)
        assert not hit1 and not hit2 and h1.handle != h2.handle
        h1.release()
        h2.release()
    finally:
        e.close()
