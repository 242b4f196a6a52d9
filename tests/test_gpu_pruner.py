"""Segment pruning on GPU-registered segments (pinot_gpu_prune_segments / pinot_gpu_server_prune_segments) and the
executor path around it (ServerQueryExecutorV1Impl.processQuery :183-216): per-segment decisions equal the oracle's
(oracle/pruner.py, pinned by ColumnValueSegmentPrunerTest), results equal the unpruned run, numSegmentsProcessed
counts the kept segments, totalDocs counts all of them, and an all-pruned query answers buildEmptyDataTable."""
import ctypes as C

import numpy as np
import pytest

import datatable as D
import pinot_oracle as O
import pruner as P
from pinot_amd import (GpuEngine, GpuServer, PinotGpuError, ServerExecutor, ServerQueryExecutor, _lib,
                       build_segment, compile_pql)
from pinot_amd.executor import QueryMarshal, _segment_handles

pytestmark = pytest.mark.gpu


def _segments(n=6, docs=3000, seed=5):
    """'time' ranges [1000 i, 1000 i + 499] per segment: range predicates select whole segments."""
    rng = np.random.default_rng(seed)
    segs = []
    for i in range(n):
        cols = {"time": ("INT", (1000 * i + rng.integers(0, 500, docs)).astype(np.int32)),
                "g": ("INT", rng.integers(0, 7, docs).astype(np.int32)),
                "m": ("LONG", rng.integers(-1000, 1000, docs).astype(np.int64)),
                "s": ("STRING", np.array(["c%d" % (i + v) for v in rng.integers(0, 3, docs)], dtype=object))}
        segs.append(build_segment("seg_%d" % i, cols, min_max=("time", "s")))
    return segs


@pytest.fixture(scope="module")
def engine():
    e = GpuEngine(0)
    yield e
    e.close()


QUERIES = [
    "SELECT COUNT(*), SUM(m), MIN(m), MAX(m), AVG(m), DISTINCTCOUNTHLL(g) FROM t WHERE time BETWEEN 1200 AND 2300",
    "SELECT COUNT(*), SUM(m) FROM t WHERE time = 3007 OR time > 5200",
    "SELECT COUNT(*), SUM(m) FROM t WHERE s = 'c4' AND time < 4000",
    "SELECT COUNT(*), SUM(m), AVG(m) FROM t WHERE time >= 2000 AND g IN (1, 2) GROUP BY g, s",
    "SELECT COUNT(*) FROM t WHERE time < 1000 OR time BETWEEN 4100 AND 4499",
    "SELECT SUM(m) FROM t WHERE time <> 5",
]


def _norm(v):
    if hasattr(v, "registers"):  # HyperLogLog
        return ("hll", bytes(v.registers), v.cardinality())
    if hasattr(v, "count") and hasattr(v, "sum"):  # AvgPair
        return ("avg", v.sum, v.count)
    return v


def _same(a, b):
    return [_norm(x) for x in a] == [_norm(x) for x in b]


def _native_flags(engine, segs, q):
    m = QueryMarshal(q)
    pruned = (C.c_uint8 * len(segs))()
    total = C.c_int64()
    _lib.check(engine.lib.pinot_gpu_prune_segments(engine.ptr, _segment_handles(segs), len(segs), C.byref(m.q),
                                                   _lib.PRUNER_DEFAULT, pruned, C.byref(total)))
    return [bool(x) for x in pruned], total.value


def test_flags_match_oracle_and_results_match_unpruned(engine):
    host = _segments()
    gsegs = [engine.register(s) for s in host]
    total_docs = sum(s.num_docs for s in host)
    pruning, plain = ServerQueryExecutor(engine), ServerQueryExecutor(engine, pruners=0)
    for text in QUERIES:
        q = compile_pql(text)
        want = [P.prune(P.ranges(s), q) for s in host]
        flags, total = _native_flags(engine, gsegs, q)
        assert flags == want, text
        assert total == total_docs
        for s, f in zip(host, want):  # a pruned segment holds no match
            assert not f or int(O.filter_mask(s, q["filter"]).sum()) == 0, text
        got, st = pruning.process_query(q, gsegs, trim=False)
        ref, st0 = plain.process_query(q, gsegs, trim=False)
        kept = len(host) - sum(want)
        if q.get("group_by"):
            assert set(got) == set(ref), text
            for k in got:
                assert _same(got[k], ref[k]), (text, k)
        else:
            assert _same(got, ref), text
        assert st.num_segments_processed == kept and st0.num_segments_processed == len(host), text
        assert st.num_total_raw_docs == total_docs == st0.num_total_raw_docs
        assert st.num_docs_scanned == st0.num_docs_scanned
        assert st.num_segments_matched == st0.num_segments_matched
    for g in gsegs:
        g.release()


def test_all_pruned_answers_the_empty_datatable(engine):
    host = _segments(3)
    gsegs = [engine.register(s) for s in host]
    total_docs = sum(s.num_docs for s in host)
    ex = ServerQueryExecutor(engine)
    for text in ("SELECT COUNT(*), SUM(m), MIN(m), MAX(m), AVG(m), DISTINCTCOUNTHLL(g) FROM t WHERE time > 99999",
                 "SELECT SUM(m), AVG(m) FROM t WHERE time BETWEEN 600 AND 900 GROUP BY g",
                 "SELECT COUNT(*) FROM t WHERE missing = 3"):
        q = compile_pql(text)
        data, st = ex.process_query_datatable(q, gsegs, server=(3, 2, 77))
        assert data == D.encode_empty(q, total_docs, (3, 2, 77)), text
        assert st.num_segments_processed == 0 and st.num_total_raw_docs == total_docs
        res, st = ex.process_query(q, gsegs)
        if q.get("group_by"):
            assert res == {}
        else:
            assert res[0] == 0 if q["aggregations"][0]["function"] == "COUNT" else res[0] == 0.0
    # a partly pruned DataTable: totalDocs is the whole table's
    q = compile_pql("SELECT COUNT(*), SUM(m) FROM t WHERE time < 1400")
    data, st = ex.process_query_datatable(q, gsegs)
    md = dict(D.decode(data)["metadata"])
    assert md["totalDocs"] == str(total_docs) and md["numSegmentsProcessed"] == "2"
    # the spent budget wins over pruning (ServerQueryExecutorV1Impl.java:116-126 runs first)
    with pytest.raises(PinotGpuError) as ei:
        ServerQueryExecutor(engine, timeout_ms=-1).process_query("SELECT COUNT(*) FROM t WHERE time > 99999", gsegs)
    assert ei.value.status == _lib.PINOT_ERR_TIMEOUT
    for g in gsegs:
        g.release()


def test_server_executor_prunes():
    host = _segments(4, seed=9)
    srv = GpuServer([0])
    gsegs = [srv.engines[0].register(s) for s in host]
    pruning, plain = ServerExecutor(srv), ServerExecutor(srv, pruners=0)
    for text in QUERIES[:3] + ["SELECT COUNT(*) FROM t WHERE time > 99999"]:
        q = compile_pql(text)
        got, st = pruning.process_query(q, gsegs)
        ref, st0 = plain.process_query(q, gsegs)
        assert _same(got, ref), text
        assert st.num_segments_processed == len(host) - sum(P.prune(P.ranges(s), q) for s in host), text
        assert st.num_total_raw_docs == st0.num_total_raw_docs
    srv.close()


def _partitioned_segments(tmp_path, n=4, docs=4000, seed=21):
    """A table partitioned on pk (Modulo 4: segment i holds partition i's values) with a bloom filter on u (sparse
    ids whose min / max ranges overlap), registered from descriptors and loaded from v1 / v3 directories written with
    the .bloom files and partition metadata (the loaded form reads them from the files)."""
    from segdir_writer import write_segment_dir
    rng = np.random.default_rng(seed)
    host, dirs = [], []
    for i in range(n):
        pk = (4 * rng.integers(0, 50, docs) + i).astype(np.int32)
        u = (rng.integers(0, 200, docs) * 97 + i).astype(np.int32)
        cols = {"pk": ("INT", pk), "u": ("INT", u), "m": ("LONG", rng.integers(-500, 500, docs).astype(np.int64)),
                "s": ("STRING", np.array(["w%d" % (i * 10 + v) for v in rng.integers(0, 5, docs)], dtype=object))}
        seg = build_segment("pseg_%d" % i, cols, min_max=True, bloom_columns=("u", "s"),
                            partitions={"pk": ("Modulo", 4), "s": ("Murmur", 3)})
        host.append(seg)
        dirs.append(write_segment_dir(seg, str(tmp_path / ("pseg_%d" % i)), version="v3" if i % 2 else "v1"))
    return host, dirs


def test_bloom_and_partition_pruning(engine, tmp_path):
    host, dirs = _partitioned_segments(tmp_path)
    for form in ("register", "load"):
        gsegs = [engine.register(s) for s in host] if form == "register" else [engine.load(d) for d in dirs]
        pruning, plain = ServerQueryExecutor(engine), ServerQueryExecutor(engine, pruners=0)
        some_pruned = 0
        for text in ("SELECT COUNT(*), SUM(m) FROM t WHERE pk = 42", "SELECT COUNT(*), SUM(m) FROM t WHERE pk = 7",
                     "SELECT COUNT(*), SUM(m) FROM t WHERE u = %d" % (97 * 13 + 2),
                     "SELECT COUNT(*), SUM(m) FROM t WHERE u = %d" % (97 * 13 + 5),
                     "SELECT COUNT(*), MAX(m) FROM t WHERE s = 'w21' OR pk = 1",
                     "SELECT COUNT(*), SUM(m) FROM t WHERE pk = 6 AND u > 100 GROUP BY s"):
            q = compile_pql(text)
            want = [P.prune(P.ranges(s), q) for s in host]
            flags, _ = _native_flags(engine, gsegs, q)
            assert flags == want, (form, text)
            some_pruned += sum(want)
            for s, f in zip(host, want):
                assert not f or int(O.filter_mask(s, q["filter"]).sum()) == 0, text
            got, st = pruning.process_query(q, gsegs, trim=False)
            ref, _ = plain.process_query(q, gsegs, trim=False)
            if q.get("group_by"):
                assert set(got) == set(ref) and all(_same(got[k], ref[k]) for k in got), text
            else:
                assert _same(got, ref), text
            assert st.num_segments_processed == len(host) - sum(want), text
        assert some_pruned >= 10, some_pruned
        for g in gsegs:
            g.release()
