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
