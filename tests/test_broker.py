"""Broker reduce over DataTable bytes (BrokerReduceService.reduceOnDataTable): the library's pinot_broker_reduce —
host code, no GPU — against the oracle (oracle/broker.py), both pinned by the reference's
InterSegmentAggregationSingleValueQueriesTest strings: each case's value is what the broker prints for 2 servers x
2 segments of the test table. GPU-produced DataTables: tests/test_gpu_datatable.py::test_broker_reduce_of_gpu_tables."""
import math

import numpy as np
import pytest

import broker as B
import datatable as D
import pinot_oracle as O
from pinot_amd import BrokerReduce, compile_pql

STATS = dict(num_docs_scanned=100, num_entries_scanned_in_filter=7, num_entries_scanned_post_filter=300,
             num_total_raw_docs=1000, num_segments_processed=2, num_segments_matched=1)


def _oracle_value(f, v):
    if f == "AVG":
        return (float(v[0]), int(v[1]))
    if f == "DISTINCTCOUNTHLL":
        return [int(x) for x in v.reg]
    return v


def _tables(q, server_result, copies=2, stats=STATS, server=(2, 1, -1)):
    fns = [a["function"].upper() for a in q["aggregations"]]
    if q.get("group_by"):
        res = {k: [_oracle_value(f, x) for f, x in zip(fns, v)] for k, v in server_result.items()}
        return [D.encode_group_by(q, res, stats, server) for _ in range(copies)]
    vals = [_oracle_value(f, v) for f, v in zip(fns, server_result)]
    return [D.encode_aggregation(q, vals, stats, server) for _ in range(copies)]


def _first_values(resp):
    out = []
    for r in resp["aggregationResults"]:
        out.append(r["groupByResult"][0]["value"] if "groupByResult" in r else r["value"])
    return out


def test_inter_segment_kats_through_datatables(sv_segment, kats):
    k = kats["inter_segment"]
    for case in k["cases"]:
        for variant, where, gb in (("unfiltered", "", ""), ("filtered", kats["filter"], ""),
                                   ("unfiltered_group_by", "", k["group_by"]),
                                   ("filtered_group_by", kats["filter"], k["group_by"])):
            q = compile_pql(case["query"] + where + gb)
            server, _ = O.execute_server([sv_segment, sv_segment], q)
            tables = _tables(q, server)
            assert _first_values(B.reduce(q, tables)) == case[variant], (case["query"], variant)
            native = BrokerReduce.reduce_datatables(q, tables)
            assert _first_values(native) == case[variant], (case["query"], variant)
            assert native["numDocsScanned"] == 2 * STATS["num_docs_scanned"]
            assert native["totalDocs"] == 2 * STATS["num_total_raw_docs"]
            assert native["numSegmentsQueried"] == 4 and native["numServersResponded"] == 2


@pytest.mark.parametrize("v", [0.015625, 1.005, 2.675, -0.000001, -0.000005, 0.000005, 123.456789, 1e-7, -0.0, 0.0,
                               2.0 ** 63, 2.0 ** 64, -1e300, 1e20 + 0.5, 9.5, 1e15 + 0.25, 0.1 + 0.2, 99999.999995,
                               math.inf, -math.inf, math.nan, 5e-324, 1.7976931348623157e308])
def test_format_value_matches_oracle(v):
    q = compile_pql("SELECT SUM(m), MIN(m) FROM t")
    tables = [D.encode_aggregation(q, [v, v], STATS)]
    native = BrokerReduce.reduce_datatables(q, tables)
    want = B.format_double(v)
    assert [r["value"] for r in native["aggregationResults"]] == [want, want]


def test_known_java_formats():
    # AggregationFunctionUtils.formatValue: whole numbers (long) + ".00000"; (long) saturates at Long.MAX / MIN
    assert B.format_double(3.0) == "3.00000" and B.format_double(-0.0) == "0.00000"
    assert B.format_double(2.0 ** 63) == "9223372036854775807.00000"
    assert B.format_double(-1e300) == "-9223372036854775808.00000"
    # %1.5f: HALF_UP on the shortest digits (0.015625 -> 0.01563; C's printf would give 0.01562)
    assert B.format_double(0.015625) == "0.01563" and B.format_double(1.005) == "1.00500"
    assert B.format_double(-0.000001) == "-0.00000"
    assert B.format_double(math.inf) == "Infinity" and B.format_double(-math.inf) == "-Infinity"


def test_random_group_by_reduce_matches_oracle():
    rng = np.random.default_rng(8)
    q = compile_pql("SELECT COUNT(*), SUM(m), MIN(m), MAX(m), AVG(m), DISTINCTCOUNTHLL(m) FROM t GROUP BY a, b TOP 7")
    tables = []
    for s in range(3):
        res = {}
        for _ in range(int(rng.integers(0, 40))):
            key = "%d\t%s" % (rng.integers(0, 12), ["x", "", "yy"][int(rng.integers(0, 3))])
            regs = [int(x) for x in rng.integers(0, 9, 256)]
            res[key] = [int(rng.integers(1, 50)), float(rng.integers(-500, 500)) / 8, float(rng.integers(-90, 90)) / 4,
                        float(rng.integers(-90, 90)) / 4, (float(rng.integers(-99, 99)) / 3, int(rng.integers(1, 9))),
                        regs]
        st = dict(STATS, num_docs_scanned=int(rng.integers(0, 1000)))
        tables.append(D.encode_group_by(q, res, st, (1, 0, -1)) if res or s else D.encode_empty(q, 10))
    want = B.reduce(q, tables, top_n=7)
    got = BrokerReduce.reduce_datatables(q, tables)
    assert got["aggregationResults"] == want["aggregationResults"]
    for k in ("numDocsScanned", "numEntriesScannedInFilter", "numEntriesScannedPostFilter", "numSegmentsProcessed",
              "numSegmentsMatched", "totalDocs", "numSegmentsQueried", "numGroupsLimitReached"):
        assert got[k] == want[k], k


def test_empty_and_malformed_tables():
    q = compile_pql("SELECT COUNT(*), MIN(m), AVG(m) FROM t")
    resp = BrokerReduce.reduce_datatables(q, [D.encode_empty(q, 55), D.encode_empty(q, 45)])
    assert [r["value"] for r in resp["aggregationResults"]] == ["0", "Infinity", "-Infinity"]
    assert resp["totalDocs"] == 100 and resp["numSegmentsProcessed"] == 0
    assert BrokerReduce.reduce_datatables(q, [])["aggregationResults"] == []
    from pinot_amd import PinotGpuError
    good = D.encode_empty(q, 5)
    for bad in (good[:30], good[:-3], b"\x00\x00\x00\x03" + good[4:]):
        with pytest.raises(PinotGpuError):
            BrokerReduce.reduce_datatables(q, [bad])
