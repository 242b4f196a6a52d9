"""DataTable bytes of device results (IntermediateResultsBlock.getDataTable, DataTableImplV2.toBytes) against the
oracle: aggregation tables byte for byte; group-by tables decoded (the broker's view) and compared map by map —
counts, sums, AvgPairs and HLL registers exact — including per-function trimmed maps and numGroupsLimitReached."""
import numpy as np
import pytest

import datatable as D
import pinot_oracle as O
from pinot_amd import GpuEngine, ServerQueryExecutor, build_segment, compile_pql

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = GpuEngine(0)
    yield e
    e.close()


def _oracle_value(f, v):
    if f == "AVG":
        return (float(v[0]), int(v[1]))
    if f == "DISTINCTCOUNTHLL":
        return [int(x) for x in v.reg]
    return v


def test_aggregation_datatable_bytes(engine, sv_segment, kats):
    g = engine.register(sv_segment)
    ex = ServerQueryExecutor(engine)
    for text in ("SELECT COUNT(*), SUM(column1), MAX(column3), MIN(column6), AVG(column7), DISTINCTCOUNTHLL(column9)"
                 " FROM testTable" + kats["filter"],
                 "SELECT COUNT(*), SUM(column1), AVG(column3) FROM testTable WHERE column1 < 0"):
        q = compile_pql(text)
        data, st = ex.process_query_datatable(q, [g], server=(1, 5, 42))
        exp, scanned = O.execute_server([sv_segment], q)
        assert st.num_docs_scanned == scanned
        stats = dict(num_docs_scanned=st.num_docs_scanned, num_entries_scanned_in_filter=st.num_entries_scanned_in_filter,
                     num_entries_scanned_post_filter=st.num_entries_scanned_post_filter,
                     num_total_raw_docs=st.num_total_raw_docs, num_segments_processed=st.num_segments_processed,
                     num_segments_matched=1 if scanned else 0)
        assert st.num_segments_matched == stats["num_segments_matched"]
        fns = [a["function"].upper() for a in q["aggregations"]]
        assert data == D.encode_aggregation(q, [_oracle_value(f, v) for f, v in zip(fns, exp)], stats,
                                            server=(1, 5, 42))
    g.release()


def _check_group_tables(d, q, exp):
    fns = [a["function"].upper() for a in q["aggregations"]]
    assert d["rows"] == len(fns) and [t for _, t in d["schema"]] == ["STRING", "OBJECT"]
    for i, (f, row) in enumerate(zip(fns, d["cells"])):
        assert row[0] == D.column_name(q["aggregations"][i])
        got = row[1]
        assert set(got) == set(exp), f
        for k, vals in exp.items():
            v = _oracle_value(f, vals[i])
            if f in ("SUM", "MIN", "MAX", "COUNT"):
                assert got[k] == v, (f, k)
            else:
                assert got[k] == v, (f, k)


def test_group_by_datatable_untrimmed(engine, sv_segment, kats):
    g = engine.register(sv_segment)
    ex = ServerQueryExecutor(engine)
    q = compile_pql("SELECT COUNT(*), SUM(column1), AVG(column3), MIN(column6), DISTINCTCOUNTHLL(column7) "
                    "FROM testTable" + kats["filter"] + " GROUP BY column11, column12")
    data, st = ex.process_query_datatable(q, [g], trim=False)
    exp, _ = O.execute_server([sv_segment], q)
    d = D.decode(data)
    _check_group_tables(d, q, exp)
    md = dict(d["metadata"])
    assert md["numDocsScanned"] == str(st.num_docs_scanned) and "numGroupsLimitReached" not in md
    assert d["dictionary"] == [("functionName", [(i, D.column_name(a)) for i, a in enumerate(q["aggregations"])])]
    g.release()


def test_group_by_datatable_trimmed_per_function_and_limit_flag(engine):
    # > 20,000 groups (4 x max(5 * topN, 5000)): each function's map holds its own trimmed groups
    rng = np.random.default_rng(11)
    n = 300_000
    seg = build_segment("dt", {"k": ("INT", rng.integers(0, 60_000, n).tolist()),
                               "m": ("INT", rng.integers(0, 1 << 20, n).tolist())})
    g = engine.register(seg)
    q = compile_pql("SELECT COUNT(*), SUM(m), MIN(m) FROM t GROUP BY k TOP 10")
    ex = ServerQueryExecutor(engine, num_groups_limit=50_000)
    res, st = ex.group_by_result(q, [g])
    keys = res.keys()
    data, _ = ex.process_query_datatable(q, [g], trim=True)
    d = D.decode(data)
    assert dict(d["metadata"])["numGroupsLimitReached"] == "true"  # groups >= num.groups.limit
    counts, sums = res.function_values(1)
    _, mins = res.function_values(2)
    for i, (f, row) in enumerate(zip(("COUNT", "SUM", "MIN"), d["cells"])):
        sel = res.trimmed_groups(10, i)
        assert len(sel) == 5000
        assert set(row[1]) == {keys[j] for j in sel}
        for j in sel[:500]:
            assert row[1][keys[j]] == (int(counts[j]) if f == "COUNT" else float(sums[j]) if f == "SUM" else
                                      float(mins[j]))
    exp, _ = O.execute_server([seg], q, num_groups_limit=50_000)
    assert len(exp) == len(keys)
    view, _ = ex.process_query_datatable(q, [g], trim=True, zero_copy=True)  # the native buffer, no copy
    assert isinstance(view, memoryview) and view.readonly and bytes(view) == data
    # two zero-copy views of one result (trimmed, then untrimmed): the second call must not free the first's bytes
    from pinot_amd import _lib
    from pinot_amd.executor import QueryMarshal
    m = QueryMarshal(q, 50_000, ex.max_init, ex.timeout_ms)
    v1 = res.data_table(m, _lib.ExecStats(), 10, None, True)
    c1 = bytes(v1)
    v2 = res.data_table(m, _lib.ExecStats(), None, None, True)
    c2 = bytes(v2)
    assert len(c2) > len(c1) and bytes(v1) == c1 and bytes(v2) == c2
    assert D.decode(c1)["cells"][0][1].keys() <= D.decode(c2)["cells"][0][1].keys()
    del res
    assert bytes(v1) == c1  # the views keep the result (and its buffers) alive
    g.release()


def test_broker_reduce_of_gpu_tables(engine, sv_segment, kats):
    """The reference's inter-segment KAT strings (2 servers x 2 segments) from GPU-built DataTables reduced by the
    library's pinot_broker_reduce (BrokerReduceService.reduceOnDataTable)."""
    from pinot_amd import BrokerReduce
    g = engine.register(sv_segment)
    ex = ServerQueryExecutor(engine)
    k = kats["inter_segment"]
    for case in k["cases"]:
        for variant, where, gb in (("unfiltered", "", ""), ("filtered", kats["filter"], ""),
                                   ("unfiltered_group_by", "", k["group_by"]),
                                   ("filtered_group_by", kats["filter"], k["group_by"])):
            q = compile_pql(case["query"] + where + gb)
            tables = [ex.process_query_datatable(q, [g, g], server=(2, 1, -1))[0] for _ in range(2)]
            resp = BrokerReduce.reduce_datatables(q, tables)
            got = [r["groupByResult"][0]["value"] if "groupByResult" in r else r["value"]
                   for r in resp["aggregationResults"]]
            assert got == case[variant], (case["query"], variant)
            exp = case["stats"][variant]
            assert [resp["numDocsScanned"], resp["numEntriesScannedPostFilter"], resp["totalDocs"]] == \
                [exp[0], exp[2], exp[3]], (case["query"], variant)
    g.release()
