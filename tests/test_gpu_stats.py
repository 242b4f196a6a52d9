"""numEntriesScannedInFilter with stats.exact=1 (csrc/filter_stats.cpp: the reference's iterator protocol replayed
over the device-computed leaf bitsets) against the reference's known answer and against oracle/iter_stats.py on
random trees over sorted, bitmap, scan, raw and multi-value leaves."""
import numpy as np
import pytest

import iter_stats
from conftest import build_segment, load_sv_columns
from pinot_amd import GpuEngine, ServerQueryExecutor, compile_pql
from test_gpu_parity import _random_segment, _random_tree
from test_mv import mv_segment

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = GpuEngine(0)
    e.set_config("stats.exact=1")
    yield e
    e.close()


def test_kat_entries_scanned_in_filter(engine, kats):
    """The reference's segment loads no bitmap inverted index (default IndexLoadingConfig): 84134 per segment,
    336536 over 2 servers x 2 segments (InterSegmentAggregationSingleValueQueriesTest)."""
    seg = build_segment("testTable_126164076_167572854", load_sv_columns())
    g = engine.register(seg)
    ex = ServerQueryExecutor(engine)
    for case in kats["inter_segment"]["cases"]:
        for variant, gb in (("filtered", ""), ("filtered_group_by", kats["inter_segment"]["group_by"])):
            _, st = ex.process_query(compile_pql(case["query"] + kats["filter"] + gb), [g, g])
            assert 2 * st.num_entries_scanned_in_filter == case["stats"][variant][1], (case["query"], variant)
    _, st = ex.process_query(compile_pql("SELECT COUNT(*) FROM t"), [g])
    assert st.num_entries_scanned_in_filter == 0
    g.release()


@pytest.mark.parametrize("seed", range(4))
def test_random_trees_match_the_oracle(engine, seed):
    rng = np.random.default_rng(1500 + seed)
    n = int(rng.choice([1, 64, 777, 5000]))
    seg = _random_segment(rng, n) if seed % 2 == 0 else mv_segment(rng, n)
    g = engine.register(seg)
    ex = ServerQueryExecutor(engine)
    for _ in range(12):
        tree = _random_tree(rng, seg)
        q = {"aggregations": [{"function": "COUNT", "column": "*"}], "filter": tree, "group_by": None}
        _, st = ex.process_query(q, [g])
        assert st.num_entries_scanned_in_filter == iter_stats.entries_scanned_in_filter(seg, tree), tree
    g.release()
