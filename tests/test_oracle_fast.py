"""The vectorised oracle group-by (execute_group_by_arrays, used for the 1M-key GPU parity tests) against the
per-group restatement execute_server, which tests/test_oracle_kats.py pins to the reference's known answers."""
import numpy as np
import pytest

import pinot_oracle as O
from pinot_amd.segment import build_segment


def _segments(rng, n, nseg, card0, card1, different_dicts=False):
    segs = []
    for i in range(nseg):
        shift = 3 * i if different_dicts else 0
        cols = {"g0": ("INT", (rng.integers(0, card0, n) + shift).tolist()),
                "g1": ("STRING", ["v%03d" % x for x in rng.integers(0, card1, n)]),
                "m": ("INT", rng.integers(-1000, 100000, n).tolist()),
                "d": ("DOUBLE", np.round(rng.normal(0, 100, n), 2).tolist()),
                "h": ("LONG", rng.integers(-2 ** 40, 2 ** 40, n // 7 + 1)[rng.integers(0, n // 7 + 1, n)].tolist())}
        segs.append(build_segment("s%d" % i, cols))
    return segs


QUERY = {"aggregations": [{"function": "COUNT", "column": "*"}, {"function": "SUM", "column": "m"},
                          {"function": "AVG", "column": "m"}, {"function": "MIN", "column": "d"},
                          {"function": "MAX", "column": "m"}, {"function": "DISTINCTCOUNTHLL", "column": "h"}],
         "filter": {"operator": "RANGE", "column": "m", "values": ["[0\t\t*)"]},
         "group_by": {"columns": ["g0", "g1"], "top_n": 10}}


def _compare(segs, q, limit, threshold):
    exp, scanned = O.execute_server(segs, q, num_groups_limit=limit) if threshold == 10000 else (None, None)
    if exp is None:
        per = []
        scanned = 0
        for s in segs:
            mask = O.filter_mask(s, q.get("filter"))
            scanned += int(mask.sum())
            per.append(O.group_by_segment(s, q, mask, num_groups_limit=limit, array_threshold=threshold))
        exp = O.combine_group_by(q, per, num_groups_limit=limit)
    got = O.execute_group_by_arrays(segs, q, num_groups_limit=limit, array_threshold=threshold)
    assert got["scanned"] == scanned
    keys = [O.key_string(got, int(k)) for k in got["keys"]]
    assert sorted(keys) == sorted(exp)
    for i, (a, r) in enumerate(zip(q["aggregations"], got["fns"])):
        f = a["function"].upper()
        for g, k in enumerate(keys):
            e = exp[k][i]
            if f == "COUNT":
                assert r["count"][g] == e
            elif f == "SUM":
                assert r["sum"][g] == e
            elif f == "AVG":
                assert (r["sum"][g], r["count"][g]) == e
            elif f == "MIN":
                assert abs(r["min"][g] - e) <= 1e-9 * max(1, abs(e))
            elif f == "MAX":
                assert r["max"][g] == e
            else:
                assert r["card"][g] == e.cardinality()
                assert (r["hll"][g].astype(np.int64) == e.reg).all()


@pytest.mark.parametrize("different_dicts", [False, True])
def test_fast_group_by_matches_restatement(different_dicts):
    rng = np.random.default_rng(5)
    segs = _segments(rng, 3000, 2, 40, 30, different_dicts)
    _compare(segs, QUERY, 100000, 10000)


def test_fast_group_by_admission_and_inter_segment_cap():
    """num.groups.limit first-appearance admission per segment and the 2 x limit cap across 3 segments."""
    rng = np.random.default_rng(9)
    segs = _segments(rng, 4000, 3, 60, 50, different_dicts=True)
    _compare(segs, QUERY, 150, 100)
    _compare(segs, QUERY, 1000, 100)


def test_cardinality_np_matches_scalar():
    from hll import cardinality
    rng = np.random.default_rng(3)
    regs = np.zeros((50, 256), dtype=np.uint8)
    for i in range(50):
        k = int(rng.integers(0, 257))
        regs[i, rng.choice(256, k, replace=False)] = rng.integers(1, 26, k)
    regs[0] = 1  # no zero registers, small estimate: linear counting of log(256 / 0) = Long.MAX_VALUE
    got = O.cardinality_np(regs)
    assert [int(x) for x in got] == [cardinality(r) for r in regs]
