"""Star-tree v2 on the host: the builder's tree (BaseSingleTreeBuilder restated, tests/startree_writer.py) and the
oracle's star-tree plan (oracle/startree.py) answer every fitting query exactly as the scan plan does — the
pre-aggregation's defining property — over random filters (EQ / IN / NOT / NOT_IN / RANGE, AND-only), group-bys on
split-order dimensions, skip-star dimensions and leaf sizes; the serialized tree reads back."""
import struct

import numpy as np
import pytest

import pinot_oracle as O
import startree as S
from pinot_amd import build_segment
from startree_writer import MAGIC, build_star_tree

DIMS = ["a", "b", "c"]
PAIRS = [("COUNT", "*"), ("SUM", "m"), ("MIN", "m"), ("MAX", "x"), ("SUM", "x"), ("AVG", "m"),
         ("DISTINCTCOUNTHLL", "c")]


def st_segment(rng, n, name="st"):
    cols = {"a": ("INT", rng.integers(0, 4, n).astype(np.int32)),
            "b": ("STRING", np.array(["b%d" % v for v in rng.integers(0, 9, n)], dtype=object)),
            "c": ("INT", rng.integers(0, 30, n).astype(np.int32) * 3),
            "m": ("INT", rng.integers(-500, 1000, n).astype(np.int32)),
            "x": ("LONG", rng.integers(0, 1 << 40, n).astype(np.int64))}
    return build_segment(name, cols, allow_sorted=False)


def random_query(rng, seg, group=None):
    leaves = []
    for c in rng.choice(DIMS, size=int(rng.integers(0, 3)), replace=False):
        vals = seg.column(c).dict_values()
        lit = lambda: str(vals[int(rng.integers(0, len(vals)))])  # noqa: E731
        op = rng.choice(["EQUALITY", "IN", "NOT", "NOT_IN", "RANGE"])
        if op in ("IN", "NOT_IN"):
            v = "\t\t".join(lit() for _ in range(int(rng.integers(1, 4))))
        elif op == "RANGE":
            a, b = sorted([lit(), lit()], key=lambda s: (int(s) if s.lstrip("-").isdigit() else s))
            v = "[%s\t\t%s]" % (a, b)
        else:
            v = lit()
        leaves.append({"operator": op, "column": c, "values": [v]})
    flt = None if not leaves else leaves[0] if len(leaves) == 1 else {"operator": "AND", "children": leaves}
    idx = rng.choice(len(PAIRS), size=int(rng.integers(1, 4)), replace=False)
    aggs = [{"function": PAIRS[i][0], "column": PAIRS[i][1]} for i in idx]
    return {"aggregations": aggs, "filter": flt,
            "group_by": {"columns": group, "top_n": 10} if group else None}


def _same(q, got, exp):
    if q["group_by"]:
        assert set(got) == set(exp)
        pairs = [(got[k], exp[k]) for k in exp]
    else:
        pairs = [(got, exp)]
    for g, e in pairs:
        for a, x, y in zip(q["aggregations"], g, e):
            if a["column"] == "x" and a["function"] == "SUM":
                assert x == pytest.approx(y, rel=1e-12)
            elif a["function"] == "DISTINCTCOUNTHLL":
                assert x.cardinality() == y.cardinality(), (q, a)
                if hasattr(x, "reg"):
                    assert list(x.reg) == list(y.reg), (q, a)
            elif a["function"] == "AVG":
                xs, xc = (x.sum, x.count) if hasattr(x, "sum") else x
                assert (xs, xc) == tuple(y), (q, a)
            else:
                assert x == y, (q, a)


@pytest.mark.parametrize("seed,leaf,skip", [(0, 10, ()), (1, 1, ()), (2, 50, ("b",)), (3, 10000, ()), (4, 3, ("a", "c"))])
def test_star_tree_equals_scan(seed, leaf, skip):
    rng = np.random.default_rng(seed)
    seg = st_segment(rng, int(rng.choice([1, 17, 400, 3000])))
    st = build_star_tree(seg, DIMS, PAIRS, max_leaf_records=leaf, skip_star=skip)
    for it in range(30):
        group = [None, ["a"], ["b", "c"], ["c", "a", "b"]][it % 4]
        q = random_query(rng, seg, group)
        assert S.fits(st, q)
        got, _ = S.execute_segment(seg, st, q)
        exp, _ = O.execute_segment(seg, q)
        _same(q, got, exp)


def test_fit_rules_and_tree_bytes():
    rng = np.random.default_rng(9)
    seg = st_segment(rng, 500)
    st = build_star_tree(seg, DIMS, PAIRS, max_leaf_records=5)
    q = {"aggregations": [{"function": "AVG", "column": "x"}], "filter": None, "group_by": None}
    assert not S.fits(st, q)  # no avg__x pair
    q = {"aggregations": [{"function": "DISTINCTCOUNTHLL", "column": "m"}], "filter": None, "group_by": None}
    assert not S.fits(st, q)  # no distinctCountHLL__m pair
    q = {"aggregations": [{"function": "SUM", "column": "m"}], "group_by": None,
         "filter": {"operator": "OR", "children": [{"operator": "EQUALITY", "column": "a", "values": ["1"]},
                                                   {"operator": "EQUALITY", "column": "a", "values": ["2"]}]}}
    assert not S.fits(st, q)  # OR
    q = {"aggregations": [{"function": "SUM", "column": "m"}], "filter": None,
         "group_by": {"columns": ["m"], "top_n": 10}}
    assert not S.fits(st, q)  # group-by on a non-dimension
    b = st.tree_bytes
    magic, version, header, ndims = struct.unpack_from("<Qiii", b, 0)
    assert (magic, version, ndims) == (MAGIC, 1, 3)
    nnodes = struct.unpack_from("<i", b, header - 4)[0]
    assert len(b) == header + 28 * nnodes == header + 28 * st.nodes.shape[0]
    root = struct.unpack_from("<7i", b, header)
    assert root[0] == -1 and root[5] == 1  # root: ALL, first child is node 1 (BFS)
    # a star-tree is much smaller than the segment and the unfiltered COUNT is one aggregated doc
    q = {"aggregations": [{"function": "COUNT", "column": "*"}], "filter": None, "group_by": None}
    res, scanned = S.execute_segment(seg, st, q)
    assert res == [500] and scanned == 1


def test_hll_bytes_layout():
    """HyperLogLog.getBytes as DataTable's serializer writes it (datatable.cpp) and the star-tree stores it."""
    from startree_writer import hll_bytes
    regs = np.zeros(256, dtype=np.uint8)
    regs[0], regs[5], regs[6], regs[255] = 3, 31, 1, 7
    b = hll_bytes(regs)
    assert len(b) == 180 and struct.unpack_from(">ii", b, 0) == (8, 172)
    w = struct.unpack_from(">43i", b, 8)
    assert w[0] == 3 | (31 << 25) and w[1] == 1 and w[42] == 7 << 15
