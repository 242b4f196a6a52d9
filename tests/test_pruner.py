"""Segment pruning (SegmentPrunerService.prune with the server's default pruners) and the all-pruned DataTable.

The oracle (oracle/pruner.py) is pinned by the reference's ColumnValueSegmentPrunerTest.test
(pinot-core/src/test/java/org/apache/pinot/query/pruner/ColumnValueSegmentPrunerTest.java:53-92): every one of its
assertions is replayed below against the oracle and against the library's pinot_segment_prune (host code: no GPU).
Randomized segments and filters then check native == oracle, and that a pruned segment never holds a matching doc.
GPU-registered segments and the executor path: tests/test_gpu_pruner.py."""
import math

import numpy as np
import pytest

import bloom as B
import datatable as D
import pinot_oracle as O
import pruner as P
from pinot_amd import PinotGpuError, build_segment, compile_pql, empty_datatable, prune_segment

BAD_QUERY = 5

# ColumnValueSegmentPrunerTest.java:53-92 (query WHERE clause, expected prune)
KAT = [
    ("foo = 'bar'", False),
    ("time = 0", True), ("time = 10", False), ("time = 20", False), ("time = 30", True),
    ("time < 10", True), ("time <= 10", False), ("time >= 10", False), ("time > 20", True),
    ("time BETWEEN 20 AND 30", False), ("time BETWEEN 30 AND 40", True),
    ("time BETWEEN 20 AND 10", True), ("time BETWEEN 30 AND 20", True), ("time BETWEEN 10 AND 10", False),
    ("time BETWEEN 20 AND 20", False),
    ("time = 0 AND time > 10", True), ("time > 0 AND time < 10", True), ("time >= 0 AND time <= 10", False),
    ("time > 20 AND time < 10", True), ("time >= 20 AND time < 30", False), ("time > 0 AND time BETWEEN 0 AND 10", False),
    ("time = 0 OR time > 10", False), ("time = 0 OR time < 10", True), ("time >= 0 OR time <= 10", False),
    ("time > 30 OR time < 10", True), ("time BETWEEN 0 AND 5 OR time BETWEEN 30 AND 35", True),
]


def _q(where, select="COUNT(*)"):
    return compile_pql("SELECT %s FROM table%s" % (select, " WHERE " + where if where else ""))


def test_reference_kat_oracle():
    # the test's metadata: time INT [10, 20]; foo STRING without min / max
    seg = {"num_docs": 100, "columns": {"time": ("INT", 10, 20), "foo": ("STRING", None, None)}}
    for where, want in KAT:
        assert P.column_value_prune(_q(where)["filter"], seg["columns"]) == want, where
        assert P.prune(seg, _q(where)) == want, where


def test_reference_kat_native():
    # the test's metadata: time minValue 10 / maxValue 20, foo none (ColumnValueSegmentPrunerTest.java:44-51)
    seg = build_segment("kat", {"time": ("INT", np.arange(10, 21, dtype=np.int32)),
                                "foo": ("STRING", np.array(["bar"] * 11, dtype=object))}, min_max=("time",))
    assert seg.columns["time"].min_value == "10" and seg.columns["foo"].min_value is None
    for where, want in KAT:
        assert prune_segment(seg, _q(where)) == want, where
        assert prune_segment(seg, _q(where), pruners=P.COLUMN_VALUE) == want, where
        assert not prune_segment(seg, _q(where), pruners=P.DATA_SCHEMA | P.VALID), where


def _random_segment(rng, n, name):
    cols = {
        "i": ("INT", rng.integers(int(rng.integers(-100, 50)), int(rng.integers(60, 200)), n).astype(np.int32)),
        "l": ("LONG", rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64) // (1 << int(rng.integers(20, 40)))),
        "f": ("FLOAT", (rng.integers(-40, 40, n) * 0.25).astype(np.float32)),
        "d": ("DOUBLE", rng.integers(int(rng.integers(-90, 0)), int(rng.integers(1, 90)), n) * 0.1),
        "s": ("STRING", np.array(["k%02d" % v for v in rng.integers(int(rng.integers(0, 40)), 80, n)], dtype=object)),
    }
    # bloom filters and partition metadata on some columns (ColumnValueSegmentPruner's bloom test,
    # PartitionSegmentPruner); each function / type pairing the creator accepts
    bloom = [c for c in "ilfds" if rng.integers(0, 2)]
    parts = {}
    for c, fns in (("i", ("Modulo", "Murmur", "HashCode", "ByteArray")), ("l", ("Murmur", "HashCode", "ByteArray")),
                   ("f", ("HashCode", "Murmur")), ("d", ("HashCode", "ByteArray")),
                   ("s", ("Murmur", "ByteArray", "HashCode"))):
        if rng.integers(0, 2):
            parts[c] = (fns[int(rng.integers(0, len(fns)))], int(rng.integers(2, 9)))
    return build_segment(name, cols, min_max=True, bloom_columns=bloom, partitions=parts)


def _literal(rng, seg, col):
    c = seg.columns[col]
    vals = c.dict_values()
    card = len(vals)  # a raw column: its sorted distinct values
    pick = rng.integers(0, 4)
    if pick == 0:  # a dictionary value
        v = vals[int(rng.integers(0, card))]
    elif pick == 1:  # just outside
        v = vals[0] if rng.integers(0, 2) else vals[card - 1]
        if c.data_type == "STRING":
            return v[:-1] if rng.integers(0, 2) else v + "z"
        v = v - 1 if rng.integers(0, 2) else v + 1
    else:  # anywhere
        if c.data_type == "STRING":
            return "k%02d" % rng.integers(-5, 90)
        v = rng.integers(-300, 300) * (0.25 if c.data_type in ("FLOAT", "DOUBLE") else 1)
    if c.data_type in ("INT", "LONG"):
        return str(int(v))
    if c.data_type in ("FLOAT", "DOUBLE"):
        return repr(float(v))
    return str(v)


def _leaf(rng, seg):
    col = "ilfds"[int(rng.integers(0, 5))]
    kind = int(rng.integers(0, 5))
    a, b = _literal(rng, seg, col), _literal(rng, seg, col)
    if kind == 0:
        return {"operator": "EQUALITY", "column": col, "values": [a]}
    if kind == 1:
        return {"operator": "NOT", "column": col, "values": [a]}
    if kind == 2:
        return {"operator": "IN", "column": col, "values": [a, b]}
    lo = "*" if rng.integers(0, 4) == 0 else a
    hi = "*" if rng.integers(0, 4) == 0 else b
    return {"operator": "RANGE", "column": col,
            "values": ["%s%s\t\t%s%s" % ("[(" [int(rng.integers(0, 2))], lo, hi, "])"[int(rng.integers(0, 2))])]}


def _tree(rng, seg, depth=0):
    if depth >= 2 or rng.integers(0, 3) == 0:
        return _leaf(rng, seg)
    return {"operator": "AND" if rng.integers(0, 2) else "OR",
            "children": [_tree(rng, seg, depth + 1) for _ in range(int(rng.integers(2, 4)))]}


def test_random_native_matches_oracle_and_is_sound():
    rng = np.random.default_rng(2024)
    pruned_seen = kept_seen = 0
    for k in range(12):
        seg = _random_segment(rng, 400, "r%d" % k)
        rs = P.ranges(seg)
        for _ in range(40):
            q = {"aggregations": [{"function": "COUNT", "column": "*"}], "filter": _tree(rng, seg), "group_by": None}
            want = P.prune(rs, q)
            assert prune_segment(seg, q) == want, q
            if want:
                pruned_seen += 1
                assert int(O.filter_mask(seg, q["filter"]).sum()) == 0, q  # pruning never drops a match
            else:
                kept_seen += 1
    assert pruned_seen > 50 and kept_seen > 50, (pruned_seen, kept_seen)


def test_data_schema_and_valid_pruners():
    seg = build_segment("s", {"a": ("INT", np.arange(5, dtype=np.int32)), "b": ("LONG", np.arange(5) * 7)})
    assert not prune_segment(seg, _q(None))
    assert prune_segment(seg, _q("zz = 1"))                    # filter column missing
    assert prune_segment(seg, _q(None, "SUM(zz)"))            # aggregation column missing
    assert not prune_segment(seg, _q(None, "COUNT(zz)"))      # COUNT's column is never required
    assert prune_segment(seg, compile_pql("SELECT SUM(a) FROM t GROUP BY zz"))
    assert not prune_segment(seg, _q("zz = 1"), pruners=0)
    # ColumnValue alone: an EQUALITY / RANGE leaf on a missing column prunes, any other leaf does not
    assert prune_segment(seg, _q("zz = 1"), pruners=P.COLUMN_VALUE)
    assert not prune_segment(seg, _q("zz <> 1"), pruners=P.COLUMN_VALUE)
    for q in ("zz = 1", "zz <> 1"):
        assert P.prune({"num_docs": 5, "columns": P.ranges(seg)["columns"]}, _q(q), P.COLUMN_VALUE) == \
            prune_segment(seg, _q(q), pruners=P.COLUMN_VALUE)
    empty = build_segment("e", {"a": ("INT", np.arange(5, dtype=np.int32))}, num_docs=0, min_max=True)
    assert prune_segment(empty, _q(None)) and P.prune(P.ranges(empty), _q(None))
    assert not prune_segment(empty, _q(None), pruners=P.DATA_SCHEMA | P.COLUMN_VALUE)


def test_literals_and_java_compare():
    seg = build_segment("t", {"f": ("FLOAT", np.array([-0.0, 1.5, 2.5], dtype=np.float32)),
                              "d": ("DOUBLE", np.array([-2.0, 0.5, 0.5])),
                              "i": ("INT", np.array([3, 9, 9], dtype=np.int32))}, min_max=True)
    rs = P.ranges(seg)
    def eq(c, v):
        return {"aggregations": [{"function": "COUNT", "column": "*"}], "group_by": None,
                "filter": {"operator": "EQUALITY", "column": c, "values": [v]}}

    def rng_(c, v):
        return {"aggregations": [{"function": "COUNT", "column": "*"}], "group_by": None,
                "filter": {"operator": "RANGE", "column": c, "values": [v]}}

    cases = [_q(w) for w in ("f = 1.5", "f = 2.50000001", "f = 2.6", "f = 0.0", "f < -0.0", "f <= -0.0",
                             "d >= 0.50000001", "d BETWEEN -1e308 AND -2.0", "i = 2147483647",
                             "i > 8 AND i < 10", "f > 1e39")]
    cases += [eq("f", "2.5f"), eq("d", "0.5d"), eq("d", " 0.5 "), eq("d", "Infinity"), eq("d", "-Infinity"),
              eq("f", "NaN"), eq("i", "+3"), eq("i", "-0"), rng_("d", "(*\t\tNaN)"), rng_("f", "(-0.0\t\t0.0)"),
              rng_("f", "[-0.0\t\t0.0]"), rng_("i", "(9\t\t*)"), rng_("i", "[9\t\t*)")]
    for q in cases:
        assert prune_segment(seg, q) == P.prune(rs, q), q
    for bad in (_q("i = 3.5"), _q("i = 'abc'"), _q("i = 2147483648"), _q("d = 'x'"), _q("i BETWEEN 1 AND 2e3"),
                eq("i", " 3"), eq("d", "inf"), eq("d", "nan")):
        with pytest.raises(PinotGpuError) as ei:
            prune_segment(seg, bad)
        assert ei.value.status == BAD_QUERY, bad
        with pytest.raises(P.BadQuery):
            P.prune(rs, bad)
    # NOT / IN leaves never parse their literals in the pruner (no BadQuery there)
    assert not prune_segment(seg, _q("i <> 'abc'"))


@pytest.mark.parametrize("select,group", [
    ("COUNT(*), SUM(m), MIN(m), MAX(m), AVG(m), DISTINCTCOUNTHLL(m)", ""),
    ("COUNT(*)", ""),
    ("SUM(m), COUNT(*), AVG(m), SUM(m)", " GROUP BY a, b"),
    ("DISTINCTCOUNTHLL(m), MIN(m)", " GROUP BY a"),
])
@pytest.mark.parametrize("server", [None, (4, 17, -1), (12, 3, 987654321)])
def test_empty_datatable_bytes(select, group, server):
    q = compile_pql("SELECT %s FROM t WHERE a = 5%s" % (select, group))
    got = empty_datatable(q, 123456789, server)
    assert got == D.encode_empty(q, 123456789, server)
    t = D.decode(got)
    md = dict(t["metadata"])
    assert md["totalDocs"] == "123456789" and md["numDocsScanned"] == "0" and md["numSegmentsProcessed"] == "0"
    if group:
        assert t["rows"] == len(q["aggregations"]) and all(c[1] == {} for c in t["cells"])
    else:
        row = t["cells"][0]
        fns = [a["function"] for a in q["aggregations"]]
        for f, v in zip(fns, row):
            want = {"COUNT": 0, "SUM": 0.0, "MIN": math.inf, "MAX": -math.inf, "AVG": (0.0, 0),
                    "DISTINCTCOUNTHLL": [0] * 256}[f]
            assert v == want, f


def test_raw_columns_host_checks_and_pruning():
    from pinot_amd import validate_segment
    from pinot_amd.segment import Column
    rng = np.random.default_rng(31)
    vals = {"i": ("INT", rng.integers(-70, 70, 900).astype(np.int32)),
            "l": ("LONG", rng.integers(-(1 << 50), 1 << 50, 900)),
            "f": ("FLOAT", (rng.integers(-40, 40, 900) * 0.25).astype(np.float32)),
            "d": ("DOUBLE", rng.integers(-400, 400, 900) * 0.125),
            "s": ("STRING", np.array(["k%02d" % v for v in rng.integers(0, 80, 900)], dtype=object))}
    seg = build_segment("raw", vals, raw_columns=("i", "l", "f", "d"), min_max=True)
    validate_segment(seg)  # the transcoding runs on the host
    rs = P.ranges(seg)
    for c in "ilfd":
        v = vals[c][1]
        assert rs["columns"][c][1] == v.min() and rs["columns"][c][2] == v.max()
    pruned = 0
    for _ in range(80):
        q = {"aggregations": [{"function": "COUNT", "column": "*"}], "filter": _tree(rng, seg), "group_by": None}
        want = P.prune(rs, q)
        assert prune_segment(seg, q) == want, q
        pruned += want
    assert pruned > 5
    short = build_segment("short", {"l": vals["l"]}, raw_columns=("l",))
    short.columns["l"].fwd = short.columns["l"].fwd[:-8]
    with pytest.raises(PinotGpuError) as ei:
        validate_segment(short)
    assert ei.value.status == 1
    s = build_segment("s", {"s": ("INT", [[1, 2], [3]])}, mv_columns=("s",))  # raw multi-value: not served
    s.columns["s"].encoding = "raw"
    with pytest.raises(PinotGpuError) as ei:
        validate_segment(s)
    assert ei.value.status == 4
    s = build_segment("s", {"s": ("STRING", np.array(["x", "y"], dtype=object))}, raw_columns=("s",))
    validate_segment(s)  # raw (var-byte) STRING: transcoded



def test_columns_without_min_max_never_prune_by_value():
    """The segment creator writes no minValue / maxValue; without them ColumnValueSegmentPruner keeps the segment
    (ColumnValueSegmentPruner.java:124-127, :170-173) — only the invalid-range test still prunes."""
    seg = build_segment("n", {"a": ("INT", np.arange(10, 21, dtype=np.int32))})
    assert seg.columns["a"].min_value is None
    for where, want in (("a = 0", False), ("a > 100", False), ("a BETWEEN 20 AND 10", True), ("a < 5", False)):
        assert prune_segment(seg, _q(where)) == want, where
        assert P.prune(P.ranges(seg), _q(where)) == want, where
    bad = build_segment("b", {"a": ("INT", np.arange(3, dtype=np.int32))}, min_max=True)
    bad.columns["a"].min_value = "x"
    with pytest.raises(PinotGpuError) as ei:
        prune_segment(bad, _q("a = 1"))
    assert ei.value.status == 1


# ---------------------------------------------------------------- bloom filters (ColumnValueSegmentPruner :140-144)
def test_bloom_filter_util_kats():
    # BloomFilterCreatorTest.testBloomFilterUtil (pinot-core/src/test/.../BloomFilterCreatorTest.java:49-67)
    assert B.compute_num_bits(1000000, 0.03) == 7298441
    assert B.compute_num_bits(10000000, 0.03) == 72984409
    assert B.compute_num_bits(10000000, 0.1) == 47925292
    assert B.compute_num_hash_functions(1000000, 7298441) == 5
    assert B.compute_num_hash_functions(10000000, 72984409) == 5
    assert B.compute_num_hash_functions(10000000, 47925292) == 3
    assert abs(B.compute_max_false_pos_probability(1000000, 5, 7298441) - 0.03) < 0.001
    assert abs(B.compute_max_false_pos_probability(10000000, 5, 72984409) - 0.03) < 0.001
    assert abs(B.compute_max_false_pos_probability(10000000, 3, 47925292) - 0.1) < 0.001


def test_bloom_filter_creator_kats():
    # BloomFilterCreatorTest.testBloomFilterCreator (:70-97): "0".."4" added to a cardinality-10000 filter
    bf = B.BloomFilter.for_cardinality(10000)
    for i in range(5):
        bf.put(str(i))
    back = B.BloomFilter.from_bytes(bf.to_bytes())
    assert all(back.might_contain(str(i)) for i in range(5))
    assert not any(back.might_contain(str(j)) for j in range(5, 10))
    # testBloomFilterSize (:99-121): at most 1 MB + Guava's 12-byte overhead (+ Pinot's 8-byte header)
    for card in (10, 100, 1000, 100000, 1000000, 5000000, 10000000):
        f = B.BloomFilter.for_cardinality(card)
        assert 8 * len(f.words) + 6 < 1024 * 1024 + 12, card
    # MurmurHash3_x64_128 of "hello" (seed 0): the widely published (h1, h2) pair
    assert B.murmur3_x64_128(b"hello") == (0xcbd8a7b341bd9b02, 0x5b1e906a48ae1d19)
    assert B.murmur3_x64_128(b"") == (0, 0)


def test_bloom_filter_prunes_inside_the_min_max_range():
    vals = np.arange(0, 1000, 10, dtype=np.int32)  # every 10th value: min / max never rule out the gaps
    seg = build_segment("b", {"x": ("INT", vals), "y": ("STRING", np.array(["v%d" % v for v in vals], dtype=object))},
                        min_max=True, bloom_columns=("x", "y"))
    rs = P.ranges(seg)
    gaps = kept = 0
    for v in range(-5, 1005):
        for q in (_q("x = %d" % v), _q("y = 'v%d'" % v)):
            want = P.prune(rs, q)
            assert prune_segment(seg, q) == want, (v, q)
            if v % 10 == 0 and 0 <= v < 1000:
                assert not want, v  # no false negatives
                kept += 1
            elif want:
                gaps += 1
    assert kept == 200 and gaps > 1600, gaps  # a 5 % false-positive filter rules out most gaps
    # the same filter handed over as .bloom bytes (BloomFilterReader) gives the same answers, and so does a
    # MURMUR128_MITZ_32 (ordinal 0) filter read from bytes
    for strategy in (1, 0):
        bf = B.BloomFilter.for_cardinality(len(vals))
        bf.strategy = strategy
        for v in vals:
            bf.put(str(int(v)))
        seg.columns["x"].create_bloom_filter = False
        seg.columns["x"].bloom_filter = bf.to_bytes()
        rs = P.ranges(seg)
        for v in range(-5, 1005, 3):
            assert prune_segment(seg, _q("x = %d" % v)) == P.prune(rs, _q("x = %d" % v)), (strategy, v)


def test_bloom_filter_rejects_malformed_bytes():
    seg = build_segment("b", {"x": ("INT", np.arange(10, dtype=np.int32))})
    good = B.BloomFilter.for_cardinality(10).to_bytes()
    for bad in (good[:10], b"\x00\x00\x00\x02" + good[4:], good[:4] + b"\x00\x00\x00\x02" + good[8:],
                good[:8] + b"\x05" + good[9:], good[:-8]):
        seg.columns["x"].bloom_filter = bad
        with pytest.raises(PinotGpuError):
            prune_segment(seg, _q("x = 3"))


# ---------------------------------------------------------------- PartitionSegmentPruner (:73-111)
def test_partition_functions_java_semantics():
    assert B.java_string_hash("abc") == 96354 and B.java_string_hash("hello") == 99162322
    assert B.partition_of("Modulo", 4, "INT", -7, "-7") == -3          # Java % keeps the sign: never held
    assert B.partition_of("modulo", 4, "STRING", "13", "13") == 1
    assert B.partition_of("HashCode", 5, "INT", -(1 << 31), str(-(1 << 31))) == -3  # abs(MIN_VALUE) stays negative
    assert B.partition_of("ByteArray", 5, "INT", 0, "0") == (31 + 48) % 5
    with pytest.raises(ValueError):
        B.partition_of("Modulo", 4, "LONG", 5, "5")


def test_partition_pruner_native_matches_oracle():
    rng = np.random.default_rng(77)
    n = 300
    checked = pruned = 0
    for fn, dt, vals in (("Modulo", "INT", rng.integers(-50, 50, n)), ("Murmur", "INT", rng.integers(0, 1000, n)),
                         ("HashCode", "LONG", rng.integers(-(1 << 40), 1 << 40, n)),
                         ("ByteArray", "STRING", ["p%d" % v for v in rng.integers(0, 30, n)]),
                         ("HashCode", "DOUBLE", rng.integers(-20, 20, n) * 0.5),
                         ("Murmur", "FLOAT", (rng.integers(-20, 20, n) * 0.25).astype(np.float32)),
                         ("HashCode", "STRING", ["h%d" % v for v in rng.integers(0, 30, n)])):
        for nparts in (3, 8):
            # a segment holding only the values of some partitions (a partitioned table's segment)
            keep = [v for v in vals if B.partition_of(fn, nparts, dt, v.item() if hasattr(v, "item") else v,
                                                     P.java_to_string(dt, v.item() if hasattr(v, "item") else v))
                    in (0, 1) or fn == "Modulo"]
            col = np.array(keep, dtype=object) if dt == "STRING" else np.asarray(keep)
            seg = build_segment("p", {"c": (dt, col)}, partitions={"c": (fn, nparts)})
            rs = P.ranges(seg)
            cand = list(dict.fromkeys(list(vals[:40]) + list(keep[:10])))
            for v in cand:
                lit = ("'%s'" % v) if dt == "STRING" else (str(int(v)) if dt in ("INT", "LONG") else repr(float(v)))
                q = _q("c = %s" % lit)
                want = P.prune(rs, q)
                assert prune_segment(seg, q) == want, (fn, dt, v)
                assert prune_segment(seg, q, pruners=P.PARTITION) == P.prune(rs, q, P.PARTITION), (fn, dt, v)
                checked += 1
                pruned += want
                if want:
                    assert int(O.filter_mask(seg, q["filter"]).sum()) == 0, (fn, dt, v)
    assert checked > 200 and pruned > 20, (checked, pruned)
