"""Multi-value columns on the host: the FixedBitMultiValueWriter layout the builder writes and the oracle / library
read (chunk offsets, row-start bitmap, packed entries), the oracle's MV semantics on hand-checked cases (applyMV
any / every, *MV aggregation functions, cartesian-product group keys with duplicates), segment directories with
<col>.mv.fwd, and the library's host-side validation of MV buffers (no GPU).

Parity of the MV path is pinned by the format restatement and these hand-checked cases: the reference's MV known
answers (InterSegmentAggregationMultiValueQueriesTest) are computed on data/test_data-mv.avro, which the reference
checkout does not hold."""
import numpy as np
import pytest

import pinot_oracle as O
from pinot_amd import build_segment
from pinot_amd.executor import validate_segment, segment_dir_info
from pinot_amd._lib import PinotGpuError
from pinot_amd.segment import build_mv_column, multi_value_fwd
from segdir_writer import write_segment_dir
from segment_dir import read_segment_dir


def mv_rows(rng, n, card, max_len, long_row=False):
    lens = rng.integers(1, max_len + 1, n)
    if long_row and n > 3:
        lens[n // 2] = 300
    return [list(rng.integers(0, card, int(k))) for k in lens]


def mv_segment(rng, n, name="mv"):
    """A segment with MV INT / LONG / DOUBLE / STRING columns beside single-value ones (the test_data-mv shape:
    MV dimensions column6 / column7 next to SV metrics)."""
    tags = mv_rows(rng, n, 40, 4, long_row=rng.random() < 0.5)
    cols = {
        "tags": ("INT", [[int(v) * 7 - 100 for v in r] for r in tags]),
        "tagl": ("LONG", [[int(v) * 10 ** 11 + 3 for v in r] for r in mv_rows(rng, n, 25, 3)]),
        "tagd": ("DOUBLE", [[float(v) * 0.25 - 2.0 for v in r] for r in mv_rows(rng, n, 30, 3)]),
        "tags_s": ("STRING", [["t%02d" % v for v in r] for r in mv_rows(rng, n, 12, 3)]),
        "g": ("INT", rng.integers(0, 6, n).astype(np.int32)),
        "m": ("INT", rng.integers(-1000, 1000, n).astype(np.int32)),
        "s": ("STRING", np.array(["s%d" % v for v in rng.integers(0, 4, n)], dtype=object)),
    }
    return build_segment(name, cols, inverted_columns=("tags", "g") if rng.random() < 0.6 else (),
                         mv_columns=("tags", "tagl", "tagd", "tags_s"), allow_sorted=False)


# ------------------------------------------------------------------ layout
@pytest.mark.parametrize("n,max_len", [(1, 1), (5, 3), (4000, 1), (3000, 9), (7, 5000)])
def test_layout_round_trip(n, max_len):
    """Builder (FixedBitMultiValueWriter.setIntArray) -> oracle reader (FixedBitMultiValueReader.getIntArray)."""
    rng = np.random.default_rng(n + max_len)
    rows = mv_rows(rng, n, 300, max_len)
    col = build_mv_column("c", rows, "INT")
    off, ent = O.mv_rows(col)
    assert off.shape[0] == n + 1 and off[-1] == sum(len(r) for r in rows)
    uniq = col.dict_values()
    for d, r in enumerate(rows):
        assert list(uniq[ent[off[d]:off[d + 1]]]) == r
    assert col.max_multi_values == max(len(r) for r in rows)


def test_rows_per_chunk_formula():
    """docsPerChunk = (int) ceil(2048 / (float) (totalNumValues / numDocs)) (Java int division first): the chunk
    offset header holds one int per chunk."""
    for n, per_row, chunk in ((10000, 3, 683), (5000, 1, 2048), (100, 2048, 1), (50, 5000, 1), (9000, 7, 293)):
        offsets = np.arange(n + 1, dtype=np.int64) * per_row
        ids = np.zeros(n * per_row, dtype=np.int32)
        buf = multi_value_fwd(ids, offsets, 1)
        chunks = (n + chunk - 1) // chunk
        assert len(buf) == 4 * chunks + (n * per_row + 7) // 8 + (n * per_row + 7) // 8
        assert list(np.frombuffer(buf[:4 * chunks], dtype=">i4")) == [c * chunk * per_row for c in range(chunks)]


# ------------------------------------------------------------------ oracle semantics, hand-checked
def _tiny():
    return build_segment("t", {
        "mv": ("INT", [[1, 2], [3], [2, 2, 5], [5, 1]]),
        "g": ("INT", np.array([0, 1, 0, 1], dtype=np.int32)),
        "x": ("INT", np.array([10, 20, 30, 40], dtype=np.int32)),
    }, mv_columns=("mv",), allow_sorted=False)


def test_mv_filter_any_and_every():
    seg = _tiny()
    eq = O.filter_mask(seg, {"operator": "EQUALITY", "column": "mv", "values": ["2"]})
    assert list(eq) == [True, False, True, False]
    ne = O.filter_mask(seg, {"operator": "NOT", "column": "mv", "values": ["2"]})  # every entry != 2
    assert list(ne) == [False, True, False, True]
    nin = O.filter_mask(seg, {"operator": "NOT_IN", "column": "mv", "values": ["1\t\t3"]})
    assert list(nin) == [False, False, True, False]
    rng_ = O.filter_mask(seg, {"operator": "RANGE", "column": "mv", "values": ["[4\t\t*)"]})
    assert list(rng_) == [False, False, True, True]


def test_mv_aggregations():
    seg = _tiny()
    q = {"aggregations": [{"function": f, "column": c} for f, c in (
        ("COUNT", "*"), ("COUNTMV", "mv"), ("SUMMV", "mv"), ("MINMV", "mv"), ("MAXMV", "mv"), ("AVGMV", "mv"),
        ("SUM", "x"))], "filter": None, "group_by": None}
    r, scanned = O.execute_server([seg], q)
    assert scanned == 4
    assert r[:5] == [4, 8, 21.0, 1.0, 5.0] and r[5] == (21.0, 8) and r[6] == 100.0
    with pytest.raises(ValueError):
        O.execute_server([seg], {"aggregations": [{"function": "SUM", "column": "mv"}], "filter": None,
                                 "group_by": None})


def test_mv_group_by_cartesian_with_duplicates():
    seg = _tiny()
    q = {"aggregations": [{"function": "COUNT", "column": "*"}, {"function": "SUM", "column": "x"},
                          {"function": "COUNTMV", "column": "mv"}],
         "filter": None, "group_by": {"columns": ["mv", "g"], "top_n": 10}}
    r, _ = O.execute_server([seg], q)
    # doc 2 ([2, 2, 5], g 0) gives keys (2,0) twice and (5,0) once, each with all 3 entries
    assert r["2\t0"] == [3, 70.0, 8]       # doc 0 (x 10, 2 entries) once + doc 2 (x 30, 3 entries) twice
    assert r["5\t0"] == [1, 30.0, 3]
    assert r["1\t0"] == [1, 10.0, 2]
    assert r["5\t1"] == [1, 40.0, 2] and r["1\t1"] == [1, 40.0, 2] and r["3\t1"] == [1, 20.0, 1]
    assert len(r) == 6


def test_mv_group_by_first_appearance_admission():
    """IntMapBasedHolder.processMultiValue (DictionaryBasedGroupKeyGenerator.java:282-300): above the array threshold
    a doc's keys take group ids in getIntRawKeys order (:344-410: the highest-index multi-value column fastest) until
    the holder holds min(product, limit) keys; later keys are dropped for every doc (INVALID_ID)."""
    seg = build_segment("adm", {
        "a": ("INT", [[2, 1], [3], [1, 3], [1, 2]]),
        "b": ("INT", [[7, 8], [8], [7], [9, 7]]),
        "x": ("INT", np.array([10, 20, 30, 40], dtype=np.int32)),
    }, mv_columns=("a", "b"), allow_sorted=False)
    q = {"aggregations": [{"function": "COUNT", "column": "*"}, {"function": "SUM", "column": "x"}],
         "filter": None, "group_by": {"columns": ["a", "b"], "top_n": 10}}
    mask = np.ones(4, dtype=bool)
    # doc 0 keys in order: (2,7) (2,8) (1,7) (1,8) — column b (index 1) fastest; the holder admits 5 keys:
    # doc 0's four, then doc 1's (3,8); doc 2's (1,7) exists, (3,7) is dropped; doc 3's (1,9) dropped, (1,7) exists,
    # (2,9) dropped, (2,7) exists
    r = O.group_by_segment(seg, q, mask, num_groups_limit=5, array_threshold=2)
    assert r == {"2\t7": [2, 50.0], "2\t8": [1, 10.0], "1\t7": [3, 80.0], "1\t8": [1, 10.0], "3\t8": [1, 20.0]}
    # without a binding limit every key of the cartesian products counts
    full = O.group_by_segment(seg, q, mask, num_groups_limit=100, array_threshold=2)
    assert len(full) == 8 and full["3\t7"] == [1, 30.0] and full["1\t9"] == [1, 40.0]


# ------------------------------------------------------------------ segment directories + host validation
@pytest.mark.parametrize("version", ["v1", "v3"])
def test_segment_dir_round_trip(tmp_path, version):
    rng = np.random.default_rng(3)
    seg = mv_segment(rng, 777)
    d = write_segment_dir(seg, str(tmp_path / "s"), version=version)
    n, cols, skipped = segment_dir_info(d)
    assert (n, cols, skipped) == (777, len(seg.columns), 0)
    back = read_segment_dir(d)
    for c in ("tags", "tagl", "tagd", "tags_s"):
        a, b = O.mv_rows(seg.column(c)), O.mv_rows(back.column(c))
        assert (a[0] == b[0]).all() and (a[1] == b[1]).all()
    q = {"aggregations": [{"function": "SUMMV", "column": "tags"}, {"function": "COUNT", "column": "*"}],
         "filter": {"operator": "NOT_IN", "column": "tags_s", "values": ["t01\t\tt02"]},
         "group_by": {"columns": ["tags_s", "g"], "top_n": 10}}
    assert O.execute_server([seg], q) == O.execute_server([back], q)


def test_validate_mv_buffers():
    rng = np.random.default_rng(4)
    seg = mv_segment(rng, 3000)
    validate_segment(seg)
    col = seg.column("tags")
    good = col.fwd
    bad = bytearray(good)
    bad[4:8] = (int.from_bytes(bad[4:8], "big") + 1).to_bytes(4, "big")  # second chunk offset off by one
    for buf, total, msg in ((bytes(bad), col.total_entries, "chunk offset"),
                            (good[:-3] if len(good) > 3 else b"", col.total_entries, "shorter"),
                            (good, col.num_docs - 1, "totalNumberOfEntries")):
        col.fwd, saved = buf, col.total_entries
        col.total_entries = total
        try:
            with pytest.raises(PinotGpuError, match=msg):
                validate_segment(seg)
        finally:
            col.fwd, col.total_entries = good, saved
    validate_segment(seg)
