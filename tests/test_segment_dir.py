"""Segment directories (§8(f)1): the reference's own Java-written v1 segments (pinot-core/src/test/resources/data/
padding{Null,Old,Percent}.tar.gz, unpacked under tests/golden/segments) and v1 / v3 directories written from
built segments, read by the oracle's reader (oracle/segment_dir.py) and checked by the engine's C++ reader on the
host (pinot_gpu_segment_dir_info: no GPU). Known answers: LoaderTest.testPadding
(pinot-core/src/test/java/org/apache/pinot/core/segment/index/loader/LoaderTest.java:144-206).
"""
import json
import os
import shutil
import struct

import numpy as np
import pytest

import pinot_oracle as O
from pinot_amd import PinotGpuError, build_segment, raw_forward_index_values, segment_dir_info
from pinot_amd.executor import validate_segment
from segment_dir import read_segment_dir
from segdir_writer import write_segment_dir

HERE = os.path.dirname(os.path.abspath(__file__))
SEGS = os.path.join(HERE, "golden", "segments")
BAD_ARG = 1


def _names(col):
    return [str(v) for v in col.dict_values()]


@pytest.mark.parametrize("name", ["paddingOld", "paddingPercent"])
def test_loader_kats_percent_padding(name):
    seg = read_segment_dir(os.path.join(SEGS, name))
    col = seg.column("name")
    assert col.padding == ord("%")  # LoaderTest.java:153,174: LEGACY_STRING_PAD_CHAR
    assert _names(col) == ["lynda 2.0", "lynda"]  # :160-163, 180-183
    assert O.index_of(col, "lynda%") == 1 and O.index_of(col, "lynda%%") == 1  # :164-165, 184-185


def test_loader_kats_null_padding():
    seg = read_segment_dir(os.path.join(SEGS, "paddingNull"))
    col = seg.column("name")
    assert col.padding == 0  # LoaderTest.java:194: DEFAULT_STRING_PAD_CHAR
    assert _names(col) == ["lynda", "lynda 2.0"]  # :200-203
    assert O.insertion_index_of(col, "lynda\0") == -2 and O.insertion_index_of(col, "lynda\0\0") == -2  # :204-205


def test_oracle_reader_matches_padding_null_fixture():
    fx = json.load(open(os.path.join(HERE, "golden", "padding_null.json")))
    seg = read_segment_dir(os.path.join(SEGS, "paddingNull"))
    for c, f in fx.items():
        col = seg.column(c)
        assert (col.data_type, col.cardinality, col.bits, col.string_width) == \
            (f["data_type"], f["cardinality"], f["bits"], f["string_width"])
        assert col.dictionary.hex() == f["dict_hex"] and col.fwd.hex() == f["fwd_hex"]


@pytest.mark.parametrize("name", ["paddingNull", "paddingOld", "paddingPercent"])
def test_engine_reader_accepts_java_segments(name):
    assert segment_dir_info(os.path.join(SEGS, name)) == (5, 4, 0)


def _random_segment(seed, n=3000):
    rng = np.random.default_rng(seed)
    cols = {
        "i": ("INT", rng.integers(-500, 500, n).astype(np.int32)),
        "l": ("LONG", rng.integers(0, 1 << 40, n).astype(np.int64)),
        "d": ("DOUBLE", rng.integers(0, 70, n) * 0.5),
        "s": ("STRING", np.array(["v%d" % v for v in rng.integers(0, 40, n)], dtype=object)),
        "srt": ("INT", np.sort(rng.integers(0, 100, n)).astype(np.int32)),
    }
    return build_segment("seg%d" % seed, cols, inverted_columns=("i", "s"))


@pytest.mark.parametrize("version", ["v1", "v3"])
def test_written_directories_round_trip(tmp_path, version):
    seg = _random_segment(5)
    d = write_segment_dir(seg, str(tmp_path / ("seg_" + version)), version=version)
    back = read_segment_dir(d)
    assert back.num_docs == seg.num_docs and list(back.columns) == list(seg.columns)
    for c in seg.columns.values():
        b = back.column(c.name)
        assert (b.data_type, b.cardinality, b.bits, b.is_sorted, b.string_width) == \
            (c.data_type, c.cardinality, c.bits, c.is_sorted, c.string_width)
        assert bytes(b.dictionary) == bytes(c.dictionary)
        assert (b.fwd, b.sorted_index, b.inverted) == (c.fwd, c.sorted_index, c.inverted)
        assert (O.dict_ids(b) == O.dict_ids(c)).all()
    assert segment_dir_info(d) == (seg.num_docs, len(seg.columns), 0)


def _bad(d, match):
    with pytest.raises(PinotGpuError) as ei:
        segment_dir_info(d)
    assert ei.value.status == BAD_ARG, ei.value
    assert match in str(ei.value), str(ei.value)


def test_missing_dictionary_file(tmp_path):
    d = write_segment_dir(_random_segment(6), str(tmp_path / "s"))
    os.remove(os.path.join(d, "l.dict"))
    _bad(d, "no dictionary")


def test_truncated_forward_index_file(tmp_path):
    d = write_segment_dir(_random_segment(6), str(tmp_path / "s"))
    p = os.path.join(d, "i.sv.unsorted.fwd")
    data = open(p, "rb").read()
    open(p, "wb").write(data[:-3])
    _bad(d, "forward index shorter")


def test_v3_bad_magic(tmp_path):
    d = write_segment_dir(_random_segment(6), str(tmp_path / "s"), version="v3")
    p = os.path.join(d, "v3", "columns.psf")
    data = bytearray(open(p, "rb").read())
    data[0] ^= 0xFF
    open(p, "wb").write(bytes(data))
    _bad(d, "magic")


def test_v3_index_map_outside_file(tmp_path):
    d = write_segment_dir(_random_segment(6), str(tmp_path / "s"), version="v3")
    with open(os.path.join(d, "v3", "index_map"), "a") as f:
        f.write("i.bloom_filter.startOffset = 999999999\ni.bloom_filter.size = 16\n")
    _bad(d, "outside columns.psf")


def test_missing_total_docs(tmp_path):
    d = write_segment_dir(_random_segment(6), str(tmp_path / "s"))
    p = os.path.join(d, "metadata.properties")
    lines = [l for l in open(p).read().splitlines() if not l.startswith("segment.total.docs")]
    open(p, "w").write("\n".join(lines) + "\n")
    _bad(d, "segment.total.docs")


def test_not_a_directory(tmp_path):
    _bad(str(tmp_path / "nope"), "not a segment directory")


def test_unserved_columns_are_left_out(tmp_path):
    d = write_segment_dir(_random_segment(7), str(tmp_path / "s"))
    p = os.path.join(d, "metadata.properties")
    # a raw (no-dictionary) multi-value column: not served, left out
    text = open(p).read().replace("column.l.isSingleValues = true", "column.l.isSingleValues = false").replace(
        "column.l.hasDictionary = true", "column.l.hasDictionary = false")
    open(p, "w").write(text)
    n, cols, skipped = segment_dir_info(d)
    assert (cols, skipped) == (4, 1)
    assert "l" not in read_segment_dir(d).columns


def test_raw_columns_read_from_chunked_forward_indexes(tmp_path):
    """.sv.raw.fwd (FixedByteChunkSingleValueReader layout): PASS_THROUGH and Snappy chunks, versions 1 and 2, v1 and
    v3 directories: the loader decompresses them and registration transcodes them (host-side checks only here)."""
    import numpy as np
    from segdir_writer import raw_chunk_file
    rng = np.random.default_rng(5)
    n = 2500
    cols = {"a": ("INT", rng.integers(-9, 9, n).astype(np.int32)), "m": ("LONG", rng.integers(0, 50, n) * 10 ** 12),
            "f": ("FLOAT", (rng.integers(0, 8, n) * 0.5).astype(np.float32)), "d": ("DOUBLE", rng.normal(size=n)),
            "s": ("STRING", np.array(["x%d" % v for v in rng.integers(0, 5, n)], dtype=object))}
    for version, comp, fver in (("v1", 1, 2), ("v3", 0, 2), ("v1", 1, 1), ("v3", 1, 2)):
        seg = build_segment("raw", cols, raw_columns=("a", "m", "f", "d"))
        for c in ("a", "m", "f", "d"):
            col = seg.columns[c]
            w = 4 if col.data_type in ("INT", "FLOAT") else 8
            col.raw_file = raw_chunk_file(col.fwd, w, n, docs_per_chunk=int(rng.integers(7, 900)),
                                          compression=comp if fver > 1 else 1, version=fver)
        d = write_segment_dir(seg, str(tmp_path / ("s_%s_%d_%d" % (version, comp, fver))), version=version)
        assert segment_dir_info(d) == (n, 5, 0)
    # a hand-written Snappy chunk using every element kind: literal, 1-byte-offset copy, 4-byte-offset copy
    seg = build_segment("h", {"a": ("INT", np.full(8, 7, dtype=np.int32))}, raw_columns=("a",))
    body = bytes([32]) + bytes([3 << 2, 0, 0, 0, 7]) + bytes([1 | (7 << 2), 4]) + bytes([3 | (16 << 2), 4, 0, 0, 0])
    seg.columns["a"].raw_file = raw_chunk_file(seg.columns["a"].fwd, 4, 8, docs_per_chunk=8, chunks=[body])
    assert segment_dir_info(write_segment_dir(seg, str(tmp_path / "hand"))) == (8, 1, 0)
    # corrupt chunk streams fail as BAD_ARG, not a crash
    for bad in (bytes([32, 3 << 2, 0, 0]), bytes([32]) + bytes([1 | (7 << 2), 9]), bytes([200])):
        seg.columns["a"].raw_file = raw_chunk_file(seg.columns["a"].fwd, 4, 8, docs_per_chunk=8, chunks=[bad])
        with pytest.raises(PinotGpuError) as ei:
            segment_dir_info(write_segment_dir(seg, str(tmp_path / ("bad%d" % bad[-1]))))
        assert ei.value.status == 1


def test_var_byte_fixture_pins_the_readers(tmp_path):
    """The reference's own var-byte file (data/varByteStrings.v1, VarByteChunkSingleValueReaderWriteTest
    .testBackwardCompatibility: 1009 entries cycling "abcde", "fgh", "ijklmn", "12345"): the oracle's reader returns
    those values, and the library's loader reads it as a raw STRING column's .sv.raw.fwd."""
    import numpy as np
    from segment_dir import read_var_byte_strings
    fixture = open(os.path.join(os.path.dirname(__file__), "golden", "var_byte_strings.v1"), "rb").read()
    expected = ["abcde", "fgh", "ijklmn", "12345"]
    vals = read_var_byte_strings(fixture, 1009)
    assert vals == [expected[i % 4] for i in range(1009)]
    seg = build_segment("vb", {"s": ("STRING", np.array(vals, dtype=object)),
                               "i": ("INT", np.arange(1009, dtype=np.int32))}, raw_columns=("s",))
    seg.columns["s"].raw_file = fixture
    assert segment_dir_info(write_segment_dir(seg, str(tmp_path / "vb"))) == (1009, 2, 0)


@pytest.mark.parametrize("comp,version,per_chunk", [(1, 2, 7), (0, 2, 1000), (1, 1, 333), (0, 2, 1)])
def test_raw_string_columns(tmp_path, comp, version, per_chunk):
    """Raw STRING columns: the writer's var-byte chunks (empty strings, multi-byte UTF-8, a partial last chunk) read
    back by the oracle's reader, and the library's loader + registration checks accept them."""
    import numpy as np
    from segdir_writer import var_byte_chunk_file
    from segment_dir import read_var_byte_strings
    rng = np.random.default_rng(per_chunk)
    pool = ["", "a", "zz", "héllo", "日本", "x" * 40, "b7"]
    vals = [pool[int(v)] for v in rng.integers(0, len(pool), 2001)]
    buf = var_byte_chunk_file(vals, docs_per_chunk=per_chunk, compression=comp if version > 1 else 1,
                              version=version)
    assert read_var_byte_strings(buf, len(vals)) == vals
    seg = build_segment("vs", {"s": ("STRING", np.array(vals, dtype=object))}, raw_columns=("s",))
    seg.columns["s"].raw_file = buf
    assert segment_dir_info(write_segment_dir(seg, str(tmp_path / "d"), version="v3")) == (2001, 1, 0)
    validate_segment(seg)


def test_raw_string_bad_bytes():
    import numpy as np
    seg = build_segment("bad", {"s": ("STRING", np.array(["ab", "c\x00d"], dtype=object))}, raw_columns=("s",))
    with pytest.raises(PinotGpuError, match="NUL"):
        validate_segment(seg)
    seg = build_segment("bad", {"s": ("STRING", np.array(["ab", "cd"], dtype=object))}, raw_columns=("s",))
    col = seg.columns["s"]
    col.fwd = col.fwd[:4] + (9).to_bytes(4, "big") + col.fwd[8:]  # offsets not ascending within the bytes
    with pytest.raises(PinotGpuError, match="offsets"):
        validate_segment(seg)


@pytest.mark.parametrize("version", ["v1", "v3"])
def test_star_tree_files_read_on_the_host(tmp_path, version):
    """The star-tree files a segment directory carries are read and checked with the segment (host only)."""
    from startree_writer import build_star_tree
    rng = np.random.default_rng(12)
    seg = _random_segment(12, 2000)
    st = build_star_tree(seg, ["i", "s"], [("COUNT", "*"), ("SUM", "l")], max_leaf_records=30)
    d = write_segment_dir(seg, str(tmp_path / "st"), version=version, star_tree=st)
    assert segment_dir_info(d)[0] == 2000
    meta = os.path.join(d, "v3" if version == "v3" else "", "star_tree_index_map")
    text = open(meta).read()
    assert "0.null.STAR_TREE.OFFSET = 0" in text and "0.count__*.FORWARD_INDEX.SIZE" in text


def test_fixed_byte_fixture_pins_the_raw_reader(tmp_path):
    """The reference's own fixed-width raw file (data/fixedByteSVRDoubles.v1,
    FixedByteChunkSingleValueReaderWriteTest.testBackwardCompatibility :263-284: a version-1 FixedByteChunk file —
    always Snappy — of 10,009 doubles, doc i = (double) i): the oracle's reader and the library's host reader
    (pinot_segment_read_raw_forward_index = segment_reader.cpp read_raw_chunks + its Snappy decoder) return i for every doc,
    and the segment loader reads it as a raw DOUBLE column's .sv.raw.fwd."""
    from segment_dir import read_fixed_byte_values
    fixture = open(os.path.join(HERE, "golden", "fixed_byte_svr_doubles.v1"), "rb").read()
    assert len(fixture) == 44397 and struct.unpack_from(">i", fixture, 0)[0] == 1  # version 1: Snappy chunks
    n = 10009
    assert read_fixed_byte_values(fixture, n, "d") == [float(i) for i in range(n)]
    got = raw_forward_index_values(fixture, "DOUBLE", n)
    assert got.dtype == np.float64 and (got == np.arange(n, dtype=np.float64)).all()
    seg = build_segment("fb", {"d": ("DOUBLE", np.arange(n, dtype=np.float64)),
                               "i": ("INT", np.arange(n, dtype=np.int32))}, raw_columns=("d",))
    seg.columns["d"].raw_file = fixture
    assert segment_dir_info(write_segment_dir(seg, str(tmp_path / "fb"))) == (n, 2, 0)
    # damaged copies are refused with a status: a truncated chunk, a wrong entry width
    with pytest.raises(PinotGpuError):
        raw_forward_index_values(fixture[:-200], "DOUBLE", n)
    with pytest.raises(PinotGpuError):
        raw_forward_index_values(fixture, "INT", n)
