"""Pinot immutable-segment column buffers, built in memory in Pinot's own byte format.

This is the *input side* of the drop-in boundary: the C-ABI
(`include/pinot_gpu.h`, `pinot_gpu_segment_register`) receives exactly these
buffers — the bytes `PinotDataBuffer` would hold for a loaded v1/v3 segment — as
host pointers, and uploads them to HBM.

Byte formats (all restated from the reference's segment creator / readers):

* dictionary: sorted ascending unique values, big-endian fixed width
  (`SegmentDictionaryCreator.java:68-206`, `FixedByteValueReaderWriter`);
  STRING values are UTF-8, zero-padded to the longest value
  (`FixedByteValueReaderWriter.java:56-68`, padding byte 0).
* unsorted forward index: dictIds fixed-bit packed MSB-first over a big-endian
  byte stream, `b = getNumBitsPerValue(card - 1)` bits per doc, buffer exactly
  ceil(N*b/8) bytes (`PinotDataBitSet.java:60-71,135-197`,
  `FixedBitSingleValueWriter.java:32-40`, `SegmentColumnarIndexCreator.java:404`).
* sorted forward index: 2 big-endian ints `[startDocId, endDocId]` (inclusive)
  per dictId (`SortedIndexReaderImpl.java:34-39`).
* bitmap inverted index: (card + 1) big-endian int offsets followed by one
  portable-format RoaringBitmap per dictId
  (`OffHeapBitmapInvertedIndexCreator.java:183-206`); Pinot only calls
  `add(int)`, so containers are array (card <= 4096) or bitmap containers.
"""
from dataclasses import dataclass, field
from typing import Dict, List, Optional
import numpy as np

DATA_TYPES = ("INT", "LONG", "FLOAT", "DOUBLE", "STRING")
_BE_DTYPE = {"INT": ">i4", "LONG": ">i8", "FLOAT": ">f4", "DOUBLE": ">f8"}
# Pinot default null values (FieldSpec.java:50,54,57)
DEFAULT_NULL_DIMENSION = {"INT": -2147483648, "LONG": -9223372036854775808,
                          "FLOAT": float("-inf"), "DOUBLE": float("-inf"), "STRING": "null"}
DEFAULT_NULL_METRIC = {"INT": 0, "LONG": 0, "FLOAT": 0.0, "DOUBLE": 0.0, "STRING": "null"}


def num_bits_per_value(max_value: int) -> int:
    """`PinotDataBitSet.getNumBitsPerValue` (PinotDataBitSet.java:60-71): at least 1 bit."""
    if max_value <= 1:
        return 1
    return int(max_value).bit_length()


def pack_fixed_bit(dict_ids: np.ndarray, bits: int) -> bytes:
    """Pack dictIds MSB-first into a big-endian bit stream of exactly ceil(N*b/8) bytes.

    Equivalent to repeated `PinotDataBitSet.writeInt(i, b, v)` (PinotDataBitSet.java:135-197).
    """
    ids = np.ascontiguousarray(dict_ids, dtype=np.uint32)
    n = ids.shape[0]
    if n == 0:
        return b""
    shifts = np.arange(bits - 1, -1, -1, dtype=np.uint32)
    out = []
    chunk = 1 << 20  # multiple of 8 values => every chunk ends on a byte boundary
    for s in range(0, n, chunk):
        v = ids[s:s + chunk]
        bitmat = ((v[:, None] >> shifts[None, :]) & 1).astype(np.uint8)
        out.append(np.packbits(bitmat.reshape(-1), bitorder="big").tobytes())
    return b"".join(out)


def unpack_fixed_bit(buf: bytes, n: int, bits: int) -> np.ndarray:
    """Vectorised `FixedBitSingleValueReader.readValues` for all docs (host-side helper)."""
    raw = np.frombuffer(buf, dtype=np.uint8)
    padded = np.zeros(raw.shape[0] + 8, dtype=np.uint64)
    padded[:raw.shape[0]] = raw
    idx = np.arange(n, dtype=np.uint64)
    bitpos = idx * np.uint64(bits)
    b0 = (bitpos >> np.uint64(3)).astype(np.int64)
    off = bitpos & np.uint64(7)
    w = np.zeros(n, dtype=np.uint64)
    for k in range(5):
        w = (w << np.uint64(8)) | padded[b0 + k]
    shift = np.uint64(40) - off - np.uint64(bits)
    return ((w >> shift) & np.uint64((1 << bits) - 1)).astype(np.int32)


# ---------------------------------------------------------------- roaring (portable format)
SERIAL_COOKIE_NO_RUNCONTAINER = 12346
SERIAL_COOKIE = 12347


def roaring_serialize(doc_ids: np.ndarray) -> bytes:
    """Portable RoaringBitmap serialisation of a sorted docId set (array + bitmap containers, no runs)."""
    d = np.asarray(doc_ids, dtype=np.uint32)
    if d.shape[0] == 0:
        return np.array([SERIAL_COOKIE_NO_RUNCONTAINER, 0], dtype="<u4").tobytes()
    keys = (d >> 16).astype(np.uint16)
    uk, starts, counts = np.unique(keys, return_index=True, return_counts=True)
    n = uk.shape[0]
    header = [np.array([SERIAL_COOKIE_NO_RUNCONTAINER, n], dtype="<u4").tobytes()]
    kc = np.empty(2 * n, dtype="<u2")
    kc[0::2] = uk
    kc[1::2] = (counts - 1).astype(np.uint16)
    header.append(kc.tobytes())
    payloads = []
    for s, c in zip(starts, counts):
        lows = (d[s:s + c] & 0xFFFF).astype(np.uint16)
        if c <= 4096:
            payloads.append(lows.astype("<u2").tobytes())
        else:
            words = np.zeros(1024, dtype=np.uint64)
            np.bitwise_or.at(words, (lows >> 6).astype(np.int64), np.left_shift(np.uint64(1), (lows & 63).astype(np.uint64)))
            payloads.append(words.astype("<u8").tobytes())
    base = 8 + 4 * n + 4 * n
    offs = np.zeros(n, dtype="<u4")
    pos = base
    for i, p in enumerate(payloads):
        offs[i] = pos
        pos += len(p)
    header.append(offs.tobytes())
    return b"".join(header) + b"".join(payloads)


def build_inverted_index(dict_ids: np.ndarray, card: int) -> bytes:
    """`OffHeapBitmapInvertedIndexCreator.seal` layout: (card+1) BE int offsets + roaring payloads."""
    order = np.argsort(dict_ids, kind="stable")
    sorted_ids = dict_ids[order]
    bounds = np.searchsorted(sorted_ids, np.arange(card + 1))
    blobs = []
    for i in range(card):
        docs = np.sort(order[bounds[i]:bounds[i + 1]])
        blobs.append(roaring_serialize(docs))
    offsets = np.zeros(card + 1, dtype=">i4")
    pos = (card + 1) * 4
    offsets[0] = pos
    for i, b in enumerate(blobs):
        pos += len(b)
        offsets[i + 1] = pos
    return offsets.tobytes() + b"".join(blobs)


# ---------------------------------------------------------------- segment model
@dataclass
class Column:
    name: str
    data_type: str
    cardinality: int
    bits: int
    is_sorted: bool
    has_inverted_index: bool
    num_docs: int
    dictionary: bytes            # BE fixed-width sorted values
    string_width: int = 0
    fwd: Optional[bytes] = None  # fixed-bit packed forward index (unsorted columns)
    sorted_index: Optional[bytes] = None  # 2*card BE ints (sorted columns)
    inverted: Optional[bytes] = None      # bitmap inverted index (unsorted columns)
    padding: int = 0                      # STRING padding byte (segment.padding.character; legacy segments '%')
    encoding: str = "dictionary"          # "raw": no-dictionary column, fwd = BE values (cardinality / bits 0)
    min_value: Optional[str] = None       # column.<c>.minValue / maxValue metadata (None: absent, never pruned on)
    max_value: Optional[str] = None
    bloom_filter: Optional[bytes] = None  # the column's .bloom bytes (BloomFilterReader format), or
    create_bloom_filter: bool = False     # built at registration from the dictionary (BloomFilterHandler)
    partition_function: Optional[str] = None  # column.<c>.partitionFunction (Modulo / Murmur / ByteArray / HashCode)
    num_partitions: int = 0
    partitions: Optional[list] = None     # partitionValues; None with a function: every dictionary value's partition
    multi_value: bool = False             # isSingleValues = false: fwd is a FixedBitMultiValueWriter file
    total_entries: int = 0                # totalNumberOfEntries (MV)
    max_multi_values: int = 0             # maxNumberOfMultiValues (MV)
    _mv_offsets: Optional[np.ndarray] = field(default=None, repr=False)  # [numDocs + 1] row starts (MV)
    _raw_values: Optional[np.ndarray] = field(default=None, repr=False)
    _dict_values: Optional[np.ndarray] = field(default=None, repr=False)
    _dict_ids: Optional[np.ndarray] = field(default=None, repr=False)

    def dict_values(self):
        """Decoded dictionary (host convenience; strings unpadded like `getUnpaddedString`)."""
        if self._dict_values is None:
            if self.data_type == "STRING":
                w = self.string_width
                raw = np.frombuffer(self.dictionary, dtype=np.uint8).reshape(self.cardinality, w) if w else \
                    np.zeros((self.cardinality, 0), dtype=np.uint8)
                vals = []
                for r in raw:
                    bs = bytes(r)
                    z = bs.find(bytes([self.padding]))  # getUnpaddedString: up to the first padding byte
                    vals.append((bs if z < 0 else bs[:z]).decode("utf-8"))
                self._dict_values = np.array(vals, dtype=object)
            else:
                self._dict_values = np.frombuffer(self.dictionary, dtype=_BE_DTYPE[self.data_type]).astype(
                    _BE_DTYPE[self.data_type].replace(">", "<"))
        return self._dict_values


@dataclass
class Segment:
    name: str
    num_docs: int
    columns: Dict[str, Column]

    def column(self, name) -> Column:
        return self.columns[name]


def _dictionary_bytes(uniq, data_type):
    if data_type == "STRING":
        enc = [s.encode("utf-8") for s in uniq]
        width = max((len(e) for e in enc), default=0)
        buf = b"".join(e + b"\x00" * (width - len(e)) for e in enc)
        return buf, width
    return np.asarray(uniq).astype(_BE_DTYPE[data_type]).tobytes(), 0


def _sorted_unique(values, data_type):
    if data_type == "STRING":
        # Java String.compareTo order == code-point order for BMP text; sort by UTF-8 bytes equivalently
        uniq = sorted(set(values), key=lambda s: s.encode("utf-8"))
        index = {v: i for i, v in enumerate(uniq)}
        ids = np.fromiter((index[v] for v in values), dtype=np.int32, count=len(values))
        return uniq, ids
    arr = np.asarray(values, dtype={"INT": np.int32, "LONG": np.int64, "FLOAT": np.float32,
                                    "DOUBLE": np.float64}[data_type])
    uniq, ids = np.unique(arr, return_inverse=True)
    return uniq, ids.astype(np.int32)


def multi_value_fwd(ids: np.ndarray, offsets: np.ndarray, bits: int) -> bytes:
    """`FixedBitMultiValueWriter` file (PC/io/writer/impl/v1/FixedBitMultiValueWriter.java:61-155): CHUNK OFFSETS (BE
    int per chunk of docsPerChunk = (int) ceil(2048 / (float) (totalNumValues / numDocs)) rows: the chunk's first
    entry), BITSET (bit e set, MSB first, when entry e starts a row: setIntArray's customBitSet.setBit), RAW DATA (the
    entries' dictIds, FixedBitIntReaderWriter at `bits`)."""
    rows = offsets.shape[0] - 1
    total = int(offsets[-1])
    if rows == 0:
        return b""
    avg = np.float32(total // rows)
    per_chunk = int(np.ceil(np.float32(2048) / avg))
    num_chunks = (rows + per_chunk - 1) // per_chunk
    chunk_offsets = offsets[0:rows:per_chunk][:num_chunks].astype(">i4").tobytes()
    starts = np.zeros(total, dtype=np.uint8)
    starts[offsets[:-1][offsets[:-1] < total]] = 1
    bitset = np.packbits(starts, bitorder="big").tobytes()
    return chunk_offsets + bitset + pack_fixed_bit(ids, bits)


def build_mv_column(name, rows, data_type, bits=None, inverted=False) -> Column:
    """A dictionary-encoded multi-value column (`SegmentColumnarIndexCreator.indexRow` with `indexOfMV`): the
    dictionary over every entry, each row's dictIds in row order. rows: one non-empty list of values per doc."""
    if any(len(r) == 0 for r in rows):
        raise ValueError("every multi-value row holds at least one value (nulls become the default value)")
    lens = np.array([len(r) for r in rows], dtype=np.int64)
    offsets = np.zeros(len(rows) + 1, dtype=np.int64)
    np.cumsum(lens, out=offsets[1:])
    flat = [v for r in rows for v in r]
    uniq, ids = _sorted_unique(flat, data_type)
    card = len(uniq)
    min_bits = num_bits_per_value(card - 1)
    bits = min_bits if bits is None else bits
    if not min_bits <= bits <= 32:
        raise ValueError("bits %d outside [%d, 32]" % (bits, min_bits))
    dbytes, width = _dictionary_bytes(uniq, data_type)
    col = Column(name=name, data_type=data_type, cardinality=card, bits=bits, is_sorted=False,
                 has_inverted_index=bool(inverted), num_docs=len(rows), dictionary=dbytes, string_width=width,
                 multi_value=True, total_entries=int(offsets[-1]), max_multi_values=int(lens.max(initial=0)))
    col._dict_ids = ids
    col._mv_offsets = offsets
    col.fwd = multi_value_fwd(ids, offsets, bits)
    if inverted:  # MV inverted index: per dictId the docs holding it (OffHeapBitmapInvertedIndexCreator.add(int[]))
        doc_of = np.repeat(np.arange(len(rows), dtype=np.int64), lens)
        pairs = np.unique(np.stack([ids.astype(np.int64), doc_of], axis=1), axis=0) if len(flat) else \
            np.zeros((0, 2), dtype=np.int64)
        bounds = np.searchsorted(pairs[:, 0], np.arange(card + 1))
        blobs = [roaring_serialize(pairs[bounds[i]:bounds[i + 1], 1]) for i in range(card)]
        hdr = np.zeros(card + 1, dtype=">i4")
        pos = (card + 1) * 4
        hdr[0] = pos
        for i, b in enumerate(blobs):
            pos += len(b)
            hdr[i + 1] = pos
        col.inverted = hdr.tobytes() + b"".join(blobs)
    return col


def build_column(name, values, data_type, inverted=False, allow_sorted=True, bits=None, raw=False) -> Column:
    """Create one column the way `SegmentColumnarIndexCreator` does for a single-value dictionary column.

    `bits` (default getNumBitsPerValue(card - 1), SegmentColumnarIndexCreator.java:404) may be wider: the
    reader takes the width from the metadata's bitsPerElement (ColumnMetadata.java:98).
    raw=True: a no-dictionary numeric column (encoding PINOT_ENCODING_RAW): `fwd` holds the values, BE fixed width;
    dict_values() / _dict_ids still describe its sorted distinct values for host-side checks."""
    if data_type not in DATA_TYPES:
        raise ValueError("unsupported data type %s" % data_type)
    if raw:
        if data_type == "STRING":
            # var-byte values, flat as the C-ABI takes them: numDocs + 1 BE int offsets, then the UTF-8 bytes
            enc = [str(v).encode("utf-8") for v in values]
            offs = np.zeros(len(enc) + 1, dtype=np.int64)
            np.cumsum([len(e) for e in enc], out=offs[1:])
            uniq, ids = _sorted_unique([str(v) for v in values], data_type)
            col = Column(name=name, data_type=data_type, cardinality=0, bits=0, is_sorted=False,
                         has_inverted_index=False, num_docs=len(enc), dictionary=b"", encoding="raw")
            col.fwd = offs.astype(">i4").tobytes() + b"".join(enc)
            col._raw_values = np.array([str(v) for v in values], dtype=object)
            col._dict_values = np.array(uniq, dtype=object)
            col._dict_ids = ids
            return col
        vals = np.asarray(values).astype(_BE_DTYPE[data_type].replace(">", "<"))
        uniq, ids = _sorted_unique(vals, data_type)
        col = Column(name=name, data_type=data_type, cardinality=0, bits=0, is_sorted=False, has_inverted_index=False,
                     num_docs=int(vals.shape[0]), dictionary=b"", encoding="raw")
        col.fwd = vals.astype(_BE_DTYPE[data_type]).tobytes()
        col._raw_values = vals
        col._dict_values = np.asarray(uniq).astype(vals.dtype)
        col._dict_ids = ids
        return col
    uniq, ids = _sorted_unique(values, data_type)
    card = len(uniq)
    n = ids.shape[0]
    min_bits = num_bits_per_value(card - 1)
    if bits is None:
        bits = min_bits
    elif not min_bits <= bits <= 32:
        raise ValueError("bits %d outside [%d, 32]" % (bits, min_bits))
    dbytes, width = _dictionary_bytes(uniq, data_type)
    is_sorted = bool(allow_sorted and (n <= 1 or bool(np.all(ids[1:] >= ids[:-1]))))
    col = Column(name=name, data_type=data_type, cardinality=card, bits=bits, is_sorted=is_sorted,
                 has_inverted_index=bool(inverted) or is_sorted, num_docs=n, dictionary=dbytes,
                 string_width=width)
    col._dict_ids = ids
    if is_sorted:
        starts = np.searchsorted(ids, np.arange(card), side="left")
        ends = np.searchsorted(ids, np.arange(card), side="right") - 1
        pairs = np.empty(2 * card, dtype=">i4")
        pairs[0::2] = starts
        pairs[1::2] = ends
        col.sorted_index = pairs.tobytes()
    else:
        col.fwd = pack_fixed_bit(ids, bits)
        if inverted:
            col.inverted = build_inverted_index(ids, card)
    return col


def _metadata_string(v, data_type):
    if data_type in ("FLOAT", "DOUBLE"):
        return repr(float(v))
    return str(v if data_type == "STRING" else int(v))


def build_segment(name, columns: Dict[str, tuple], inverted_columns=(), num_docs=None, bits=None,
                  allow_sorted=True, raw_columns=(), min_max=(), bloom_columns=(), partitions=None,
                  mv_columns=()) -> Segment:
    """columns: {name: (data_type, values)} in schema order; bits: optional {name: bitsPerElement};
    raw_columns: names written without a dictionary; min_max: names given minValue / maxValue metadata (the sorted
    values' ends, as ColumnMinMaxValueGenerator writes them), min_max=True: every column; bloom_columns: names given a
    bloom filter (built at registration from the dictionary, as the loader's BloomFilterHandler does); partitions:
    {name: (function, numPartitions)} partition metadata (the partitions of the column's values); mv_columns: names
    whose values are per-doc lists (multi-value columns)."""
    cols = {}
    n = None
    for cname, (dt, vals) in columns.items():
        if cname in mv_columns:
            col = build_mv_column(cname, vals, dt, bits=(bits or {}).get(cname), inverted=cname in inverted_columns)
        else:
            col = build_column(cname, vals, dt, inverted=cname in inverted_columns, allow_sorted=allow_sorted,
                               bits=(bits or {}).get(cname), raw=cname in raw_columns)
        if n is None:
            n = col.num_docs
        elif n != col.num_docs:
            raise ValueError("ragged columns")
        if (min_max is True or cname in min_max) and len(col.dict_values()):
            vals = col.dict_values()
            col.min_value = _metadata_string(vals[0], dt)
            col.max_value = _metadata_string(vals[len(vals) - 1], dt)
        col.create_bloom_filter = cname in bloom_columns
        if partitions and cname in partitions:
            col.partition_function, col.num_partitions = partitions[cname]
        cols[cname] = col
    return Segment(name=name, num_docs=n if num_docs is None else num_docs, columns=cols)
