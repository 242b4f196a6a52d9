"""Writes Segment objects as Pinot segment directories (test infrastructure).

v1: metadata.properties + <col>.dict, <col>.sv.unsorted.fwd | <col>.sv.sorted.fwd | <col>.mv.fwd, <col>.bitmap.inv, as
SegmentColumnarIndexCreator leaves them (file names: SegmentMetadataImpl.java:498-527, V1Constants.java:53-63).
v3: the same buffers in v3/columns.psf, each behind the 8-byte magic marker, located by v3/index_map
("<col>.<index>.startOffset = o" / ".size = n", n counting the marker: SingleFileIndexDirectory.java:166-205,320-330).
Raw (no-dictionary) columns: <col>.sv.raw.fwd as FixedByteChunkSingleValueWriter writes it
(BaseChunkSingleValueWriter.java:62-200: header ints, absolute chunk offsets, PASS_THROUGH or Snappy chunks), STRING
ones as VarByteChunkSingleValueWriter does (per-chunk row offsets, then the bytes).
Bloom filters: <col>.bloom (v3: index type bloom_filter) as BloomFilterHandler leaves them after a load
(BloomFilterCreator.java:57-64; bytes from oracle/bloom.py); partition metadata: column.<c>.partitionFunction /
numPartitions / partitionValues (V1Constants.java:135-137), the values written as "[start end]" ranges.
"""
import os
import struct

MAGIC = 0xdeadbeefdeafbead
TYPE_NAMES = {"INT": "INT", "LONG": "LONG", "FLOAT": "FLOAT", "DOUBLE": "DOUBLE", "STRING": "STRING"}


def _props(seg, version, padding):
    lines = ["segment.name = %s" % seg.name, "segment.table.name = testTable",
             "segment.dimension.column.names = %s" % ",".join(seg.columns),
             "segment.metric.column.names = ",
             "segment.total.raw.docs = %d" % seg.num_docs, "segment.total.docs = %d" % seg.num_docs]
    if version != "v1":
        lines.append("segment.index.version = %s" % version)
    if padding is not None:
        lines.append("segment.padding.character = %s" % padding)
    for c in seg.columns.values():
        k = "column.%s." % c.name
        lines += [k + "cardinality = %d" % c.cardinality, k + "totalDocs = %d" % seg.num_docs,
                  k + "totalRawDocs = %d" % seg.num_docs, k + "dataType = %s" % TYPE_NAMES[c.data_type],
                  k + "bitsPerElement = %d" % c.bits, k + "lengthOfEachEntry = %d" % c.string_width,
                  k + "columnType = DIMENSION", k + "isSorted = %s" % ("true" if c.is_sorted else "false"),
                  k + "hasNullValue = false",
                  k + "hasDictionary = %s" % ("false" if getattr(c, "encoding", "dictionary") == "raw" else "true"),
                  k + "hasInvertedIndex = %s" % ("true" if c.inverted is not None else "false"),
                  k + "isSingleValues = %s" % ("false" if getattr(c, "multi_value", False) else "true"),
                  k + "maxNumberOfMultiValues = %d" % getattr(c, "max_multi_values", 0),
                  k + "totalNumberOfEntries = %d" % (c.total_entries if getattr(c, "multi_value", False)
                                                      else seg.num_docs)]
        if getattr(c, "min_value", None) is not None:
            lines += [k + "minValue = %s" % c.min_value, k + "maxValue = %s" % c.max_value]
        if getattr(c, "partition_function", None):
            parts = sorted(_partitions(c))
            ranges, i = [], 0
            while i < len(parts):  # consecutive partitions as one "[start end]" range
                j = i
                while j + 1 < len(parts) and parts[j + 1] == parts[j] + 1:
                    j += 1
                ranges.append("[%d %d]" % (parts[i], parts[j]))
                i = j + 1
            lines += [k + "partitionFunction = %s" % c.partition_function,
                      k + "numPartitions = %d" % c.num_partitions, k + "partitionValues = %s" % ",".join(ranges)]
    return "\n".join(lines) + "\n"


def _partitions(c):
    import bloom as B
    import pruner as P
    if c.partitions is not None:
        return set(c.partitions)
    vals = [v.item() if hasattr(v, "item") else v for v in c.dict_values()]
    return {B.partition_of(c.partition_function, c.num_partitions, c.data_type, v, P.java_to_string(c.data_type, v))
            for v in vals}


def _bloom_bytes(c):
    import bloom as B
    import pruner as P
    if getattr(c, "bloom_filter", None) is not None:
        return c.bloom_filter
    if not getattr(c, "create_bloom_filter", False):
        return None
    bf = B.BloomFilter.for_cardinality(c.cardinality)
    for v in c.dict_values():
        bf.put(P.java_to_string(c.data_type, v.item() if hasattr(v, "item") else v))
    return bf.to_bytes()


def _varint(n):
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        out.append(b | (0x80 if n else 0))
        if not n:
            return bytes(out)


def _literal(data):
    out = bytearray()
    for s in range(0, len(data), 65536):
        part = data[s:s + 65536]
        n = len(part) - 1
        if n < 60:
            out.append(n << 2)
        elif n < 256:
            out += bytes([60 << 2, n])
        else:
            out += bytes([61 << 2]) + struct.pack("<H", n)
        out += part
    return bytes(out)


def snappy_compress(data):
    """A valid raw Snappy block: greedy 4-byte matches emitted as 2-byte-offset copies (<= 64 bytes), else literals."""
    data = bytes(data)
    out = bytearray(_varint(len(data)))
    table, i, lit = {}, 0, 0
    while i + 4 <= len(data):
        key = data[i:i + 4]
        j = table.get(key)
        table[key] = i
        if j is not None and i - j <= 65535:
            n = 4
            while i + n < len(data) and n < 64 and data[j + n] == data[i + n]:
                n += 1
            out += _literal(data[lit:i]) if i > lit else b""
            out += bytes([((n - 1) << 2) | 2]) + struct.pack("<H", i - j)
            i += n
            lit = i
        else:
            i += 1
    if lit < len(data):
        out += _literal(data[lit:])
    return bytes(out)


def raw_chunk_file(values_be, entry_size, num_docs, docs_per_chunk=1000, compression=1, version=2, chunks=None):
    """FixedByteChunkSingleValueWriter bytes. chunks: optional list of already-compressed chunk bodies."""
    chunk_bytes = docs_per_chunk * entry_size
    raw = [bytes(values_be[s:s + chunk_bytes]) for s in range(0, num_docs * entry_size, chunk_bytes)]
    bodies = chunks if chunks is not None else [snappy_compress(r) if compression == 1 else r for r in raw]
    head = struct.pack(">iiii", version, len(bodies), docs_per_chunk, entry_size)
    if version > 1:
        head += struct.pack(">iii", num_docs, compression, len(head) + 12)
    off = len(head) + 4 * len(bodies)
    offs = []
    for b in bodies:
        offs.append(off)
        off += len(b)
    return head + b"".join(struct.pack(">i", o) for o in offs) + b"".join(bodies)


def var_byte_chunk_file(values, docs_per_chunk=1000, compression=1, version=2):
    """VarByteChunkSingleValueWriter bytes (VarByteChunkSingleValueWriter.java:50-117): per chunk numDocsPerChunk BE
    int row offsets from the chunk start (0 for the unused rows of the last chunk), then the UTF-8 bytes; the chunk
    written up to its last byte, PASS_THROUGH or Snappy."""
    enc = [v if isinstance(v, bytes) else v.encode("utf-8") for v in values]
    longest = max((len(e) for e in enc), default=0)
    bodies = []
    for s in range(0, len(enc), docs_per_chunk):
        rows = enc[s:s + docs_per_chunk]
        head = bytearray(4 * docs_per_chunk)
        off = 4 * docs_per_chunk
        for i, r in enumerate(rows):
            head[4 * i:4 * i + 4] = struct.pack(">i", off)
            off += len(r)
        raw = bytes(head) + b"".join(rows)
        bodies.append(snappy_compress(raw) if compression == 1 else raw)
    head = struct.pack(">iiii", version, len(bodies), docs_per_chunk, longest)
    if version > 1:
        head += struct.pack(">iii", len(enc), compression, len(head) + 12)
    off = len(head) + 4 * len(bodies)
    offs = []
    for b in bodies:
        offs.append(off)
        off += len(b)
    return head + b"".join(struct.pack(">i", o) for o in offs) + b"".join(bodies)


def _buffers(c):
    if getattr(c, "encoding", "dictionary") == "raw" and c.data_type == "STRING":
        yield "forward_index", c.name + ".sv.raw.fwd", getattr(c, "raw_file", None) or var_byte_chunk_file(
            list(c._raw_values))
        return
    if getattr(c, "encoding", "dictionary") == "raw":
        w = 4 if c.data_type in ("INT", "FLOAT") else 8
        yield "forward_index", c.name + ".sv.raw.fwd", getattr(c, "raw_file", None) or raw_chunk_file(
            c.fwd, w, c.num_docs)
        return
    yield "dictionary", c.name + ".dict", c.dictionary
    bloom = _bloom_bytes(c)
    if bloom is not None:
        yield "bloom_filter", c.name + ".bloom", bloom
    if getattr(c, "multi_value", False):
        yield "forward_index", c.name + ".mv.fwd", c.fwd
        if c.inverted is not None:
            yield "inverted_index", c.name + ".bitmap.inv", c.inverted
    elif c.is_sorted:
        yield "forward_index", c.name + ".sv.sorted.fwd", c.sorted_index
    else:
        yield "forward_index", c.name + ".sv.unsorted.fwd", c.fwd
        if c.inverted is not None:
            yield "inverted_index", c.name + ".bitmap.inv", c.inverted


def _star_tree_files(seg, st, d):
    """star_tree_index (the tree, then each dimension's fixed-bit forward index, then each pair's PASS_THROUGH
    FixedByteChunk raw index — a var-byte one for AVG's BYTES AvgPairs: StarTreeIndexCombiner) + star_tree_index_map + the startree.v2.* metadata lines."""
    from pinot_amd.segment import pack_fixed_bit
    import numpy as np
    parts = [("null", "STAR_TREE", st.tree_bytes)]
    for j, dim in enumerate(st.dimensions):
        parts.append((dim, "FORWARD_INDEX", pack_fixed_bit(st.dims[:, j], seg.column(dim).bits)))
    for pair in st.pairs:
        v = st.metrics[pair]
        if getattr(v, "ndim", 1) == 2:  # HyperLogLog BYTES values (HyperLogLog.getBytes) in a var-byte raw index
            from startree_writer import hll_bytes
            parts.append((pair, "FORWARD_INDEX", var_byte_chunk_file([hll_bytes(r) for r in v], docs_per_chunk=64,
                                                                     compression=1)))
            continue
        if isinstance(v, tuple):  # AvgPair BYTES values (AvgPair.toBytes) in a var-byte raw index
            vals = [struct.pack(">dq", float(s), int(c)) for s, c in zip(v[0], v[1])]
            parts.append((pair, "FORWARD_INDEX", var_byte_chunk_file(vals, docs_per_chunk=64, compression=0)))
            continue
        be = v.astype(">i8" if v.dtype.kind in "iu" else ">f8").tobytes()
        parts.append((pair, "FORWARD_INDEX", raw_chunk_file(be, 8, st.num_docs, compression=0)))
    blob, lines, off = bytearray(), [], 0
    for col, typ, data in parts:
        lines += ["0.%s.%s.OFFSET = %d" % (col, typ, off), "0.%s.%s.SIZE = %d" % (col, typ, len(data))]
        blob += data
        off += len(data)
    with open(os.path.join(d, "star_tree_index"), "wb") as f:
        f.write(bytes(blob))
    with open(os.path.join(d, "star_tree_index_map"), "w") as f:
        f.write("\n".join(lines) + "\n")
    pre = "startree.v2.0."
    return ["startree.v2.count = 1", pre + "total.docs = %d" % st.num_docs,
            pre + "split.order = %s" % ",".join(st.dimensions),
            pre + "function.column.pairs = %s" % ",".join(st.pairs),
            pre + "max.leaf.records = %d" % st.max_leaf_records]


def write_segment_dir(seg, index_dir, version="v1", padding="\\\\u0000", crc=None, creation_time=0, star_tree=None):
    """padding: the metadata value as written (default the escaped NUL Pinot writes); None leaves the key out.
    crc: write creation.meta (SegmentIndexCreationDriverImpl: DataOutputStream.writeLong(crc), writeLong(time))."""
    os.makedirs(index_dir, exist_ok=True)
    if crc is not None:
        d = os.path.join(index_dir, "v3") if version == "v3" else index_dir
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "creation.meta"), "wb") as f:
            f.write(struct.pack(">qq", crc, creation_time))
    if version == "v3":
        d = os.path.join(index_dir, "v3")
        os.makedirs(d, exist_ok=True)
        psf, index_map = bytearray(), []
        for c in seg.columns.values():
            for index, _, data in _buffers(c):
                index_map.append("%s.%s.startOffset = %d" % (c.name, index, len(psf)))
                index_map.append("%s.%s.size = %d" % (c.name, index, len(data) + 8))
                psf += struct.pack(">Q", MAGIC) + bytes(data)
        with open(os.path.join(d, "columns.psf"), "wb") as f:
            f.write(bytes(psf))
        with open(os.path.join(d, "index_map"), "w") as f:
            f.write("\n".join(index_map) + "\n")
        extra = _star_tree_files(seg, star_tree, d) if star_tree is not None else []
        with open(os.path.join(d, "metadata.properties"), "w") as f:
            f.write(_props(seg, version, padding) + "".join(l + "\n" for l in extra))
        return index_dir
    for c in seg.columns.values():
        for _, fname, data in _buffers(c):
            with open(os.path.join(index_dir, fname), "wb") as f:
                f.write(bytes(data))
    extra = _star_tree_files(seg, star_tree, index_dir) if star_tree is not None else []
    with open(os.path.join(index_dir, "metadata.properties"), "w") as f:
        f.write(_props(seg, version, padding) + "".join(l + "\n" for l in extra))
    return index_dir
