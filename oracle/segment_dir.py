"""Oracle reader of Pinot segment directories (test infrastructure: only tests/ import it).

Restates, independently of the engine's C++ reader (incubator-pinot_amd/csrc/segment_reader.cpp), what the
reference's loader reads for single-value dictionary columns (PC = pinot-core/src/main/java/org/apache/pinot/core):
  SegmentDirectoryPaths.findSegmentDirectory: <dir>/v3 if present (PC/segment/store/SegmentDirectoryPaths.java:41-56)
  metadata.properties keys: V1Constants.MetadataKeys (PC/segment/creator/impl/V1Constants.java:81-146), read as
  SegmentMetadataImpl.init / ColumnMetadata.fromPropertiesConfiguration do (padding: segment.padding.character,
  unescapeJava, default the legacy '%': PC/segment/index/ColumnMetadata.java:111-115)
  v1: <col>.dict / <col>.sv.unsorted.fwd / <col>.sv.sorted.fwd / <col>.mv.fwd / <col>.bitmap.inv (FilePerIndexDirectory.java:148-168)
  v3: columns.psf + index_map, 8-byte magic 0xdeadbeefdeafbead at each entry (SingleFileIndexDirectory.java:62-320)
Returns pinot_amd.segment.Segment objects (the data model the oracle's query functions take).
"""
import os
import struct

from pinot_amd.segment import Column, Segment

MAGIC = 0xdeadbeefdeafbead


def _unescape(s):
    out, i = [], 0
    while i < len(s):
        c = s[i]
        if c == "\\" and i + 1 < len(s):
            n = s[i + 1]
            if n == "u" and i + 5 < len(s):
                out.append(chr(int(s[i + 2:i + 6], 16)))
                i += 6
                continue
            out.append({"t": "\t", "n": "\n", "r": "\r", "f": "\f"}.get(n, n))
            i += 2
            continue
        out.append(c)
        i += 1
    return "".join(out)


def read_properties(path):
    """Raw values (escapes kept: lists split on unescaped ',' first); '#'/'!' comments; '=' ':' or blank separators."""
    props = {}
    with open(path, encoding="latin-1") as f:
        for line in f.read().splitlines():
            line = line.strip()
            if not line or line[0] in "#!":
                continue
            sep = None
            i = 0
            while i < len(line):
                if line[i] == "\\":
                    i += 2
                    continue
                if line[i] in "=: \t":
                    sep = i
                    break
                i += 1
            if sep is None:
                props[_unescape(line)] = ""
                continue
            key, val = line[:sep].strip(), line[sep + 1:].strip()
            if line[sep] in " \t" and val[:1] in ("=", ":"):
                val = val[1:].strip()
            props[_unescape(key)] = val
    return props


def _list(props, key):
    v = props.get(key)
    if v is None:
        return []
    parts, cur, i = [], "", 0
    while i < len(v):
        if v[i] == "\\" and i + 1 < len(v):
            cur += v[i:i + 2]
            i += 2
            continue
        if v[i] == ",":
            parts.append(cur)
            cur = ""
        else:
            cur += v[i]
        i += 1
    parts.append(cur)
    return [p for p in (_unescape(x).strip() for x in parts) if p]


def _bool(props, key, default=False):
    v = props.get(key)
    return default if v is None else _unescape(v).strip().lower() in ("true", "on", "yes")


def read_segment_dir(index_dir):
    v3 = os.path.join(index_dir, "v3")
    d = v3 if os.path.isdir(v3) else index_dir
    meta = os.path.join(d, "metadata.properties")
    if not os.path.exists(meta):
        meta = os.path.join(index_dir, "metadata.properties")
    props = read_properties(meta)
    version = _unescape(props.get("segment.index.version", "v1"))
    pad = ord("%")
    if "segment.padding.character" in props:
        pad = ord(_unescape(_unescape(props["segment.padding.character"]))[0])
    entries = {}
    if version == "v3":
        with open(os.path.join(d, "columns.psf"), "rb") as f:
            psf = f.read()
        im = read_properties(os.path.join(d, "index_map"))
        raw = {}
        for k, v in im.items():
            idx, what = k.rsplit(".", 1)
            raw.setdefault(idx, {})[what] = int(v)
        for idx, e in raw.items():
            off, size = e["startOffset"], e["size"]
            assert struct.unpack(">Q", psf[off:off + 8])[0] == MAGIC, idx
            entries[idx] = psf[off + 8:off + size]

    def index_bytes(col, index, v1_name):
        if version == "v3":
            return entries.get(col + "." + index)
        p = os.path.join(d, v1_name)
        if not os.path.exists(p):
            return None
        with open(p, "rb") as f:
            return f.read()

    names = []
    for key in ("segment.dimension.column.names", "segment.metric.column.names", "segment.time.column.name",
                "segment.datetime.column.names"):
        for c in _list(props, key):
            if c not in names:
                names.append(c)
    n = int(_unescape(props["segment.total.docs"]))
    cols = {}
    for c in names:
        k = "column.%s." % c
        dt = _unescape(props[k + "dataType"]).upper()
        if dt not in ("INT", "LONG", "FLOAT", "DOUBLE", "STRING") or not _bool(props, k + "hasDictionary", True):
            continue
        mv = not _bool(props, k + "isSingleValues", True)
        is_sorted = _bool(props, k + "isSorted") and not mv
        fwd = index_bytes(c, "forward_index", c + (".mv.fwd" if mv else ".sv.sorted.fwd" if is_sorted
                                                   else ".sv.unsorted.fwd"))
        inv = None if is_sorted or not _bool(props, k + "hasInvertedIndex") else \
            index_bytes(c, "inverted_index", c + ".bitmap.inv")
        col = Column(name=c, data_type=dt, cardinality=int(props[k + "cardinality"]),
                     bits=int(props[k + "bitsPerElement"]), is_sorted=is_sorted,
                     has_inverted_index=is_sorted or inv is not None, num_docs=n,
                     dictionary=index_bytes(c, "dictionary", c + ".dict"),
                     string_width=int(props.get(k + "lengthOfEachEntry", "0")),
                     fwd=None if is_sorted else fwd, sorted_index=fwd if is_sorted else None, inverted=inv,
                     padding=pad if dt == "STRING" else 0)
        if mv:  # FixedBitMultiValueReader file (V1Constants.java:61)
            col.multi_value = True
            col.total_entries = int(props[k + "totalNumberOfEntries"])
            col.max_multi_values = int(props.get(k + "maxNumberOfMultiValues", "0"))
        cols[c] = col
    return Segment(name=_unescape(props.get("segment.name", "")), num_docs=n, columns=cols)


# ---------------------------------------------------------------- raw (var-byte) STRING forward indexes
def snappy_uncompress(data):
    """Raw Snappy block (format_description.txt of snappy 1.1: varint length, then literal / copy elements)."""
    data = bytes(data)
    n, shift, i = 0, 0, 0
    while True:
        b = data[i]
        i += 1
        n |= (b & 0x7F) << shift
        shift += 7
        if not b & 0x80:
            break
    out = bytearray()
    while i < len(data):
        tag = data[i]
        i += 1
        kind = tag & 3
        if kind == 0:
            ln = tag >> 2
            if ln >= 60:
                k = ln - 59
                ln = int.from_bytes(data[i:i + k], "little")
                i += k
            ln += 1
            out += data[i:i + ln]
            i += ln
            continue
        if kind == 1:
            ln = ((tag >> 2) & 7) + 4
            off = ((tag >> 5) << 8) | data[i]
            i += 1
        elif kind == 2:
            ln = (tag >> 2) + 1
            off = int.from_bytes(data[i:i + 2], "little")
            i += 2
        else:
            ln = (tag >> 2) + 1
            off = int.from_bytes(data[i:i + 4], "little")
            i += 4
        if off == 0 or off > len(out):
            raise ValueError("snappy copy offset")
        for _ in range(ln):
            out.append(out[-off])
    if len(out) != n:
        raise ValueError("snappy length")
    return bytes(out)


def read_var_byte_strings(buf, num_docs):
    """VarByteChunkSingleValueReader.getString for docs [0, num_docs) (VarByteChunkSingleValueReader.java:58-115 over
    BaseChunkSingleValueReader.java:57-147's header: version, numChunks, numDocsPerChunk, lengthOfLongestEntry[,
    totalDocs, compressionType, dataHeaderStart]; version 1 is Snappy)."""
    version, num_chunks, per_chunk, _longest = struct.unpack_from(">iiii", buf, 0)
    comp, header = 1, 16
    if version > 1:
        _total, comp, header = struct.unpack_from(">iii", buf, 16)
    offs = list(struct.unpack_from(">%di" % num_chunks, buf, header)) + [len(buf)]
    out = []
    for c in range(num_chunks):
        if len(out) >= num_docs:
            break
        chunk = bytes(buf[offs[c]:offs[c + 1]])
        chunk = snappy_uncompress(chunk) if comp == 1 else chunk
        rows = struct.unpack_from(">%di" % per_chunk, chunk, 0)
        for r in range(per_chunk):
            if len(out) >= num_docs:
                break
            e = rows[r + 1] if r + 1 < per_chunk and rows[r + 1] != 0 else len(chunk)
            out.append(chunk[rows[r]:e].decode("utf-8"))
    return out


# ---------------------------------------------------------------- raw fixed-width forward indexes
def read_fixed_byte_values(buf, num_docs, fmt):
    """FixedByteChunkSingleValueReader.getInt / getLong / getFloat / getDouble for docs [0, num_docs)
    (FixedByteChunkSingleValueReader.java over BaseChunkSingleValueReader.java:57-96's header; version 1 is always
    Snappy): each decompressed chunk holds numDocsPerChunk big-endian values of lengthOfLongestEntry bytes.
    fmt: the struct code of one value ("i", "q", "f", "d")."""
    version, num_chunks, per_chunk, longest = struct.unpack_from(">iiii", buf, 0)
    assert longest == struct.calcsize(">" + fmt)
    comp, header = 1, 16
    if version > 1:
        _total, comp, header = struct.unpack_from(">iii", buf, 16)
    offs = list(struct.unpack_from(">%di" % num_chunks, buf, header)) + [len(buf)]
    out = []
    for c in range(num_chunks):
        if len(out) >= num_docs:
            break
        chunk = bytes(buf[offs[c]:offs[c + 1]])
        chunk = snappy_uncompress(chunk) if comp == 1 else chunk
        k = min(per_chunk, num_docs - len(out), len(chunk) // longest)
        out.extend(struct.unpack_from(">%d%s" % (k, fmt), chunk, 0))
    return out
