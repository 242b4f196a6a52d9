"""Writes Segment objects as Pinot segment directories (test infrastructure).

v1: metadata.properties + <col>.dict, <col>.sv.unsorted.fwd | <col>.sv.sorted.fwd, <col>.bitmap.inv, as
SegmentColumnarIndexCreator leaves them (file names: SegmentMetadataImpl.java:498-527, V1Constants.java:53-63).
v3: the same buffers in v3/columns.psf, each behind the 8-byte magic marker, located by v3/index_map
("<col>.<index>.startOffset = o" / ".size = n", n counting the marker: SingleFileIndexDirectory.java:166-205,320-330).
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
                  k + "hasNullValue = false", k + "hasDictionary = true",
                  k + "hasInvertedIndex = %s" % ("true" if c.inverted is not None else "false"),
                  k + "isSingleValues = true", k + "maxNumberOfMultiValues = 0",
                  k + "totalNumberOfEntries = %d" % seg.num_docs]
    return "\n".join(lines) + "\n"


def _buffers(c):
    yield "dictionary", c.name + ".dict", c.dictionary
    if c.is_sorted:
        yield "forward_index", c.name + ".sv.sorted.fwd", c.sorted_index
    else:
        yield "forward_index", c.name + ".sv.unsorted.fwd", c.fwd
        if c.inverted is not None:
            yield "inverted_index", c.name + ".bitmap.inv", c.inverted


def write_segment_dir(seg, index_dir, version="v1", padding="\\\\u0000"):
    """padding: the metadata value as written (default the escaped NUL Pinot writes); None leaves the key out."""
    os.makedirs(index_dir, exist_ok=True)
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
        with open(os.path.join(d, "metadata.properties"), "w") as f:
            f.write(_props(seg, version, padding))
        return index_dir
    for c in seg.columns.values():
        for _, fname, data in _buffers(c):
            with open(os.path.join(index_dir, fname), "wb") as f:
                f.write(bytes(data))
    with open(os.path.join(index_dir, "metadata.properties"), "w") as f:
        f.write(_props(seg, version, padding))
    return index_dir
