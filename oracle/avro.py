"""Minimal Avro object-container reader (null codec only).

TEST INFRASTRUCTURE — part of the oracle. Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import anything under oracle/.

Used to load the reference's own test fixtures
(`pinot-core/src/test/resources/data/test_data-sv.avro`,
`simpleData200001.avro`) the way Pinot's `AvroRecordReader` does, so the
known-answer tests of `InnerSegmentAggregationSingleValueQueriesTest` /
`InterSegmentAggregationSingleValueQueriesTest` / `QueryExecutorTest` can be
replayed. Only the subset of the Avro 1.x binary encoding those files use is
implemented: records of int/long/float/double/string/boolean fields, arrays of those (the
multi-value columns of pinot-tools' airlineStats_data.avro) and ["null", T] unions.
"""
import json
import struct

MAGIC = b"Obj\x01"


class _Buf:
    __slots__ = ("b", "p")

    def __init__(self, b):
        self.b = b
        self.p = 0

    def long(self):
        # zig-zag varint
        shift = 0
        acc = 0
        b = self.b
        while True:
            c = b[self.p]
            self.p += 1
            acc |= (c & 0x7F) << shift
            if c < 0x80:
                break
            shift += 7
        return (acc >> 1) ^ -(acc & 1)

    def raw(self, n):
        r = self.b[self.p:self.p + n]
        self.p += n
        return r

    def string(self):
        n = self.long()
        return self.raw(n).decode("utf-8")

    def float(self):
        return struct.unpack("<f", self.raw(4))[0]

    def double(self):
        return struct.unpack("<d", self.raw(8))[0]


def _reader_for(t):
    if isinstance(t, list):
        subs = [_reader_for(x) for x in t]

        def rd(buf):
            return subs[buf.long()](buf)
        return rd
    if isinstance(t, dict):
        if t.get("type") == "array":  # blocked: count (negative -> byte size follows), items, 0
            item = _reader_for(t["items"])

            def rd_array(buf):
                out = []
                while True:
                    n = buf.long()
                    if n == 0:
                        return out
                    if n < 0:
                        buf.long()
                        n = -n
                    for _ in range(n):
                        out.append(item(buf))
            return rd_array
        t = t["type"]
    if t == "null":
        return lambda buf: None
    if t in ("int", "long"):
        return _Buf.long
    if t == "string":
        return _Buf.string
    if t == "float":
        return _Buf.float
    if t == "double":
        return _Buf.double
    if t == "boolean":
        return lambda buf: buf.raw(1) != b"\x00"
    raise NotImplementedError("avro type %r" % (t,))


def read_avro(path):
    """Return (field_names, {field: list_of_values}) for a null-codec Avro file."""
    with open(path, "rb") as f:
        data = f.read()
    buf = _Buf(data)
    if buf.raw(4) != MAGIC:
        raise ValueError("not an avro container: %s" % path)
    meta = {}
    while True:
        n = buf.long()
        if n == 0:
            break
        if n < 0:
            buf.long()
            n = -n
        for _ in range(n):
            k = buf.string()
            vlen = buf.long()
            meta[k] = buf.raw(vlen)
    sync = buf.raw(16)
    codec = meta.get("avro.codec", b"null")
    if codec != b"null":
        raise NotImplementedError("avro codec %r" % codec)
    schema = json.loads(meta["avro.schema"].decode("utf-8"))
    names = [f["name"] for f in schema["fields"]]
    readers = [_reader_for(f["type"]) for f in schema["fields"]]
    cols = {n: [] for n in names}
    lists = [cols[n] for n in names]
    while buf.p < len(data):
        count = buf.long()
        buf.long()  # block byte size
        for _ in range(count):
            for rd, lst in zip(readers, lists):
                lst.append(rd(buf))
        if buf.raw(16) != sync:
            raise ValueError("avro sync marker mismatch")
    return names, cols
