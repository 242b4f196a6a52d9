"""CPU oracle for the server -> broker DataTable bytes: a restatement of DataTableImplV2 and ObjectSerDeUtils.

TEST INFRASTRUCTURE (see pinot_oracle.py's header): only tests/ use it, as the checker of the engine's
pinot_datatable_* bytes. PC = pinot-core/src/main/java/org/apache/pinot/core.

  encode_aggregation   IntermediateResultsBlock.getAggregationResultDataTable (PC/operator/blocks/
                       IntermediateResultsBlock.java:234-270) + attachMetadataToDataTable (:298-317), built as
                       DataTableBuilder does (PC/common/datatable/DataTableBuilder.java:72-160) and written by
                       DataTableImplV2.toBytes (PC/common/datatable/DataTableImplV2.java:233-347)
  decode               DataTableImplV2(ByteBuffer) (:104-171) + getters (:366-468) + ObjectSerDeUtils.deserialize
                       (PC/common/ObjectSerDeUtils.java:144-330)
  encode_empty         DataTableBuilder.buildEmptyDataTable (PC/common/datatable/DataTableBuilder.java:292-370) with the
                       metadata processQuery puts on it when every segment was pruned
                       (PC/query/executor/ServerQueryExecutorV1Impl.java:187-196), keys in that insertion order
  java_hashmap_order   java.util.HashMap iteration order (String.hashCode / Integer.hashCode, spread h ^ h >>> 16,
                       capacity 16 doubling at load 0.75, insertion order within a bucket)

Parity: the reference's tests hold no DataTable byte fixture (DataTableSerDeTest is randomized round trips), and
the Java code cannot run here; this restatement follows the Java sources line by line — parity for the byte
layout rests on that restatement ("parity unpinned" against Java-written bytes). stream-lib 2.7.0
HyperLogLog.getBytes / RegisterSet (not in the reference tree) is restated from its published source: int log2m,
int size * 4, then the register words (6 five-bit registers per int).
"""
import struct

OBJ_STRING, OBJ_LONG, OBJ_DOUBLE, OBJ_AVG_PAIR, OBJ_MIN_MAX, OBJ_HLL, OBJ_MAP = 0, 1, 2, 4, 5, 6, 8
HLL_WORDS = 43  # RegisterSet.getSizeForCount(256)


def java_string_hash(s):
    """java.lang.String.hashCode over UTF-16 code units."""
    b = s.encode("utf-16-be")
    h = 0
    for cu in struct.unpack(">%dH" % (len(b) // 2), b):
        h = (31 * h + cu) & 0xFFFFFFFF
    return h


def java_hashmap_order(hashes):
    cap = 16
    while len(hashes) > 0.75 * cap:
        cap <<= 1
    buckets = [[] for _ in range(cap)]
    for i, h in enumerate(hashes):
        h &= 0xFFFFFFFF
        buckets[(h ^ (h >> 16)) & (cap - 1)].append(i)
    return [i for b in buckets for i in b]


def _i32(v):
    return struct.pack(">i", v)


def _i64(v):
    return struct.pack(">q", v)


def _f64(v):
    return struct.pack(">d", v)


def _str(s):
    b = s.encode("utf-8")
    return _i32(len(b)) + b


def hll_to_bytes(registers):
    """stream-lib HyperLogLog.getBytes (log2m 8): RegisterSet.set puts register p at bit 5 * (p % 6) of word p / 6."""
    words = [0] * HLL_WORDS
    for p, r in enumerate(registers):
        words[p // 6] |= (int(r) & 0x1F) << (5 * (p % 6))
    return _i32(8) + _i32(HLL_WORDS * 4) + b"".join(struct.pack(">I", w) for w in words)


def hll_from_bytes(b):
    log2m, n = struct.unpack(">ii", b[:8])
    assert log2m == 8 and n == HLL_WORDS * 4, (log2m, n)
    words = struct.unpack(">%dI" % HLL_WORDS, b[8:8 + n])
    return [(words[p // 6] >> (5 * (p % 6))) & 0x1F for p in range(256)]


def column_name(agg):
    """AggregationFunction.getColumnName (CountAggregationFunction.java:43-45, SumAggregationFunction.java:42-44 ...)."""
    f = agg["function"].upper()
    name = {"COUNT": None, "SUM": "sum", "MIN": "min", "MAX": "max", "AVG": "avg",
            "DISTINCTCOUNTHLL": "distinctCountHLL"}[f]
    return "count_star" if name is None else name + "_" + agg["column"]


def metadata(stats, groups_limit_reached=False, server=None):
    """attachMetadataToDataTable (IntermediateResultsBlock.java:298-317), + ServerQueryExecutorV1Impl.java:244-245."""
    md = [("numDocsScanned", str(stats["num_docs_scanned"])),
          ("numEntriesScannedInFilter", str(stats["num_entries_scanned_in_filter"])),
          ("numEntriesScannedPostFilter", str(stats["num_entries_scanned_post_filter"])),
          ("numSegmentsProcessed", str(stats["num_segments_processed"])),
          ("numSegmentsMatched", str(stats["num_segments_matched"])),
          ("totalDocs", str(stats["num_total_raw_docs"]))]
    if groups_limit_reached:
        md.append(("numGroupsLimitReached", "true"))
    if server:
        md.append(("numSegmentsQueried", str(server[0])))
        md.append(("timeUsedMs", str(server[1])))
        if server[2] >= 0:
            md.append(("requestId", str(server[2])))
    return md


def _table(rows, cols, dictionaries, md, schema, fixed, var):
    d = _i32(len(dictionaries))
    for i in java_hashmap_order([java_string_hash(c) for c, _ in dictionaries]):
        col, vals = dictionaries[i]
        d += _str(col) + _i32(len(vals))
        for k in java_hashmap_order(list(range(len(vals)))):
            d += _i32(k) + _str(vals[k])
    m = _i32(len(md))
    for i in java_hashmap_order([java_string_hash(k) for k, _ in md]):
        m += _str(md[i][0]) + _str(md[i][1])
    out = _i32(2) + _i32(rows) + _i32(cols)
    off = 13 * 4
    for sec in (d, m, schema, fixed):
        out += _i32(off) + _i32(len(sec))
        off += len(sec)
    out += _i32(off) + _i32(len(var))
    return out + d + m + schema + fixed + var


def _schema(names, types):
    return _i32(len(names)) + b"".join(_str(n) for n in names) + b"".join(_str(t) for t in types)


def encode_aggregation(query, values, stats, server=None):
    """values: the oracle's combined intermediate results (COUNT int, SUM/MIN/MAX float, AVG (sum, count),
    DISTINCTCOUNTHLL registers)."""
    aggs = query["aggregations"]
    types = []
    for a in aggs:
        f = a["function"].upper()
        types.append("LONG" if f == "COUNT" else "OBJECT" if f in ("AVG", "DISTINCTCOUNTHLL") else "DOUBLE")
    fixed, var = b"", b""
    for a, v in zip(aggs, values):
        f = a["function"].upper()
        if f == "COUNT":
            fixed += _i64(int(v))
        elif f in ("SUM", "MIN", "MAX"):
            fixed += _f64(float(v))
        else:
            typ, body = (OBJ_AVG_PAIR, _f64(float(v[0])) + _i64(int(v[1]))) if f == "AVG" else (OBJ_HLL, hll_to_bytes(v))
            fixed += _i32(len(var)) + _i32(len(body))
            var += _i32(typ) + body
    return _table(1, len(aggs), [], metadata(stats, False, server), _schema([column_name(a) for a in aggs], types),
                  fixed, var)


def encode_empty(query, total_docs, server=None):
    md = [("totalDocs", str(total_docs)), ("numDocsScanned", "0"), ("numEntriesScannedInFilter", "0"),
          ("numEntriesScannedPostFilter", "0"), ("numSegmentsProcessed", "0"), ("numSegmentsMatched", "0")]
    if server:
        md += [("numSegmentsQueried", str(server[0])), ("timeUsedMs", str(server[1]))]
        if server[2] >= 0:
            md.append(("requestId", str(server[2])))
    aggs = query["aggregations"]
    if not query.get("group_by"):
        # one row of extractAggregationResult(createAggregationResultHolder()) per function (:331-369)
        types, fixed, var = [], b"", b""
        for a in aggs:
            f = a["function"].upper()
            if f == "COUNT":
                types.append("LONG")
                fixed += _i64(0)
            elif f in ("SUM", "MIN", "MAX"):
                types.append("DOUBLE")
                fixed += _f64({"SUM": 0.0, "MIN": float("inf"), "MAX": float("-inf")}[f])
            else:
                types.append("OBJECT")
                typ, body = (OBJ_AVG_PAIR, _f64(0.0) + _i64(0)) if f == "AVG" else (OBJ_HLL, hll_to_bytes([0] * 256))
                fixed += _i32(len(var)) + _i32(len(body))
                var += _i32(typ) + body
        return _table(1, len(aggs), [], md, _schema([column_name(a) for a in aggs], types), fixed, var)
    # group-by (:314-329): per function its name (STRING, dictionary-encoded) and an empty HashMap
    names, fixed, var = [], b"", b""
    for a in aggs:
        n = column_name(a)
        if n not in names:
            names.append(n)
        body = _i32(0)
        fixed += _i32(names.index(n)) + _i32(len(var)) + _i32(len(body))
        var += _i32(OBJ_MAP) + body
    return _table(len(aggs), 2, [("functionName", names)], md,
                  _schema(["functionName", "GroupByResultMap"], ["STRING", "OBJECT"]), fixed, var)


def encode_group_by(query, result, stats, server=None):
    """IntermediateResultsBlock.getAggregationGroupByResultDataTable (:272-292) of a combined group map
    {key: [value per function]} (values as encode_aggregation takes them; None = trimmed from that function's map).
    Map entries are written in ascending key order (the reference's ConcurrentHashMap order is arbitrary)."""
    aggs = query["aggregations"]
    names, fixed, var = [], b"", b""
    for i, a in enumerate(aggs):
        f = a["function"].upper()
        n = column_name(a)
        if n not in names:
            names.append(n)
        items = sorted((k, v[i]) for k, v in result.items() if v[i] is not None)
        vt = {"COUNT": OBJ_LONG, "AVG": OBJ_AVG_PAIR, "DISTINCTCOUNTHLL": OBJ_HLL}.get(f, OBJ_DOUBLE)
        body = _i32(len(items))
        if items:
            body += _i32(OBJ_STRING) + _i32(vt)
            for k, v in items:
                kb = k.encode("utf-8")
                if f == "COUNT":
                    vb = _i64(int(v))
                elif f == "AVG":
                    vb = _f64(float(v[0])) + _i64(int(v[1]))
                elif f == "DISTINCTCOUNTHLL":
                    vb = hll_to_bytes(v)
                else:
                    vb = _f64(float(v))
                body += _i32(len(kb)) + kb + _i32(len(vb)) + vb
        fixed += _i32(names.index(n)) + _i32(len(var)) + _i32(len(body))
        var += _i32(OBJ_MAP) + body
    return _table(len(aggs), 2, [("functionName", names)], metadata(stats, False, server),
                  _schema(["functionName", "GroupByResultMap"], ["STRING", "OBJECT"]), fixed, var)


# ------------------------------------------------------------------ decoding (the broker side)
class _Reader:
    def __init__(self, b, pos=0):
        self.b, self.p = b, pos

    def i32(self):
        v = struct.unpack_from(">i", self.b, self.p)[0]
        self.p += 4
        return v

    def i64(self):
        v = struct.unpack_from(">q", self.b, self.p)[0]
        self.p += 8
        return v

    def f64(self):
        v = struct.unpack_from(">d", self.b, self.p)[0]
        self.p += 8
        return v

    def raw(self, n):
        v = self.b[self.p:self.p + n]
        self.p += n
        return v

    def str(self):
        return self.raw(self.i32()).decode("utf-8")


def deserialize_object(typ, b):
    """ObjectSerDeUtils.deserialize (ObjectSerDeUtils.java:144-330) for the types the hot path produces."""
    r = _Reader(b)
    if typ == OBJ_STRING:
        return b.decode("utf-8")
    if typ == OBJ_LONG:
        return r.i64()
    if typ == OBJ_DOUBLE:
        return r.f64()
    if typ == OBJ_AVG_PAIR:
        return (r.f64(), r.i64())
    if typ == OBJ_HLL:
        return hll_from_bytes(b)
    if typ == OBJ_MAP:
        n = r.i32()
        out = {}
        if n == 0:
            return out
        kt, vt = r.i32(), r.i32()
        for _ in range(n):
            k = deserialize_object(kt, r.raw(r.i32()))
            out[k] = deserialize_object(vt, r.raw(r.i32()))
        return out
    raise NotImplementedError(typ)


def decode(b):
    """DataTableImplV2 from bytes: {"rows", "columns", "dictionary", "metadata", "schema": [(name, type)],
    "cells": [[value per column] per row]}; the metadata / dictionary section order is kept (as lists)."""
    r = _Reader(b)
    assert r.i32() == 2
    rows, cols = r.i32(), r.i32()
    sec = [(r.i32(), r.i32()) for _ in range(5)]
    out = {"rows": rows, "columns": cols}
    d = _Reader(b, sec[0][0])
    dictionary = []
    if sec[0][1]:
        for _ in range(d.i32()):
            col = d.str()
            dictionary.append((col, [(d.i32(), d.str()) for _ in range(d.i32())]))
    out["dictionary"] = dictionary
    m = _Reader(b, sec[1][0])
    out["metadata"] = [(m.str(), m.str()) for _ in range(m.i32())]
    schema = []
    if sec[2][1]:
        s = _Reader(b, sec[2][0])
        n = s.i32()
        names = [s.str() for _ in range(n)]
        schema = list(zip(names, [s.str() for _ in range(n)]))
    out["schema"] = schema
    fixed, var = sec[3][0], sec[4][0]
    sizes = {"INT": 4, "LONG": 8, "FLOAT": 8, "DOUBLE": 8, "STRING": 4}
    row_size = sum(sizes.get(t, 8) for _, t in schema)
    dicts = {c: dict(v) for c, v in dictionary}
    cells = []
    for i in range(rows):
        f = _Reader(b, fixed + i * row_size)
        row = []
        for name, t in schema:
            if t == "LONG":
                row.append(f.i64())
            elif t == "DOUBLE":
                row.append(f.f64())
            elif t == "INT":
                row.append(f.i32())
            elif t == "STRING":
                row.append(dicts[name][f.i32()])
            else:
                pos, size = f.i32(), f.i32()
                v = _Reader(b, var + pos)
                typ = v.i32()
                row.append(deserialize_object(typ, v.raw(size)))
        cells.append(row)
    out["cells"] = cells
    return out
