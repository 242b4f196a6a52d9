"""CPU oracle for segment pruning: the step processQuery runs before planning.

TEST INFRASTRUCTURE (see pinot_oracle.py's header): only tests/ use it, as the checker of the library's
pinot_segment_prune / pinot_gpu_prune_segments. PC = pinot-core/src/main/java/org/apache/pinot/core.

  prune                  SegmentPrunerService.prune (PC/query/pruner/SegmentPrunerService.java:52-60) over the
                         server's default pruners in order (pinot-server/.../DefaultHelixStarterServerConfig.java:60-64)
  data_schema_prune      DataSchemaSegmentPruner.prune (PC/query/pruner/DataSchemaSegmentPruner.java:38-41) with
                         ServerQueryRequest.getAllColumns (PC/query/request/ServerQueryRequest.java:81-133)
  column_value_prune     ColumnValueSegmentPruner.pruneSegment (PC/query/pruner/ColumnValueSegmentPruner.java:92-200)
                         + AbstractSegmentPruner.pruneNonLeaf / getValue (AbstractSegmentPruner.java:56-105)
  valid_prune            ValidSegmentPruner.prune (PC/query/pruner/ValidSegmentPruner.java:47-58)

  partition_prune        PartitionSegmentPruner.pruneSegment (PC/query/pruner/PartitionSegmentPruner.java:73-111)

Pinned by the reference's own known-answer test, ColumnValueSegmentPrunerTest.test
(pinot-core/src/test/java/org/apache/pinot/query/pruner/ColumnValueSegmentPrunerTest.java:53-92), replayed in
tests/test_pruner.py. The bloom-filter test of ColumnValueSegmentPruner (:140-144) and the partition functions use
oracle/bloom.py.

A segment is described as {"num_docs": n, "columns": {name: (data_type, min, max)}, "bloom": {name: BloomFilter},
"partitions": {name: (function, numPartitions, set of partitions)}} with min / max None when the metadata has none;
`ranges(seg)` derives it from a pinot_amd Segment (the dictionary's ends, its bloom / partition options).
"""
import math
import re

import numpy as np

import bloom as B

DATA_SCHEMA, COLUMN_VALUE, VALID, PARTITION = 1, 2, 4, 8
DEFAULT = DATA_SCHEMA | COLUMN_VALUE | VALID | PARTITION  # DefaultHelixStarterServerConfig.java:60-65


class BadQuery(ValueError):
    """BadQueryRequestException from AbstractSegmentPruner.getValue (a literal the column's type cannot parse)."""


_INT = re.compile(r"[+-]?[0-9]+\Z")


def convert(data_type, s):
    """FieldSpec.DataType.convert: Integer.valueOf / Long.valueOf / Float.valueOf / Double.valueOf / the string."""
    if data_type in ("INT", "LONG"):
        if not _INT.match(s):
            raise BadQuery(s)
        v = int(s)
        lim = 31 if data_type == "INT" else 63
        if not -(1 << lim) <= v < (1 << lim):
            raise BadQuery(s)
        return v
    if data_type in ("FLOAT", "DOUBLE"):
        t = s.strip()
        if t[-1:] in ("f", "F", "d", "D") and t not in ("NaN", "Infinity") and not t.endswith("Infinity"):
            t = t[:-1]
        if "_" in t:  # Python's float() takes digit separators; Java's does not
            raise BadQuery(s)
        try:
            v = float({"NaN": "nan", "Infinity": "inf", "+Infinity": "inf", "-Infinity": "-inf"}.get(t, t))
        except ValueError:
            raise BadQuery(s)
        if t.lower() in ("nan", "inf", "+inf", "-inf", "infinity", "+infinity", "-infinity") and \
                t not in ("NaN", "Infinity", "+Infinity", "-Infinity"):
            raise BadQuery(s)
        if data_type == "FLOAT":  # Float.valueOf: rounded to float (overflow -> +-Infinity)
            with np.errstate(over="ignore"):
                v = float(np.float32(v))
        return v
    return s


def java_compare(data_type, a, b):
    """Comparable.compareTo: Integer / Long; Float / Double.compare (NaN largest, -0.0 < 0.0); String (UTF-8 byte
    order, the convention the dictionaries are searched with)."""
    if data_type == "STRING":
        a, b = a.encode("utf-8"), b.encode("utf-8")
        return (a > b) - (a < b)
    if data_type in ("FLOAT", "DOUBLE"):
        if a < b:
            return -1
        if a > b:
            return 1
        an, bn = math.isnan(a), math.isnan(b)
        if an or bn:
            return 0 if an == bn else (1 if an else -1)
        sa, sb = math.copysign(1, a) < 0, math.copysign(1, b) < 0
        return 0 if sa == sb else (-1 if sa else 1)
    return (a > b) - (a < b)


def parse_range(s):
    """RangePredicate (PC/common/predicate/RangePredicate.java:41-67)."""
    s = s.strip()
    parts = s.split("\t\t")
    lower, upper = parts[0][1:], parts[1][:-1]
    inc_lower = not s.startswith("(") or lower == "*"
    inc_upper = not s.endswith(")") or upper == "*"
    return lower, upper, inc_lower, inc_upper


def java_to_string(data_type, v):
    """Integer / Long / Float / Double.toString of the typed value, or the string (what mightContain hashes)."""
    import pinot_oracle as O
    if data_type in ("INT", "LONG"):
        return str(v)
    if data_type == "FLOAT":
        return O.java_float_to_string(v)
    if data_type == "DOUBLE":
        return O.java_double_to_string(v)
    return v


def prune_nonleaf(tree, leaf):
    """AbstractSegmentPruner.pruneNonLeaf (:56-90): AND prunes when any child does, OR when every child does."""
    op = tree["operator"]
    if op in ("AND", "OR"):
        kids = tree["children"]
        if not kids:
            return False
        if op == "AND":
            return any(prune_nonleaf(c, leaf) for c in kids)
        return all(prune_nonleaf(c, leaf) for c in kids)
    return leaf(tree)


def column_value_prune(tree, columns, blooms=None):
    return prune_nonleaf(tree, lambda t: _column_value_leaf(t, columns, blooms or {}))


def _column_value_leaf(tree, columns, blooms):
    op = tree["operator"]
    if op not in ("EQUALITY", "RANGE"):
        return False
    if tree["column"] not in columns:
        return True  # "Should not reach here after DataSchemaSegmentPruner"
    dt, mn, mx = columns[tree["column"]]
    if op == "EQUALITY":
        v = convert(dt, tree["values"][0])
        prune = mn is not None and mx is not None and (java_compare(dt, v, mn) < 0 or java_compare(dt, v, mx) > 0)
        if not prune and tree["column"] in blooms:  # the bloom filter test (ColumnValueSegmentPruner.java:140-144)
            prune = not blooms[tree["column"]].might_contain(java_to_string(dt, v))
        return prune
    lower, upper, inc_lower, inc_upper = parse_range(tree["values"][0])
    lo = None if lower == "*" else convert(dt, lower)
    hi = None if upper == "*" else convert(dt, upper)
    if lo is not None and hi is not None:
        r = java_compare(dt, lo, hi)
        if (r > 0) if (inc_lower and inc_upper) else (r >= 0):
            return True
    if mn is None or mx is None:
        return False
    if lo is not None:
        r = java_compare(dt, lo, mx)
        if (r > 0) if inc_lower else (r >= 0):
            return True
    if hi is not None:
        r = java_compare(dt, hi, mn)
        if (r < 0) if inc_upper else (r <= 0):
            return True
    return False


def _filter_columns(tree, out):
    if tree is None:
        return
    if tree["operator"] in ("AND", "OR"):
        for c in tree["children"]:
            _filter_columns(c, out)
    else:
        out.add(tree["column"])


def query_columns(query):
    cols = set()
    _filter_columns(query.get("filter"), cols)
    for a in query["aggregations"]:
        if a["function"].upper() != "COUNT":
            cols.add(a["column"])
    if query.get("group_by"):
        cols.update(query["group_by"]["columns"])
    return cols


def data_schema_prune(query, columns):
    return not query_columns(query) <= set(columns)


def valid_prune(num_docs):
    return num_docs == 0


def partition_prune(tree, columns, partitions):
    """PartitionSegmentPruner.pruneSegment (:85-110): EQUALITY leaves on columns with partition metadata."""
    def leaf(t):
        if t["operator"] != "EQUALITY":
            return False
        if t["column"] not in columns:
            return True
        if t["column"] not in partitions:
            return False
        dt = columns[t["column"]][0]
        fn, n, parts = partitions[t["column"]]
        v = convert(dt, t["values"][0])
        return B.partition_of(fn, n, dt, v, java_to_string(dt, v)) not in parts
    return prune_nonleaf(tree, leaf)


def prune(segment, query, pruners=DEFAULT):
    cols = segment["columns"]
    if pruners & DATA_SCHEMA and data_schema_prune(query, cols):
        return True
    if pruners & COLUMN_VALUE and query.get("filter") is not None and \
            column_value_prune(query["filter"], cols, segment.get("bloom")):
        return True
    if pruners & VALID and valid_prune(segment["num_docs"]):
        return True
    return bool(pruners & PARTITION) and query.get("filter") is not None and \
        partition_prune(query["filter"], cols, segment.get("partitions", {}))


def ranges(seg):
    """{"num_docs", "columns": {name: (type, min, max)}} of a pinot_amd Segment: min / max = its column metadata's
    minValue / maxValue (ColumnMetadata.java:155-156), None when absent (the creator writes none; the loader's
    ColumnMinMaxValueGenerator adds them for the time column in its default mode)."""
    cols, blooms, parts = {}, {}, {}
    for name, c in seg.columns.items():
        if getattr(c, "min_value", None) is None:
            cols[name] = (c.data_type, None, None)
        else:
            cols[name] = (c.data_type, convert(c.data_type, c.min_value), convert(c.data_type, c.max_value))
        vals = c.dict_values()
        strings = [java_to_string(c.data_type, v.item() if hasattr(v, "item") else v) for v in vals]
        if getattr(c, "bloom_filter", None) is not None:
            blooms[name] = B.BloomFilter.from_bytes(c.bloom_filter)
        elif getattr(c, "create_bloom_filter", False):  # BloomFilterHandler: every dictionary value's toString
            bf = B.BloomFilter.for_cardinality(c.cardinality)
            for s in strings:
                bf.put(s)
            blooms[name] = bf
        if getattr(c, "partition_function", None):
            if c.partitions is not None:
                ps = set(c.partitions)
            else:
                ps = {B.partition_of(c.partition_function, c.num_partitions, c.data_type,
                                     v.item() if hasattr(v, "item") else v, s) for v, s in zip(vals, strings)}
            parts[name] = (c.partition_function, c.num_partitions, ps)
    return {"num_docs": seg.num_docs, "columns": cols, "bloom": blooms, "partitions": parts}
