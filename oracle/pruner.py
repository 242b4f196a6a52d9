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

Pinned by the reference's own known-answer test, ColumnValueSegmentPrunerTest.test
(pinot-core/src/test/java/org/apache/pinot/query/pruner/ColumnValueSegmentPrunerTest.java:53-92), replayed in
tests/test_pruner.py. Bloom filters and PartitionSegmentPruner are not restated (no such metadata in a segment
descriptor).

A segment is described as {"num_docs": n, "columns": {name: (data_type, min, max)}} with min / max None when the
metadata has none; `ranges(seg)` derives it from a pinot_amd Segment (the dictionary's ends).
"""
import math
import re

import numpy as np

DATA_SCHEMA, COLUMN_VALUE, VALID = 1, 2, 4
DEFAULT = DATA_SCHEMA | COLUMN_VALUE | VALID


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


def column_value_prune(tree, columns):
    op = tree["operator"]
    if op in ("AND", "OR"):
        kids = tree["children"]
        if not kids:
            return False
        if op == "AND":
            return any(column_value_prune(c, columns) for c in kids)
        return all(column_value_prune(c, columns) for c in kids)
    if op not in ("EQUALITY", "RANGE"):
        return False
    if tree["column"] not in columns:
        return True  # "Should not reach here after DataSchemaSegmentPruner"
    dt, mn, mx = columns[tree["column"]]
    if op == "EQUALITY":
        v = convert(dt, tree["values"][0])
        if mn is None or mx is None:
            return False
        return java_compare(dt, v, mn) < 0 or java_compare(dt, v, mx) > 0
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


def prune(segment, query, pruners=DEFAULT):
    cols = segment["columns"]
    if pruners & DATA_SCHEMA and data_schema_prune(query, cols):
        return True
    if pruners & COLUMN_VALUE and query.get("filter") is not None and column_value_prune(query["filter"], cols):
        return True
    return bool(pruners & VALID) and valid_prune(segment["num_docs"])


def ranges(seg):
    """{"num_docs", "columns": {name: (type, min, max)}} of a pinot_amd Segment: min / max = its column metadata's
    minValue / maxValue (ColumnMetadata.java:155-156), None when absent (the creator writes none; the loader's
    ColumnMinMaxValueGenerator adds them for the time column in its default mode)."""
    cols = {}
    for name, c in seg.columns.items():
        if getattr(c, "min_value", None) is None:
            cols[name] = (c.data_type, None, None)
            continue
        cols[name] = (c.data_type, convert(c.data_type, c.min_value), convert(c.data_type, c.max_value))
    return {"num_docs": seg.num_docs, "columns": cols}
