"""CPU oracle for the broker reduce over the servers' DataTables.

TEST INFRASTRUCTURE (see pinot_oracle.py's header): only tests/ use it, as the checker of the library's
pinot_broker_reduce. PC = pinot-core/src/main/java/org/apache/pinot/core.

  reduce        BrokerReduceService.reduceOnDataTable (PC/query/reduce/BrokerReduceService.java:69-270):
                statistics summed from the metadata (:94-176); setAggregationResults (:347-393);
                setGroupByHavingResults without HAVING (:405-530) with AggregationGroupByTrimmingService
                .trimFinalResults (PC/query/aggregation/groupby/AggregationGroupByTrimmingService.java:123-149)
  format_value  AggregationFunctionUtils.formatValue (PC/query/aggregation/function/AggregationFunctionUtils.java
                :113-128): Long.toString; whole doubles up to Long.MAX_VALUE as (long) + ".00000"; otherwise
                String.format("%1.5f"), which Java rounds HALF_UP on the shortest repr digits (FormattedFloatingDecimal)

Pinned by the reference's InterSegmentAggregationSingleValueQueriesTest strings (tests/golden/reference_kats.json,
the broker-formatted values of 2 servers x 2 segments), replayed in tests/test_broker.py.
"""
import decimal
import math

from datatable import decode
from hll import cardinality as hll_cardinality

LONG_MAX = 9223372036854775807


def format_double(d):
    if math.isnan(d):
        return "NaN"
    if math.isinf(d):
        return "Infinity" if d > 0 else "-Infinity"
    if d == math.floor(d) and d <= float(LONG_MAX):  # DoubleMath.isMathematicalInteger, then (long) d
        return "%d.00000" % max(min(int(d), LONG_MAX), -LONG_MAX - 1)
    ctx = decimal.Context(prec=420, rounding=decimal.ROUND_HALF_UP)
    q = decimal.Decimal(repr(abs(d))).quantize(decimal.Decimal("0.00001"), context=ctx)
    return ("-" if math.copysign(1, d) < 0 else "") + format(q, "f")


def format_value(v):
    return str(v) if isinstance(v, int) else format_double(v)


def _merge(f, a, b):
    if f in ("COUNT", "SUM"):
        return a + b
    if f == "MIN":
        return min(a, b)
    if f == "MAX":
        return max(a, b)
    if f == "AVG":
        return (a[0] + b[0], a[1] + b[1])
    return [max(x, y) for x, y in zip(a, b)]


def _final(f, v):
    if f == "AVG":
        return v[0] / v[1] if v[1] else -math.inf
    if f == "DISTINCTCOUNTHLL":
        return int(hll_cardinality(v))
    return int(v) if f == "COUNT" else float(v)


def reduce(query, tables, top_n=10):
    fns = [a["function"].upper() for a in query["aggregations"]]
    stats = dict(numDocsScanned=0, numEntriesScannedInFilter=0, numEntriesScannedPostFilter=0, numSegmentsQueried=0,
                 numSegmentsProcessed=0, numSegmentsMatched=0, totalDocs=0)
    limit = False
    decoded = [decode(t) for t in tables]
    rows = []
    for t in decoded:
        md = dict(t["metadata"])
        for k in stats:
            if k in md:
                stats[k] += int(md[k])
        limit |= md.get("numGroupsLimitReached", "").lower() == "true"
        if t["schema"] and t["rows"] > 0:
            rows.append(t)
    results = []
    if rows and not query.get("group_by"):
        acc = None
        for t in rows:
            vals = t["cells"][0]
            acc = list(vals) if acc is None else [_merge(f, a, b) for f, a, b in zip(fns, acc, vals)]
        for (name, _), f, v in zip(rows[-1]["schema"], fns, acc):
            results.append({"function": name, "value": format_value(_final(f, v))})
    elif rows:
        for i, f in enumerate(fns):
            merged = {}
            name = None
            for t in rows:
                name = name or t["cells"][i][0]
                for k, v in t["cells"][i][1].items():
                    merged[k] = _merge(f, merged[k], v) if k in merged else v
            fin = [(k, _final(f, v)) for k, v in merged.items()]
            # MIN ascending, every other function descending (ComparableSorter); ties by key
            fin.sort(key=lambda kv: kv[0])
            fin.sort(key=lambda kv: kv[1], reverse=(f != "MIN"))
            results.append({"groupByResult": [{"value": format_value(v), "group": k.split("\t")}
                                              for k, v in fin[:top_n]],
                            "function": name, "groupByColumns": list(query["group_by"]["columns"])})
    out = {"aggregationResults": results, "numGroupsLimitReached": limit}
    out.update(stats)
    return out
