"""Star-tree v2 builder (test infrastructure): the pre-aggregated star-tree of a Segment, in Pinot's byte format.

Restates BaseSingleTreeBuilder.build (PC/startree/v2/builder/BaseSingleTreeBuilder.java) with the on-heap record
store (OnHeapSingleTreeBuilder.java:67-160): the segment's records as (dimension dictIds in split order, metric
values per function-column pair) sorted and merged on all dimensions; constructStarTree (children per dimension
value over contiguous runs, a star child — the run's records with that dimension set to STAR and merged on the
remaining dimensions, appended — when the dimension is not in skip-star and has > 1 child; recursion while a child
holds > maxLeafRecords records); createAggregatedDocs (a leaf's records merged; a node with a star child takes the
star child's aggregated doc; else its children's aggregated records merged; dimensions below the node set to STAR);
StarTreeBuilderUtils.serializeTree (little-endian: magic 0xBADDA55B00DAD00D, version 1, header size, dimension
count, (index, name length, UTF-8 name) per dimension, node count, then 7 ints per node in BFS order with children
sorted by dimension value, star (-1) first). STAR is stored as 0 in the dimension forward indexes
(StarTreeV2Constants.STAR_IN_FORWARD_INDEX). PC = pinot-core/src/main/java/org/apache/pinot/core.

Metrics (ValueAggregatorFactory): COUNT -> LONG count of the records, SUM -> DOUBLE, MIN / MAX -> DOUBLE, AVG -> AvgPair
(double sum, long count; AvgPair.toBytes as the BYTES value, 16 B big-endian), DISTINCTCOUNTHLL -> HyperLogLog
(log2m 8; HyperLogLog.getBytes as the BYTES value: int log2m, int 172, the RegisterSet's 43 BE ints); the pair
column name is AggregationFunctionColumnPair.toColumnName: "<type>__<column>" ("count__*").
"""
import struct
from dataclasses import dataclass, field
from typing import Dict, List

import numpy as np

MAGIC = 0xBADDA55B00DAD00D
ALL = -1
STAR_IN_FORWARD_INDEX = 0


@dataclass
class StarTree:
    dimensions: List[str]            # split order
    pairs: List[str]                 # function-column pair names ("sum__d8", "count__*")
    max_leaf_records: int
    dims: np.ndarray                 # int64 [num_docs, num_dims] dictIds (STAR -> 0)
    metrics: Dict[str, np.ndarray]   # pair -> LONG (count) / DOUBLE values per star doc
    nodes: np.ndarray                # int32 [num_nodes, 7] (dimId, value, start, end, aggDoc, firstChild, lastChild)
    tree_bytes: bytes = b""
    skip_star: tuple = field(default_factory=tuple)

    @property
    def num_docs(self):
        return self.dims.shape[0]


def pair_name(function, column):
    return "%s__%s" % (function.lower() if function.upper() != "DISTINCTCOUNTHLL" else "distinctCountHLL", column)


class _Node:
    __slots__ = ("dim", "value", "start", "end", "agg", "children", "child_dim")

    def __init__(self, dim, value, start, end):
        self.dim, self.value, self.start, self.end = dim, value, start, end
        self.agg, self.children, self.child_dim = -1, None, -1


def _merge(kinds, a, b):
    out = []
    for k, x, y in zip(kinds, a, b):
        if k == "avg":  # AvgValueAggregator.applyAggregatedValue: AvgPair sum + sum, count + count
            out.append((x[0] + y[0], x[1] + y[1]))
        elif k == "distinctcounthll":  # DistinctCountHLLValueAggregator: HyperLogLog.addAll (register max)
            out.append(np.maximum(x, y))
        else:
            out.append(x + y if k in ("count", "sum") else (min(x, y) if k == "min" else max(x, y)))
    return out


def build_star_tree(seg, dimensions, pairs, max_leaf_records=10000, skip_star=()):
    """pairs: [(FUNCTION, column)] with FUNCTION in COUNT (column "*"), SUM, MIN, MAX, AVG (AvgPair values),
    DISTINCTCOUNTHLL (HyperLogLog registers)."""
    n = seg.num_docs
    k = len(dimensions)
    raw_dims = np.stack([np.asarray(seg.column(d)._dict_ids if seg.column(d)._dict_ids is not None else
                                    _read_ids(seg.column(d)), dtype=np.int64) for d in dimensions], axis=1) \
        if n else np.zeros((0, k), dtype=np.int64)
    kinds = [f.lower() for f, _ in pairs]
    names = [pair_name(f, c) for f, c in pairs]
    raw_metrics = []
    for f, c in pairs:
        if f.upper() == "COUNT":
            raw_metrics.append(np.ones(n, dtype=np.int64))
        elif f.upper() == "DISTINCTCOUNTHLL":  # getInitialAggregatedValue: a HyperLogLog offered the value
            import pinot_oracle as O
            from hll import register_and_rank_np
            col = seg.column(c)
            j, r = register_and_rank_np(O._value_hashes(col)[np.asarray(O.dict_ids(col))])
            regs = np.zeros((n, 256), dtype=np.uint8)
            regs[np.arange(n), j] = r
            raw_metrics.append(regs)
        else:
            col = seg.column(c)
            raw_metrics.append(np.asarray(col.dict_values(), dtype=np.float64)[np.asarray(col._dict_ids)])
    skip = {dimensions.index(d) for d in skip_star}

    # sortAndAggregateSegmentRecords: sort on all dimensions, merge identical tuples
    recs_d, recs_m = [], []
    if n:
        order = np.lexsort(tuple(raw_dims[:, j] for j in range(k - 1, -1, -1)))
        sd = raw_dims[order]
        sm = [m[order] for m in raw_metrics]
        new = np.ones(n, dtype=bool)
        new[1:] = np.any(sd[1:] != sd[:-1], axis=1)
        starts = np.nonzero(new)[0]
        recs_d = [list(map(int, sd[s])) for s in starts]
        for j, kind in enumerate(kinds):
            if kind == "distinctcounthll":
                recs_m.append(list(np.maximum.reduceat(sm[j], starts, axis=0)))
                continue
            if kind == "avg":  # getInitialAggregatedValue: AvgPair(value, 1)
                recs_m.append(list(zip(np.add.reduceat(sm[j], starts).tolist(),
                                       np.diff(np.append(starts, n)).tolist())))
                continue
            red = {"count": np.add, "sum": np.add, "min": np.minimum, "max": np.maximum}[kind]
            v = red.reduceat(sm[j], starts)
            recs_m.append(v.tolist())
        recs_m = [list(r) for r in zip(*recs_m)] if kinds else [[] for _ in starts]
    dims_list = recs_d
    mets_list = recs_m

    def append(d, m):
        dims_list.append(d)
        mets_list.append(m)

    root = _Node(ALL, ALL, ALL, ALL)  # TreeNode defaults: the root's doc range is never read

    def star_records(start, end, dim):  # generateRecordsForStarNode
        rows = list(range(start, end))
        rows.sort(key=lambda i: tuple(dims_list[i][dim + 1:]))
        out = []
        cur_key, cur_d, cur_m = None, None, None
        for i in rows:
            key = tuple(dims_list[i][dim + 1:])
            if key != cur_key:
                if cur_d is not None:
                    out.append((cur_d, cur_m))
                cur_key = key
                cur_d = list(dims_list[i])
                cur_d[dim] = STAR_IN_FORWARD_INDEX
                cur_m = list(mets_list[i])
            else:
                cur_m = _merge(kinds, cur_m, mets_list[i])
        if cur_d is not None:
            out.append((cur_d, cur_m))
        return out

    def construct(node, start, end):
        child_dim = node.dim + 1
        if child_dim == k:
            return
        node.child_dim = child_dim
        children = {}
        s = start
        for i in range(start + 1, end + 1):
            if i == end or dims_list[i][child_dim] != dims_list[s][child_dim]:
                v = dims_list[s][child_dim]
                children[v] = _Node(child_dim, v, s, i)
                s = i
        if child_dim not in skip and len(children) > 1:
            st = _Node(child_dim, ALL, len(dims_list), 0)
            for d, m in star_records(start, end, child_dim):
                append(d, m)
            st.end = len(dims_list)
            children[ALL] = st
        node.children = children
        for c in list(children.values()):
            if c.end - c.start > max_leaf_records:
                construct(c, c.start, c.end)

    if dims_list:
        construct(root, 0, len(dims_list))

    def aggregated(node):  # createAggregatedDocs
        if node.children is None:
            m = None
            for i in range(node.start, node.end):
                m = list(mets_list[i]) if m is None else _merge(kinds, m, mets_list[i])
            d = list(dims_list[node.start])
            for j in range(node.dim + 1, k):
                d[j] = STAR_IN_FORWARD_INDEX
            node.agg = len(dims_list)
            append(d, m)
            return d, m
        if ALL in node.children:
            rec = None
            for c in node.children.values():  # HashMap order is irrelevant to the result
                if c.value == ALL:
                    rec = aggregated(c)
                    node.agg = c.agg
                else:
                    aggregated(c)
            return rec
        m, d = None, None
        for c in node.children.values():
            cd, cm = aggregated(c)
            m = list(cm) if m is None else _merge(kinds, m, cm)
            d = list(cd)
        for j in range(node.dim + 1, k):
            d[j] = STAR_IN_FORWARD_INDEX
        node.agg = len(dims_list)
        append(d, m)
        return d, m

    if dims_list:
        aggregated(root)

    # BFS serialisation, children sorted by dimension value
    nodes = []
    queue = [root]
    qi = 0
    while qi < len(queue):
        nd = queue[qi]
        if nd.children is None:
            nodes.append((nd.dim, nd.value, nd.start, nd.end, nd.agg, -1, -1))
        else:
            kids = sorted(nd.children.values(), key=lambda c: c.value)
            first = len(queue)
            nodes.append((nd.dim, nd.value, nd.start, nd.end, nd.agg, first, first + len(kids) - 1))
            queue.extend(kids)
        qi += 1
    nodes = np.array(nodes, dtype=np.int32).reshape(-1, 7)
    dims = np.array(dims_list, dtype=np.int64).reshape(-1, k)
    metrics = {}
    for j, (name, kind) in enumerate(zip(names, kinds)):
        col = [m[j] for m in mets_list]
        if kind == "distinctcounthll":  # HyperLogLog registers per star doc, uint8 [num_docs, 256]
            metrics[name] = np.stack(col).astype(np.uint8) if col else np.zeros((0, 256), dtype=np.uint8)
            continue
        if kind == "avg":  # AvgPair per star doc: (sum double, count long)
            metrics[name] = (np.array([x[0] for x in col], dtype=np.float64), np.array([x[1] for x in col], dtype=np.int64))
            continue
        metrics[name] = np.array(col, dtype=np.int64 if kind == "count" else np.float64)
    st = StarTree(dimensions=list(dimensions), pairs=names, max_leaf_records=max_leaf_records, dims=dims,
                  metrics=metrics, nodes=nodes, skip_star=tuple(skip_star))
    st.tree_bytes = serialize_tree(dimensions, nodes)
    return st


def _read_ids(col):
    import pinot_oracle as O
    return O.dict_ids(col)


def hll_bytes(regs):
    """stream-lib HyperLogLog.getBytes of 256 registers: BE int log2m (8), BE int size in bytes (43 words * 4),
    then the RegisterSet words (register p at bit 5 * (p % 6) of word p / 6)."""
    words = [0] * 43
    for p_, r in enumerate(regs):
        words[p_ // 6] |= int(r) << (5 * (p_ % 6))
    return struct.pack(">ii", 8, 172) + struct.pack(">43i", *[w - (1 << 32) if w >= 1 << 31 else w for w in words])


def serialize_tree(dimensions, nodes):
    """StarTreeBuilderUtils.serializeTree (little-endian)."""
    head = b""
    for i, d in enumerate(dimensions):
        b = d.encode("utf-8")
        head += struct.pack("<ii", i, len(b)) + b
    header_size = 8 + 4 + 4 + 4 + len(head) + 4
    out = struct.pack("<Qiii", MAGIC, 1, header_size, len(dimensions)) + head + struct.pack("<i", nodes.shape[0])
    return out + nodes.astype("<i4").tobytes()
