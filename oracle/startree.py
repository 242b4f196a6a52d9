"""Star-tree v2 query plan (CPU restatement; TEST INFRASTRUCTURE, see pinot_oracle.py's header).

PC = pinot-core/src/main/java/org/apache/pinot/core.
  * StarTreeUtils.isFitForStarTree (PC/startree/StarTreeUtils.java:50-95): every aggregation's function-column pair
    is in the tree, group-by columns and filter columns are split-order dimensions, no OR in the filter;
  * StarTreeFilterOperator (PC/startree/operator/StarTreeFilterOperator.java): predicate evaluators per column on the
    segment's dictionary (always-false -> empty, always-true dropped), the BFS traversal (a node with nothing left
    to match contributes its aggregated doc; a leaf its doc range plus the predicates still to apply; a predicate
    dimension's children are those of its matching dictIds; a dimension neither filtered nor grouped takes the star
    child when there is one; a grouped dimension takes every non-star child), then the remaining predicates over the
    star-tree docs (AND);
  * StarTreeAggregationExecutor / StarTreeGroupByExecutor: the function applied to the pre-aggregated column
    (COUNT sums count__*, SUM sums sum__x, MIN / MAX over min__x / max__x, AVG merges the avg__x AvgPairs,
    DISTINCTCOUNTHLL merges the distinctCountHLL__x HyperLogLogs), the docs scanned = the matched star docs.
A query the tree does not fit runs the regular plan (pinot_oracle.execute_segment).
"""
import numpy as np

import pinot_oracle as O

ALL = -1
_FN = {"COUNT": "count", "SUM": "sum", "MIN": "min", "MAX": "max", "AVG": "avg", "DISTINCTCOUNTHLL": "distinctCountHLL"}


def pair_of(agg):
    f = agg["function"].upper()
    if f not in _FN:
        return None
    return "%s__%s" % (_FN[f], "*" if f == "COUNT" else agg["column"])


def _leaves(tree):
    if tree is None:
        return []
    if tree["operator"] in ("AND", "OR"):
        out = []
        for c in tree["children"]:
            out += _leaves(c)
        return out
    return [tree]


def _has_or(tree):
    return tree is not None and (tree["operator"] == "OR" or
                                 (tree["operator"] == "AND" and any(_has_or(c) for c in tree["children"])))


def fits(st, query):
    for a in query["aggregations"]:
        p = pair_of(a)
        if p is None or p not in st.pairs:
            return False
    dims = set(st.dimensions)
    gb = query.get("group_by")
    if gb and not set(gb["columns"]) <= dims:
        return False
    f = query.get("filter")
    if f is None:
        return True
    return not _has_or(f) and all(l["column"] in dims for l in _leaves(f))


def _node(st, i):
    return tuple(int(x) for x in st.nodes[i])  # (dim, value, start, end, agg, first, last)


def matched_docs(segment, st, query):
    """The star-tree docs the filter operator returns (bool[num_star_docs]), or None when the result is empty."""
    gb = set(query["group_by"]["columns"]) if query.get("group_by") else set()
    evs = {}
    for leaf in _leaves(query.get("filter")):
        ev = O.make_evaluator(leaf, segment.column(leaf["column"]))
        if ev.always_false:
            return None
        if not ev.always_true:
            evs.setdefault(leaf["column"], []).append(ev)
    gb -= set(evs)
    dim_index = {d: i for i, d in enumerate(st.dimensions)}
    matching = {c: np.logical_and.reduce([e.matching for e in es]) for c, es in evs.items()}
    ndocs = st.num_docs
    out = np.zeros(ndocs, dtype=bool)
    remaining_cols = set()
    queue = [(0, frozenset(evs), frozenset(gb))]
    qi = 0
    while qi < len(queue):
        nid, rem_p, rem_g = queue[qi]
        qi += 1
        dim, value, start, end, agg, first, last = _node(st, nid)
        if not rem_p and not rem_g:
            out[agg] = True
            continue
        if first == -1:
            out[start:end] = True
            remaining_cols |= rem_p
            continue
        next_dim = st.dimensions[_node(st, first)[0]]
        kids = range(first, last + 1)
        if next_dim in rem_p:
            m = matching[next_dim]
            if not m.any():
                return None
            new_p = rem_p - {next_dim}
            for c in kids:
                v = _node(st, c)[1]
                if v != ALL and m[v]:
                    queue.append((c, new_p, rem_g))
        else:
            if next_dim not in rem_g:
                star = [c for c in kids if _node(st, c)[1] == ALL]
                if star:
                    queue.append((star[0], rem_p, rem_g))
                    continue
                new_g = rem_g
            else:
                new_g = rem_g - {next_dim}
            for c in kids:
                if _node(st, c)[1] != ALL:
                    queue.append((c, rem_p, new_g))
    for c in remaining_cols:
        out &= matching[c][st.dims[:, dim_index[c]]]
    return out


def execute_segment(segment, st, query):
    """(intermediate result, numDocsScanned) of one segment on its star-tree, as pinot_oracle.execute_segment."""
    docs = matched_docs(segment, st, query)
    sel = np.nonzero(docs)[0] if docs is not None else np.zeros(0, dtype=np.int64)
    aggs = query["aggregations"]
    if not query.get("group_by"):
        return [_agg(st, a, sel) for a in aggs], int(sel.shape[0])
    cols = query["group_by"]["columns"]
    ids = [st.dims[sel, st.dimensions.index(c)] for c in cols]
    groups = {}
    for r in range(sel.shape[0]):
        groups.setdefault(tuple(int(x[r]) for x in ids), []).append(sel[r])
    out = {}
    for key, rows in groups.items():
        parts = [O._string_value(segment.column(c), segment.column(c).dict_values()[v]) for c, v in zip(cols, key)]
        out["\t".join(parts)] = [_agg(st, a, np.array(rows, dtype=np.int64)) for a in aggs]
    return out, int(sel.shape[0])


def _agg(st, a, sel):
    f = a["function"].upper()
    if f == "AVG":  # AvgAggregationFunction.aggregate over AvgPair values: sums and counts added
        s, c = st.metrics[pair_of(a)]
        return (O._seq_sum(s[sel]), int(c[sel].sum()))
    if f == "DISTINCTCOUNTHLL":  # DistinctCountHLLAggregationFunction over HyperLogLog values: addAll
        h = O.HyperLogLog()
        regs = st.metrics[pair_of(a)][sel]
        if regs.shape[0]:
            h.reg = regs.max(axis=0).astype(np.int32)
        return h
    v = st.metrics[pair_of(a)][sel]
    if f == "COUNT":
        return int(v.sum())
    if f == "SUM":
        return O._seq_sum(v.astype(np.float64))
    if f == "MIN":
        return float(v.min()) if v.shape[0] else float("inf")
    return float(v.max()) if v.shape[0] else float("-inf")


def execute_server(segments, trees, query):
    """Per segment the star-tree plan when its tree fits, else the regular plan; combined as the server does."""
    results = []
    for seg, st in zip(segments, trees):
        if st is not None and fits(st, query):
            results.append(execute_segment(seg, st, query))
        else:
            results.append(O.execute_segment(seg, query))
    scanned = sum(r[1] for r in results)
    fns = [O.sv(a["function"]) for a in query["aggregations"]]
    if query.get("group_by"):
        return O.combine_group_by(query, [r[0] for r in results]), scanned
    acc = None
    for r, _ in results:
        acc = list(r) if acc is None else [O.merge_agg(f, x, y) for f, x, y in zip(fns, acc, r)]
    return acc, scanned
