"""numEntriesScannedInFilter as the reference's filter iterators count it (CPU restatement).

TEST INFRASTRUCTURE (see pinot_oracle.py's header): the checker of the library's stats.exact=1 mode
(csrc/filter_stats.cpp). PC = pinot-core/src/main/java/org/apache/pinot/core.

A scan-based iterator counts every doc it examines: SVScanDocIdIterator / MVScanDocIdIterator next(), advance()
(-> next()), isMatch() and applyAnd() (PC/operator/dociditerators/SVScanDocIdIterator.java:77-159). Which docs it
examines follows from the doc-id sets the filter operators build and the iterators they hand out:
AndBlockDocIdSet (PC/operator/docidsets/AndBlockDocIdSet.java:50-227: updateMinMaxRange, fastIterator),
OrBlockDocIdSet, SortedDocIdSet, BitmapDocIdSet, ScanBasedSingleValueDocIdSet, and the iterators AndDocIdIterator,
OrDocIdIterator, SortedDocIdIterator, BitmapDocIdIterator, RangelessBitmapDocIdIterator. DocIdSetOperator calls the
root iterator's next() until EOF. Pinned by the reference's InterSegmentAggregationSingleValueQueriesTest statistics
(tests/test_oracle_kats.py).
"""
import numpy as np

import pinot_oracle as O

EOF = -(1 << 31)


class _Bits:
    def __init__(self, mask):
        self.m = np.asarray(mask, dtype=bool)
        self.n = self.m.shape[0]
        self.idx = np.nonzero(self.m)[0]

    def next_set(self, d):
        i = int(np.searchsorted(self.idx, d))
        return int(self.idx[i]) if i < self.idx.shape[0] else -1


class Scan:
    index_based, scan_based = False, True

    def __init__(self, bits):
        self.b, self.cur, self.start, self.end, self.scanned = bits, -1, 0, 0, 0

    def set_start(self, s):
        self.cur, self.start = s - 1, s

    def set_end(self, e):
        self.end = e

    def next(self):
        if self.cur == EOF:
            return EOF
        last = min(self.end, self.b.n - 1)
        if self.cur < last:
            f = self.b.next_set(self.cur + 1)
            if 0 <= f <= last:
                self.scanned += f - self.cur
                self.cur = f
                return f
            self.scanned += last - self.cur
        self.cur = EOF
        return EOF

    def advance(self, t):
        if self.cur == EOF:
            return EOF
        if t < self.start:
            t = self.start
        elif t > self.end:
            self.cur = EOF
        if self.cur >= t:
            return self.cur
        self.cur = t - 1
        return self.next()

    def is_match(self, d):
        if self.cur == EOF:
            return False
        self.scanned += 1
        return bool(self.b.m[d])

    def apply_and(self, answer):
        out = np.zeros_like(answer)
        d = -1
        for x in np.nonzero(answer)[0]:
            if d >= self.end:
                break
            d = int(x)
            if d >= self.start:
                self.scanned += 1
                out[d] = self.b.m[d]
        return out


class BitmapIt:
    index_based, scan_based = True, False

    def __init__(self, mask, start=0, end=(1 << 31) - 1, ranged=True):
        self.b, self.cur, self.pos, self.start, self.end, self.ranged = _Bits(mask), -1, -1, start, end, ranged

    def next(self):
        if self.cur == EOF:
            return EOF
        x = self.b.next_set(self.pos + 1)
        if x < 0:
            self.cur = EOF
            return EOF
        self.pos = x
        if self.ranged:
            while x < self.start:
                y = self.b.next_set(x + 1)
                if y < 0:
                    break
                x = self.pos = y
            if x < self.start or self.end < x:
                self.cur = EOF
                return EOF
        self.cur = x
        return x

    def advance(self, t):
        assert not t < self.cur, "bitmap iterator moved backwards"
        if self.cur == t:
            return self.cur
        c = self.next()
        while c < t and c != EOF:
            c = self.next()
        return c


class SortedIt:
    index_based, scan_based = True, False

    def __init__(self, pairs):
        self.p, self.ptr, self.cur = pairs, 0, -1

    def advance(self, t):
        p = self.p
        if self.ptr == len(p) or t > p[-1][1]:
            self.ptr = len(p)
            self.cur = EOF
            return EOF
        if self.cur >= t:
            return self.cur
        while self.ptr < len(p):
            if p[self.ptr][0] > t:
                self.cur = p[self.ptr][0]
                break
            if p[self.ptr][0] <= t <= p[self.ptr][1]:
                self.cur = t
                break
            self.ptr += 1
        if self.ptr == len(p):
            self.cur = EOF
        return self.cur

    def next(self):
        p = self.p
        if self.ptr == len(p) or self.cur > p[-1][1]:
            self.ptr = len(p)
            self.cur = EOF
            return EOF
        self.cur += 1
        if self.ptr < len(p) and self.cur > p[self.ptr][1]:
            self.ptr += 1
            self.cur = EOF if self.ptr == len(p) else p[self.ptr][0]
        elif self.cur < p[self.ptr][0]:
            self.cur = p[self.ptr][0]
        return self.cur


class EmptyIt:
    index_based = scan_based = False

    def next(self):
        return EOF

    def advance(self, t):
        return EOF


class AndIt:
    index_based = scan_based = False

    def __init__(self, its):
        ni = sum(i.index_based for i in its)
        ns = sum(i.scan_based for i in its)
        self.has_scan = ni > 0 and ns > 0
        self.its = [i for i in its if not (self.has_scan and i.scan_based)]
        self.scans = [i for i in its if self.has_scan and i.scan_based]
        self.cur, self.cmax = -1, -1

    def advance(self, t):
        if self.cur == EOF or self.cur >= t:
            return self.cur
        self.cmax = t - 1
        return self.next()

    def next(self):
        if self.cur == EOF:
            return EOF
        self.cmax += 1
        n, i = len(self.its), 0
        while i < n:
            p = self.its[i].advance(self.cmax)
            if p == EOF:
                self.cmax = EOF
                break
            if p > self.cmax:
                self.cmax = p
                if i > 0:
                    i = -1
            if self.has_scan and i == n - 1:
                for s in self.scans:
                    if not s.is_match(self.cmax):
                        i = -1
                        self.cmax += 1
                        break
            i += 1
        self.cur = self.cmax
        return self.cur


class OrIt:
    index_based = scan_based = False

    def __init__(self, its, mn, mx):
        self.its, self.minv, self.maxv, self.cur = list(its), mn, mx, -1
        self.nxt = [i.advance(mn) for i in self.its]
        self._drop()

    def _drop(self):
        keep = [(i, d) for i, d in zip(self.its, self.nxt) if d != EOF]
        # removeExhaustedIterators swaps the last live iterator in; the order only decides who is advanced first,
        # which does not change any iterator's own examined docs
        self.its, self.nxt = [k[0] for k in keep], [k[1] for k in keep]

    def _step(self, t=None):
        best, ex = None, False
        for k, it in enumerate(self.its):
            d = self.nxt[k]
            if t is None and d == self.cur:
                d = self.nxt[k] = it.next()
            elif t is not None and d < t:
                d = self.nxt[k] = it.advance(t)
            if d != EOF:
                best = d if best is None else min(best, d)
            else:
                ex = True
        if best is None or best > self.maxv:
            self.cur = EOF
        else:
            self.cur = best
            if ex:
                self._drop()
        return self.cur

    def next(self):
        if self.cur == EOF:
            return EOF
        return self._step()

    def advance(self, t):
        if self.cur == EOF:
            return EOF
        if t > self.maxv:
            self.cur = EOF
            return EOF
        if t <= self.cur:
            return self.cur
        return self._step(max(t, self.minv))


class Set:
    def __init__(self, kind, mask=None, n=0, mv=False):
        self.kind, self.mask, self.kids, self.mv, self.n = kind, mask, [], mv, n
        self.minv, self.maxv = 0, n - 1
        self.pairs = []
        if kind == "SORTED":
            idx = np.nonzero(mask)[0]
            if idx.shape[0]:
                breaks = np.nonzero(np.diff(idx) != 1)[0]
                starts = np.concatenate([[idx[0]], idx[breaks + 1]])
                ends = np.concatenate([idx[breaks], [idx[-1]]])
                self.pairs = [(int(a), int(b)) for a, b in zip(starts, ends)]
        if kind == "SCAN":
            self.scan = Scan(_Bits(mask))
            self.scan.set_start(0)
            self.scan.set_end(n - 1)

    def min_doc(self):
        return (self.pairs[0][0] if self.pairs else 0) if self.kind == "SORTED" else self.minv

    def max_doc(self):
        return (self.pairs[-1][1] if self.pairs else 0) if self.kind == "SORTED" else self.maxv

    def set_start(self, s):
        if self.kind == "SCAN":
            self.minv = s
            self.scan.set_start(s)
        elif self.kind in ("BITMAP", "OR"):
            self.minv = s if self.kind == "BITMAP" else max(self.minv, s)
        elif self.kind == "AND":
            self.minv = max(self.minv, s)
            self.update_range()

    def set_end(self, e):
        if self.kind == "SCAN":
            self.maxv = e
            self.scan.set_end(e)
        elif self.kind in ("BITMAP", "OR"):
            self.maxv = e if self.kind == "BITMAP" else min(self.maxv, e)
        elif self.kind == "AND":
            self.maxv = min(self.maxv, e)
            self.update_range()

    def update_range(self):
        for k in self.kids:
            self.minv = max(self.minv, k.min_doc())
            self.maxv = min(self.maxv, k.max_doc())
        for k in self.kids:
            k.set_start(self.minv)
            k.set_end(self.maxv)

    def entries(self):
        return (self.scan.scanned if self.kind == "SCAN" else 0) + sum(k.entries() for k in self.kids)

    def _pairs_mask(self, pairs, n):
        m = np.zeros(n, dtype=bool)
        for a, b in pairs:
            m[a:b + 1] = True
        return m

    def iterator(self):
        if self.kind == "SORTED":
            return SortedIt(self.pairs) if self.pairs else EmptyIt()
        if self.kind == "BITMAP":
            return BitmapIt(self.mask, self.minv, self.maxv)
        if self.kind == "SCAN":
            return self.scan
        if self.kind == "AND":
            return self._and_iterator()
        return self._or_iterator()

    def _and_iterator(self):
        sorted_, bitmaps, scans, rest = [], [], [], []
        for k in self.kids:
            if k.kind == "SORTED":
                sorted_.append(k)
            elif k.kind == "BITMAP":
                bitmaps.append(k)
            elif k.kind == "SCAN":
                scans.append(k)
            else:
                rest.append(k.iterator())
        if not sorted_ and not bitmaps:
            return AndIt([k.iterator() for k in self.kids])
        n = self.n
        answer = None
        for s in sorted_:
            m = self._pairs_mask(s.pairs, n)
            answer = m if answer is None else answer & m
        for b in bitmaps:
            answer = b.mask.copy() if answer is None else answer & b.mask
        for s in scans:
            answer = answer & s.scan.apply_and(answer)
        first = BitmapIt(answer, ranged=False)
        return first if not rest else AndIt([first] + rest)

    def _or_iterator(self):
        its = []
        if any(k.kind == "BITMAP" for k in self.kids):
            n = self.n
            u = np.zeros(n, dtype=bool)
            for k in self.kids:
                if k.kind == "SORTED":
                    u |= self._pairs_mask(k.pairs, n)
                elif k.kind == "BITMAP":
                    u |= k.mask
                else:
                    its.append(k.iterator())
            b = BitmapIt(u, self.minv, self.maxv)
            if not its:
                return b
            its.append(b)
        else:
            its = [k.iterator() for k in self.kids]
        return OrIt(its, self.minv, self.maxv)


def _priority(s):
    return {"SORTED": 0, "BITMAP": 1, "AND": 2, "OR": 3}.get(s.kind, 5 if s.mv else 4)


def _build(segment, tree):
    """(kind, set): kind in "SET", "EMPTY", "ALL" — FilterPlanNode / FilterOperatorUtils folding."""
    op = tree["operator"]
    n = segment.num_docs
    if op in ("AND", "OR"):
        s = Set(op, n=n)
        for c in tree["children"]:
            k, cs = _build(segment, c)
            if op == "AND":
                if k == "EMPTY":
                    return "EMPTY", None
                if k == "SET":
                    s.kids.append(cs)
            else:
                if k == "ALL":
                    return "ALL", None
                if k == "SET":
                    s.kids.append(cs)
        if not s.kids:
            return ("ALL" if op == "AND" else "EMPTY"), None
        if len(s.kids) == 1:
            return "SET", s.kids[0]
        if op == "AND":
            s.kids.sort(key=_priority)  # stable
            s.minv, s.maxv = -(1 << 31), (1 << 31) - 1
            s.update_range()
        else:
            s.minv = min(k.min_doc() for k in s.kids)
            s.maxv = max(k.max_doc() for k in s.kids)
        return "SET", s
    col = segment.column(tree["column"])
    if getattr(col, "encoding", "dictionary") == "raw":
        mask = O.raw_leaf_mask(tree, col)
        kind = "SCAN"
        ev = None
    else:
        ev = O.make_evaluator(tree, col)
        if ev.always_false:
            return "EMPTY", None
        if ev.always_true:
            return "ALL", None
        mask = O.filter_mask(segment, tree)
        kind = "SCAN"
        if col.has_inverted_index and ev.kind != "RANGE":
            kind = "SORTED" if col.is_sorted else "BITMAP"
    return "SET", Set(kind, mask=mask, n=n, mv=O.is_mv(col))


def entries_scanned_in_filter(segment, tree):
    """numEntriesScannedInFilter of one segment (DocIdSetOperator: the root iterator's next() until EOF)."""
    if tree is None or segment.num_docs == 0:
        return 0
    kind, root = _build(segment, tree)
    if kind != "SET":
        return 0
    it = root.iterator()
    while it.next() != EOF:
        pass
    return root.entries()
