// numEntriesScannedInFilter as a Java server reports it (stats.exact=1).
//
// The reference counts one entry per doc a scan-based iterator examines (SVScanDocIdIterator.java:77-159,
// MVScanDocIdIterator.java:78-160: next(), advance() -> next(), isMatch(), applyAnd()), and which docs those are
// follows from the iterator protocol the filter tree's doc-id sets drive: AndBlockDocIdSet.fastIterator (:144-227:
// sorted ranges and bitmaps intersected first, each scan child then applyAnd'ed over the running answer, nested
// AND / OR children leap-frogged against the answer by AndDocIdIterator), AndDocIdIterator (:55-117, index-based
// iterators leap-frogged, scan-based ones asked isMatch at each candidate), OrBlockDocIdSet / OrDocIdIterator, and the
// doc ranges (min / max doc ids) AndBlockDocIdSet pushes into its children. The GPU evaluates every leaf in bulk, so
// the count is a property of that protocol, not of the work done here: this file replays the protocol on the
// host over the leaves' match bitsets (each computed on the device by exec_filter, downloaded), iterator by
// iterator, with the same tie and end-of-range behaviour. Cost: one device filter + D2H per leaf and a host pass
// proportional to the docs the iterators visit — opt-in, off the query's hot path.
#include <algorithm>
#include <memory>
#include <vector>

#include "engine.h"

namespace pinot {
namespace {

constexpr int kEOF = INT32_MIN;  // Constants.EOF

struct Bits {
  std::vector<uint64_t> w;
  int32_t n = 0;
  bool test(int32_t d) const { return (w[(size_t)d >> 6] >> (d & 63)) & 1ull; }
  // first set bit >= d (d >= 0), or -1
  int32_t next_set(int32_t d) const {
    if (d >= n) return -1;
    size_t i = (size_t)d >> 6;
    uint64_t x = w[i] & (~0ull << (d & 63));
    while (true) {
      if (x) {
        const int32_t r = (int32_t)(i * 64 + __builtin_ctzll(x));
        return r < n ? r : -1;
      }
      if (++i >= w.size()) return -1;
      x = w[i];
    }
  }
};

struct Iter {
  virtual ~Iter() = default;
  virtual int next() = 0;
  virtual int advance(int target) = 0;
  virtual bool index_based() const { return false; }
  virtual bool scan_based() const { return false; }
};

struct EmptyIter : Iter {  // EmptyBlockDocIdIterator
  int next() override { return kEOF; }
  int advance(int) override { return kEOF; }
};

// SVScanDocIdIterator / MVScanDocIdIterator: one entry per examined doc
struct ScanIter : Iter {
  const Bits *m;
  int cur = -1, start = 0, end = 0;
  int64_t scanned = 0;
  bool scan_based() const override { return true; }
  void set_start(int s) { cur = s - 1; start = s; }
  void set_end(int e) { end = e; }
  int next() override {
    if (cur == kEOF) return kEOF;
    // while (hasNext && cur < end) { cur++; scanned++; if match return cur }
    const int last = std::min(end, m->n - 1);
    if (cur < last) {
      const int32_t f = m->next_set(cur + 1);
      if (f >= 0 && f <= last) {
        scanned += f - cur;
        cur = f;
        return cur;
      }
      scanned += last - cur;
    }
    cur = kEOF;
    return kEOF;
  }
  int advance(int t) override {
    if (cur == kEOF) return kEOF;
    if (t < start) t = start;
    else if (t > end) cur = kEOF;
    if (cur >= t) return cur;
    cur = t - 1;
    return next();
  }
  bool is_match(int d) {
    if (cur == kEOF) return false;
    scanned++;
    return m->test(d);
  }
  Bits apply_and(const Bits &answer) {  // docs of answer, in order, while the previous one is < end
    Bits r;
    r.n = answer.n;
    r.w.assign(answer.w.size(), 0);
    int d = -1;
    for (int32_t x = answer.next_set(0); x >= 0 && d < end; x = answer.next_set(x + 1)) {
      d = x;
      if (d >= start) {
        scanned++;
        if (m->test(d)) r.w[(size_t)d >> 6] |= 1ull << (d & 63);
      }
    }
    return r;
  }
};

// BitmapDocIdIterator (start / end) and RangelessBitmapDocIdIterator (rangeless)
struct BitmapIter : Iter {
  Bits b;
  int cur = -1, start = 0, end = INT32_MAX;
  int pos = -1;  // last doc the IntIterator returned
  bool ranged = true;
  bool index_based() const override { return true; }
  int next() override {
    if (cur == kEOF) return kEOF;
    int x = b.next_set(pos + 1);
    if (x < 0) return cur = kEOF;
    pos = x;
    if (ranged) {
      while (x < start) {
        const int y = b.next_set(x + 1);
        if (y < 0) break;
        x = pos = y;
      }
      if (x < start || end < x) return cur = kEOF;
    }
    return cur = x;
  }
  int advance(int t) override {
    require(!(t < cur), PINOT_ERR_DEVICE, "bitmap iterator moved backwards (the reference throws here)");
    if (cur == t) return cur;
    int c = next();
    while (c < t && c != kEOF) c = next();
    return c;
  }
};

struct SortedIter : Iter {  // SortedDocIdIterator
  std::vector<std::pair<int, int>> p;
  size_t ptr = 0;
  int cur = -1;
  bool index_based() const override { return true; }
  int advance(int t) override {
    if (ptr == p.size() || t > p.back().second) {
      ptr = p.size();
      return cur = kEOF;
    }
    if (cur >= t) return cur;
    while (ptr < p.size()) {
      if (p[ptr].first > t) { cur = p[ptr].first; break; }
      if (t >= p[ptr].first && t <= p[ptr].second) { cur = t; break; }
      ptr++;
    }
    if (ptr == p.size()) cur = kEOF;
    return cur;
  }
  int next() override {
    if (ptr == p.size() || cur > p.back().second) {
      ptr = p.size();
      return cur = kEOF;
    }
    cur = cur + 1;
    if (ptr < p.size() && cur > p[ptr].second) {
      ptr++;
      cur = ptr == p.size() ? kEOF : p[ptr].first;
    } else if (cur < p[ptr].first) {
      cur = p[ptr].first;
    }
    return cur;
  }
};

struct AndIter : Iter {  // AndDocIdIterator
  std::vector<Iter *> its;
  std::vector<ScanIter *> scans;
  std::vector<int> ptrs;
  bool has_scan = false;
  int cur = -1, cmax = -1;
  explicit AndIter(const std::vector<Iter *> &in) {
    int n_index = 0, n_scan = 0;
    for (Iter *i : in) {
      n_index += i->index_based();
      n_scan += i->scan_based();
    }
    if (n_index > 0 && n_scan > 0) {
      has_scan = true;
      for (Iter *i : in) {
        if (i->scan_based()) scans.push_back(static_cast<ScanIter *>(i));
        else its.push_back(i);
      }
    } else {
      its = in;
    }
    ptrs.assign(its.size(), -1);
  }
  int advance(int t) override {
    if (cur == kEOF) return cur;
    if (cur >= t) return cur;
    cmax = t - 1;
    return next();
  }
  int next() override {
    if (cur == kEOF) return cur;
    cmax = cmax + 1;
    const int n = (int)its.size();
    for (int i = 0; i < n; i++) {
      ptrs[i] = its[i]->advance(cmax);
      if (ptrs[i] == kEOF) {
        cmax = kEOF;
        break;
      }
      if (ptrs[i] > cmax) {
        cmax = ptrs[i];
        if (i > 0) i = -1;
      }
      if (has_scan && i == n - 1) {
        for (ScanIter *s : scans)
          if (!s->is_match(cmax)) {
            i = -1;
            cmax = cmax + 1;
            break;
          }
      }
    }
    return cur = cmax;
  }
};

struct OrIter : Iter {  // OrDocIdIterator
  std::vector<Iter *> its;
  std::vector<int> nxt;
  int nlive, minv, maxv, cur = -1;
  OrIter(const std::vector<Iter *> &in, int mn, int mx) : its(in), nlive((int)in.size()), minv(mn), maxv(mx) {
    nxt.resize(in.size());
    for (int i = 0; i < nlive; i++) nxt[i] = its[i]->advance(mn);
    drop_exhausted();
  }
  void drop_exhausted() {
    int i = 0;
    while (i < nlive) {
      if (nxt[i] == kEOF) {
        nlive--;
        its[i] = its[nlive];
        nxt[i] = nxt[nlive];
      } else {
        i++;
      }
    }
  }
  int next() override {
    if (cur == kEOF) return kEOF;
    int best = INT32_MAX;
    bool exhausted = false;
    for (int i = 0; i < nlive; i++) {
      int d = nxt[i];
      if (d == cur) nxt[i] = d = its[i]->next();
      if (d != kEOF) best = std::min(best, d);
      else exhausted = true;
    }
    if (best > maxv) {
      cur = kEOF;
    } else {
      cur = best;
      if (exhausted) drop_exhausted();
    }
    return cur;
  }
  int advance(int t) override {
    if (cur == kEOF) return kEOF;
    if (t > maxv) return cur = kEOF;
    if (t <= cur) return cur;
    if (t < minv) t = minv;
    int best = INT32_MAX;
    bool exhausted = false;
    for (int i = 0; i < nlive; i++) {
      int d = nxt[i];
      if (d < t) nxt[i] = d = its[i]->advance(t);
      if (d != kEOF) best = std::min(best, d);
      else exhausted = true;
    }
    if (best > maxv) {
      cur = kEOF;
    } else {
      cur = best;
      if (exhausted) drop_exhausted();
    }
    return cur;
  }
};

// FilterBlockDocIdSet of the tree: the leaves' sets and AndBlockDocIdSet / OrBlockDocIdSet
struct DocSet {
  enum Kind { SORTED, BITMAP, SCAN, AND, OR } kind;
  Bits bits;                                 // leaves: the docs the predicate matches
  std::vector<std::pair<int, int>> pairs;    // SORTED: matching doc ranges
  std::unique_ptr<ScanIter> scan;            // SCAN: the set's one iterator
  std::vector<std::unique_ptr<DocSet>> kids;
  int minv = 0, maxv = 0;                    // BITMAP / SCAN: start / end; AND / OR: min / max doc ids
  bool mv = false;                           // SCAN over a multi-value column
  std::vector<std::unique_ptr<Iter>> owned;  // iterators this set created

  int min_doc() const { return kind == SORTED ? (pairs.empty() ? 0 : pairs.front().first) : minv; }
  int max_doc() const { return kind == SORTED ? (pairs.empty() ? 0 : pairs.back().second) : maxv; }
  void set_start(int s) {
    switch (kind) {
      case SORTED: break;  // stored by SortedDocIdSet, unused by its iterator
      case SCAN: minv = s; scan->set_start(s); break;
      case BITMAP: minv = s; break;
      case AND: minv = std::max(minv, s); update_range(); break;
      case OR: minv = std::max(minv, s); break;
    }
  }
  void set_end(int e) {
    switch (kind) {
      case SORTED: break;
      case SCAN: maxv = e; scan->set_end(e); break;
      case BITMAP: maxv = e; break;
      case AND: maxv = std::min(maxv, e); update_range(); break;
      case OR: maxv = std::min(maxv, e); break;
    }
  }
  void update_range() {  // AndBlockDocIdSet.updateMinMaxRange
    for (auto &k : kids) {
      minv = std::max(minv, k->min_doc());
      maxv = std::min(maxv, k->max_doc());
    }
    for (auto &k : kids) {
      k->set_start(minv);
      k->set_end(maxv);
    }
  }
  int64_t entries() const {
    int64_t s = kind == SCAN ? scan->scanned : 0;
    for (auto &k : kids) s += k->entries();
    return s;
  }
  Iter *keep(std::unique_ptr<Iter> it) {
    owned.push_back(std::move(it));
    return owned.back().get();
  }
  Iter *bitmap_iter(const Bits &b, int start, int end) {
    auto it = std::make_unique<BitmapIter>();
    it->b = b;
    it->start = start;
    it->end = end;
    return keep(std::move(it));
  }
  Iter *iterator() {
    switch (kind) {
      case SORTED: {
        if (pairs.empty()) return keep(std::make_unique<EmptyIter>());
        auto it = std::make_unique<SortedIter>();
        it->p = pairs;
        return keep(std::move(it));
      }
      case BITMAP: return bitmap_iter(bits, minv, maxv);
      case SCAN: return scan.get();
      case AND: return and_iterator();
      case OR: return or_iterator();
    }
    return nullptr;
  }
  Iter *and_iterator() {  // AndBlockDocIdSet.fastIterator
    std::vector<DocSet *> sorted, bitmaps, scans;
    std::vector<Iter *> rest;
    for (auto &k : kids) {
      if (k->kind == SORTED) sorted.push_back(k.get());
      else if (k->kind == BITMAP) bitmaps.push_back(k.get());
      else if (k->kind == SCAN) scans.push_back(k.get());
      else rest.push_back(k->iterator());
    }
    if (sorted.empty() && bitmaps.empty()) {
      std::vector<Iter *> all;
      rest.clear();
      for (auto &k : kids) all.push_back(k->iterator());
      return keep(std::make_unique<AndIter>(all));
    }
    Bits answer;
    bool have = false;
    const int32_t n = kids.front()->bits.n ? kids.front()->bits.n : 0;
    auto from_pairs = [&](const std::vector<std::pair<int, int>> &p, int32_t nd) {
      Bits b;
      b.n = nd;
      b.w.assign(((size_t)nd + 63) / 64, 0);
      for (auto &r : p)
        for (int d = r.first; d <= r.second; d++) b.w[(size_t)d >> 6] |= 1ull << (d & 63);
      return b;
    };
    if (!sorted.empty()) {  // SortedRangeIntersection of the range lists
      const int32_t nd = sorted.front()->bits.n;
      answer = from_pairs(sorted.front()->pairs, nd);
      for (size_t i = 1; i < sorted.size(); i++) {
        Bits o = from_pairs(sorted[i]->pairs, nd);
        for (size_t w = 0; w < answer.w.size(); w++) answer.w[w] &= o.w[w];
      }
      have = true;
    }
    for (DocSet *b : bitmaps) {  // the bitmaps as built (no start / end clipping)
      if (!have) {
        answer = b->bits;
        have = true;
      } else {
        for (size_t w = 0; w < answer.w.size(); w++) answer.w[w] &= b->bits.w[w];
      }
    }
    (void)n;
    for (DocSet *s : scans) {
      Bits r = s->scan->apply_and(answer);
      for (size_t w = 0; w < answer.w.size(); w++) answer.w[w] &= r.w[w];
    }
    auto it = std::make_unique<BitmapIter>();
    it->b = answer;
    it->ranged = false;  // RangelessBitmapDocIdIterator
    Iter *first = keep(std::move(it));
    if (rest.empty()) return first;
    std::vector<Iter *> all{first};
    all.insert(all.end(), rest.begin(), rest.end());
    return keep(std::make_unique<AndIter>(all));
  }
  Iter *or_iterator() {  // OrBlockDocIdSet.iterator
    bool bitmap_or = false;
    for (auto &k : kids) bitmap_or = bitmap_or || k->kind == BITMAP;
    std::vector<Iter *> its;
    if (bitmap_or) {
      Bits u;
      u.n = kids.front()->bits.n;
      for (auto &k : kids)
        if (k->bits.n) u.n = k->bits.n;
      u.w.assign(((size_t)u.n + 63) / 64, 0);
      for (auto &k : kids) {
        if (k->kind == SORTED) {
          for (auto &r : k->pairs)
            for (int d = r.first; d <= r.second; d++) u.w[(size_t)d >> 6] |= 1ull << (d & 63);
        } else if (k->kind == BITMAP) {
          for (size_t w = 0; w < u.w.size(); w++) u.w[w] |= k->bits.w[w];
        } else {
          its.push_back(k->iterator());
        }
      }
      Iter *b = bitmap_iter(u, minv, maxv);
      if (its.empty()) return b;
      its.push_back(b);
    } else {
      for (auto &k : kids) its.push_back(k->iterator());
    }
    return keep(std::make_unique<OrIter>(its, minv, maxv));
  }
};

int node_priority(const DocSet &d) {  // FilterOperatorUtils.reorderAndFilterChildOperators
  switch (d.kind) {
    case DocSet::SORTED: return 0;
    case DocSet::BITMAP: return 1;
    case DocSet::AND: return 2;
    case DocSet::OR: return 3;
    default: return d.mv ? 5 : 4;
  }
}

enum Folded { F_SET, F_EMPTY, F_ALL };

// The doc-id set tree of one segment, folded as FilterPlanNode / FilterOperatorUtils fold it (planner.cpp construct)
Folded build(Engine &e, SegmentData &s, const FilterTreeInput &t, std::unique_ptr<DocSet> &out) {
  if (t.op == PINOT_FILTER_AND || t.op == PINOT_FILTER_OR) {
    const bool is_and = t.op == PINOT_FILTER_AND;
    auto set = std::make_unique<DocSet>();
    set->kind = is_and ? DocSet::AND : DocSet::OR;
    for (const auto &ct : t.children) {
      std::unique_ptr<DocSet> c;
      const Folded f = build(e, s, ct, c);
      if (is_and) {
        if (f == F_EMPTY) return F_EMPTY;
        if (f == F_SET) set->kids.push_back(std::move(c));
      } else {
        if (f == F_ALL) return F_ALL;
        if (f == F_SET) set->kids.push_back(std::move(c));
      }
    }
    if (set->kids.empty()) return is_and ? F_ALL : F_EMPTY;
    if (set->kids.size() == 1) {
      out = std::move(set->kids[0]);
      return F_SET;
    }
    if (is_and) {
      std::stable_sort(set->kids.begin(), set->kids.end(), [](const std::unique_ptr<DocSet> &a,
                                                              const std::unique_ptr<DocSet> &b) {
        return node_priority(*a) < node_priority(*b);
      });
      set->minv = INT32_MIN;  // AndBlockDocIdSet: Integer.MIN_VALUE / MAX_VALUE, then the children's
      set->maxv = INT32_MAX;
      set->update_range();
    } else {
      set->minv = INT32_MAX;
      set->maxv = INT32_MIN;
      for (auto &k : set->kids) {
        set->minv = std::min(set->minv, k->min_doc());
        set->maxv = std::max(set->maxv, k->max_doc());
      }
    }
    out = std::move(set);
    return F_SET;
  }
  const FilterNode leaf = plan_filter(s, &t);
  const auto ci = s.by_name.find(t.column);
  // a raw column's RawValueBased evaluators are never always-true / always-false: its leaf is always scanned
  const bool raw = ci != s.by_name.end() && s.cols[ci->second]->raw;
  if (!raw && leaf.type == FilterNode::EMPTY) return F_EMPTY;
  if (!raw && leaf.type == FilterNode::MATCH_ALL) return F_ALL;
  auto set = std::make_unique<DocSet>();
  set->bits.n = s.num_docs;
  set->bits.w.assign((size_t)s.nwords(), 0);
  int64_t cnt = 0;
  exec_filter(e, s, &t, set->bits.w.data(), &cnt);
  set->minv = 0;
  set->maxv = s.num_docs - 1;
  if (leaf.type == FilterNode::SORTED) {
    set->kind = DocSet::SORTED;
    for (int32_t d = set->bits.next_set(0); d >= 0;) {  // the matching runs
      int32_t e2 = d;
      while (e2 + 1 < s.num_docs && set->bits.test(e2 + 1)) e2++;
      set->pairs.emplace_back(d, e2);
      d = set->bits.next_set(e2 + 1);
    }
  } else if (leaf.type == FilterNode::BITMAP) {
    set->kind = DocSet::BITMAP;
  } else {
    set->kind = DocSet::SCAN;
    set->mv = leaf.col >= 0 && s.cols[leaf.col]->mv;
    set->scan = std::make_unique<ScanIter>();
    set->scan->m = &set->bits;
    set->scan->set_start(0);
    set->scan->set_end(s.num_docs - 1);
  }
  out = std::move(set);
  return F_SET;
}

}  // namespace

int64_t filter_entries_scanned(Engine &e, SegmentData &s, const FilterTreeInput *tree) {
  if (!tree || s.num_docs == 0) return 0;
  std::unique_ptr<DocSet> root;
  if (build(e, s, *tree, root) != F_SET) return 0;
  // DocIdSetOperator: iterator().next() until EOF
  Iter *it = root->iterator();
  for (int d = it->next(); d != kEOF; d = it->next()) {
  }
  return root->entries();
}

}  // namespace pinot
