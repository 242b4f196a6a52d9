// Internal to the executor sources (executor.cpp: filter plans + aggregation; executor_group.cpp: group-by;
// executor_group_ext.cpp: multi-value / star-tree / bitset-path group-by and the multi-GPU partials;
// executor_server.cpp: the multi-GPU server's host pieces): the per-query plumbing they share — the filter-plan
// compiler, the query arena and scratch, kernel timing, the group-by key space and accumulator plans. Not part of the
// C-ABI (include/pinot_gpu.h) and not used outside these files.
#pragma once
#include <algorithm>
#include <cstring>
#include <functional>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "engine.h"
#include "mv_hash.h"

namespace pinot {

inline std::string agg_column(const pinot_agg_spec &a) {
  if (a.column == nullptr) return "*";
  return a.column;
}

struct Arena {
  std::vector<uint8_t> bytes;
  // Copies n bytes and reserves `pad` zero bytes after them (kernels may read a little past the end).
  size_t add(const void *p, size_t n, size_t pad = 16) {
    size_t off = (bytes.size() + 15) & ~size_t(15);
    bytes.resize(off + n + pad, 0);
    if (n) memcpy(bytes.data() + off, p, n);
    return off;
  }
};

// One device step of a segment's filter plan.
struct FilterStep {
  enum Kind { SCAN, RANGES, ROARING, COMBINE, FILL, MV_SCAN, FUSED_OP } kind;  // FUSED_OP: a nested term's close
  int col = -1;
  int leaf_kind = LEAF_RANGE;
  uint32_t lo = 0, span = 0;
  uint64_t lut64 = 0;
  size_t off = 0;  // arena offset (LUT words / ranges / ids)
  int n = 0;
  int negate = 0;  // SCAN: negate; ROARING: exclusive; FILL: value
  int mode = CM_WRITE;
  int dst = 0, src = 0;
  int join = JOIN_NEW;  // fused leaves: how the leaf joins the filter program (FusedJoin)
  // ROARING with more than kMaxFusedRoaringIds dictIds: the ids' containers listed per roaring key (arena: the key
  // directory [keys + 1] at key_off, the container indices at list_off) so the fused kernels OR a chunk's containers
  // without a search per id; 0 keys = not built (such a leaf is expanded to the `pre` bitset)
  int keys = 0;
  size_t key_off = 0, list_off = 0;
};

constexpr int kMaxFusedRoaringIds = 256;      // bitmap leaves with more dictIds need their per-key container list
constexpr int64_t kMaxFusedRoaringList = 1 << 18;  // ... of at most this many containers (arena bytes), else `pre`

struct SegPlan {
  SegmentData *seg = nullptr;
  bool empty = false, match_all = false;
  std::vector<FilterStep> steps;
  int slots = 1;
  int64_t scan_leaves = 0;
  // fused mode: scan leaves of the top-level conjunction, evaluated inside k_scan_query; `steps`
  // (if any) build the rest of the conjunction into slot 0, the kernel's `pre` bitset
  std::vector<FilterStep> fused_leaves;
  bool has_pre = false;
};

// FilterNode tree -> step list. eval(node, dst, mode): leaves write/AND/OR straight into dst; a composite
// child of a different operator is evaluated into a fresh slot and combined.
class Compiler {
 public:
  Compiler(Engine &e, SegPlan &sp, Arena &ar) : e_(e), sp_(sp), ar_(ar), seg_(*sp.seg) {}

  void run(const FilterTreeInput *tree) {
    FilterNode root = plan_filter(seg_, tree);
    if (root.type == FilterNode::EMPTY) { sp_.empty = true; return; }
    if (root.type == FilterNode::MATCH_ALL) { sp_.match_all = true; return; }
    next_slot_ = 1;
    eval(root, 0, CM_WRITE);
  }

  // Fused plan: the scan leaves of the top-level conjunction (AndFilterOperator puts scans last and
  // applies them only to the candidates of the index children, AndBlockDocIdSet.java:144-227) become
  // k_scan_query leaves; every other conjunct is built into slot 0 = the kernel's `pre` bitset.
  // Fused plan: the top-level conjunction (AndFilterOperator: index children first, scans last,
  // AndBlockDocIdSet.java:144-227) becomes a program of terms evaluated per chunk in registers: a term is
  // one leaf — scan (decoded from the staged column), sorted (doc ranges) or bitmap (roaring containers,
  // at most kMaxFusedRoaringIds dictIds) — or an AND / OR of such leaves (OrBlockDocIdSet.java:78-120).
  // Deeper subtrees, wider scans (> max_fused_bits: the group kernel's 16 wave stages are small) and long
  // bitmap lists are built into slot 0 = the kernel's `pre` bitset by the launch sequence.
  void run_fused(const FilterTreeInput *tree, int max_fused_bits = 32, int max_stack = kMaxFusedStack) {
    FilterNode root = plan_filter(seg_, tree);
    if (root.type == FilterNode::EMPTY) { sp_.empty = true; return; }
    if (root.type == FilterNode::MATCH_ALL) { sp_.match_all = true; return; }
    next_slot_ = 1;
    max_fused_bits_ = max_fused_bits;
    max_stack_ = max_stack;
    std::vector<const FilterNode *> conj;
    if (root.type == FilterNode::AND) {
      for (const auto &c : root.children) conj.push_back(&c);
    } else {
      conj.push_back(&root);
    }
    for (const FilterNode *c : conj) {
      const int mode = sp_.has_pre ? CM_AND : CM_WRITE;
      if (c->type == FilterNode::AND || c->type == FilterNode::OR) {
        if (fuse_term(*c)) continue;
        eval(*c, 0, mode);
        sp_.has_pre = true;
        continue;
      }
      if (c->type == FilterNode::EMPTY || c->type == FilterNode::MATCH_ALL) {
        eval(*c, 0, mode);
        sp_.has_pre = true;
        continue;
      }
      FilterStep st = leaf_step(*c);
      if (fusable(st)) {
        st.join = JOIN_NEW;
        sp_.fused_leaves.push_back(st);
      } else {
        st.dst = 0;
        st.mode = mode;
        sp_.steps.push_back(st);
        sp_.has_pre = true;
      }
    }
  }

 private:
  bool fusable(const FilterStep &st) const {
    if (st.kind == FilterStep::SCAN) return seg_.cols[st.col]->bits <= max_fused_bits_;
    if (st.kind == FilterStep::RANGES) return true;
    return st.kind == FilterStep::ROARING && (st.n <= kMaxFusedRoaringIds || st.keys > 0);
  }
  // The registers a term's postfix program holds below its running term (gen_term): a child combined into a running
  // term of another operator is pushed. first_need: as a node's first child (it starts the running term); join_need:
  // as a later child joining with operator op.
  static int first_need(const FilterNode &n) {
    if (n.type != FilterNode::AND && n.type != FilterNode::OR) return 0;
    const int op = n.type == FilterNode::OR ? JOIN_OR : JOIN_AND;
    int need = 0, best = -1;
    size_t first = 0;
    for (size_t i = 0; i < n.children.size(); i++) {  // the costliest joiner goes first (it then costs first_need)
      const int j = join_need(n.children[i], op);
      if (j > best) best = j, first = i;
    }
    for (size_t i = 0; i < n.children.size(); i++)
      need = std::max(need, i == first ? first_need(n.children[i]) : join_need(n.children[i], op));
    return need;
  }
  static int join_need(const FilterNode &n, int op) {
    if (n.type != FilterNode::AND && n.type != FilterNode::OR) return 0;
    const int nop = n.type == FilterNode::OR ? JOIN_OR : JOIN_AND;
    if (nop == op) {  // the same operator: its children join the running term directly
      int need = 0;
      for (const auto &c : n.children) need = std::max(need, join_need(c, op));
      return need;
    }
    return 1 + first_need(n);
  }
  // The tree with every node's costliest joiner first (AND / OR children commute): the deepest subtree starts the
  // running term instead of being pushed, so a chain of nested terms of any depth needs no register stack and a
  // bushy tree needs its Strahler number's worth (FilterOperatorUtils.java:74-122 builds either shape).
  static FilterNode deepest_first(const FilterNode &n) {
    if (n.type != FilterNode::AND && n.type != FilterNode::OR) return n;
    FilterNode r = n;
    const int op = n.type == FilterNode::OR ? JOIN_OR : JOIN_AND;
    for (auto &c : r.children) c = deepest_first(c);
    int best = -1;
    size_t first = 0;
    for (size_t i = 0; i < r.children.size(); i++) {
      const int j = join_need(r.children[i], op);
      if (j > best) best = j, first = i;
    }
    if (first) std::rotate(r.children.begin(), r.children.begin() + first, r.children.begin() + first + 1);
    return r;
  }
  // An AND / OR tree of fusable leaves -> one term of the fused program, in postfix over the kernel's register stack
  // (JOIN_PUSH / FUSED_OP: a child whose operator differs from its parent's is built above the parent's running
  // term, then combined). Trees deeper than the stack, or with an unfusable leaf, take the `pre` bitset instead.
  enum GenMode { GEN_START, GEN_PUSH, GEN_COMBINE };
  bool gen_term(const FilterNode &n, GenMode mode, int op, std::vector<FilterStep> &out, int &depth, int &max_depth) {
    if (n.type == FilterNode::EMPTY || n.type == FilterNode::MATCH_ALL) return false;
    if (n.type != FilterNode::AND && n.type != FilterNode::OR) {
      FilterStep st = leaf_step(n);
      if (!fusable(st)) return false;
      st.join = mode == GEN_START ? JOIN_NEW : mode == GEN_PUSH ? JOIN_PUSH : op;
      if (mode == GEN_PUSH) max_depth = std::max(max_depth, ++depth);
      out.push_back(st);
      return true;
    }
    if (n.children.empty()) return false;
    const int nop = n.type == FilterNode::OR ? JOIN_OR : JOIN_AND;
    if (mode == GEN_COMBINE && nop == op) {  // the parent's operator: its children join the running term directly
      for (const auto &c : n.children)
        if (!gen_term(c, GEN_COMBINE, op, out, depth, max_depth)) return false;
      return true;
    }
    const bool nested = mode == GEN_COMBINE;
    if (!gen_term(n.children[0], nested ? GEN_PUSH : mode, -1, out, depth, max_depth)) return false;
    for (size_t i = 1; i < n.children.size(); i++)
      if (!gen_term(n.children[i], GEN_COMBINE, nop, out, depth, max_depth)) return false;
    if (nested) {  // close: term = (the parent's running term) op term
      FilterStep cl{FilterStep::FUSED_OP};
      cl.join = op;
      out.push_back(cl);
      depth--;
    }
    return true;
  }
  bool fuse_term(const FilterNode &n0) {
    const int64_t scans_before = sp_.scan_leaves;
    std::vector<FilterStep> steps;
    int depth = 0, max_depth = 0;
    const FilterNode n = deepest_first(n0);
    if (!gen_term(n, GEN_START, -1, steps, depth, max_depth) || max_depth > max_stack_) {
      sp_.scan_leaves = scans_before;  // eval() plans these leaves again
      return false;
    }
    for (auto &st : steps) sp_.fused_leaves.push_back(st);
    return true;
  }
  int alloc_slot() {
    const int s = next_slot_++;
    sp_.slots = std::max(sp_.slots, next_slot_);
    return s;
  }
  void eval(const FilterNode &n, int dst, int mode) {
    if (n.type != FilterNode::AND && n.type != FilterNode::OR) {
      leaf(n, dst, mode);
      return;
    }
    const int op = n.type == FilterNode::AND ? CM_AND : CM_OR;
    if (mode != CM_WRITE && mode != op) {  // e.g. OR-node into an AND accumulation: build it aside
      const int t = alloc_slot();
      eval(n, t, CM_WRITE);
      FilterStep c{FilterStep::COMBINE};
      c.dst = dst;
      c.src = t;
      c.mode = mode;
      sp_.steps.push_back(c);
      next_slot_--;
      return;
    }
    for (size_t i = 0; i < n.children.size(); i++) eval(n.children[i], dst, i == 0 && mode == CM_WRITE ? CM_WRITE : op);
  }
  void leaf(const FilterNode &n, int dst, int mode) {
    FilterStep st = leaf_step(n);
    st.dst = dst;
    st.mode = mode;
    sp_.steps.push_back(st);
  }
  // Physical leaf (getLeafFilterOperator + this engine's cost model): SCAN, RANGES or ROARING.
  FilterStep leaf_step(const FilterNode &n) {
    const ColumnData &c = *seg_.cols[n.col];
    const Evaluator &ev = *n.ev;
    const bool force_scan = e_.force_filter == "scan";
    const bool force_index = e_.force_filter == "index";
    FilterStep st{FilterStep::SCAN};
    st.col = n.col;
    if ((n.type == FilterNode::SORTED || c.is_sorted) && !force_scan) {
      // SortedInvertedIndexBasedFilterOperator: runs of matching dictIds -> merged [start, end] doc ranges
      std::vector<int32_t> ranges;
      for (int32_t i = 0; i < c.card;) {
        if (!ev.matching[i]) { i++; continue; }
        int32_t j = i;
        while (j + 1 < c.card && ev.matching[j + 1]) j++;
        const int32_t s = c.sorted_start[i], en = c.sorted_end[j];
        if (en >= s) {
          if (!ranges.empty() && ranges.back() + 1 == s) ranges.back() = en;
          else { ranges.push_back(s); ranges.push_back(en); }
        }
        i = j + 1;
      }
      st.kind = FilterStep::RANGES;
      st.n = (int)ranges.size() / 2;
      st.off = ar_.add(ranges.data(), ranges.size() * 4);
      return st;
    }
    if (n.type == FilterNode::BITMAP && !force_scan) {
      // BitmapBasedFilterOperator: OR the bitmaps of the matching dictIds, or of the non-matching ones and flip
      const bool excl = ev.exclusive();
      std::vector<int32_t> ids;
      uint64_t payload = 0;
      for (int32_t i = 0; i < c.card; i++) {
        if ((ev.matching[i] != 0) != excl) {
          ids.push_back(i);
          payload += c.inv_bytes[i];
        }
      }
      // cost model: roaring payload + one bitset write vs. streaming the packed column
      const uint64_t idx_cost = payload + (uint64_t)seg_.num_docs / 8;
      if (force_index || idx_cost < c.fwd_bytes) {
        st.kind = FilterStep::ROARING;
        st.n = (int)ids.size();
        st.negate = excl ? 1 : 0;
        st.off = ar_.add(ids.data(), ids.size() * 4);
        if (st.n > kMaxFusedRoaringIds) key_list(c, ids, st);
        return st;
      }
    }
    if (c.mv) {  // MVScanDocIdIterator: applyMV over each doc's entries (any / every one for exclusive predicates)
      sp_.scan_leaves++;
      std::vector<uint32_t> lut((c.card + 31) / 32 + 1, 0u);
      for (int32_t i = 0; i < c.card; i++)
        if (ev.matching[i]) lut[i >> 5] |= 1u << (i & 31);
      st.kind = FilterStep::MV_SCAN;
      st.negate = ev.exclusive() ? 1 : 0;
      st.off = ar_.add(lut.data(), lut.size() * 4);
      return st;
    }
    scan_leaf(c, ev, st);
    return st;
  }
  // The ids' containers bucketed by roaring key (counting sort over the keys): a chunk's containers are then the
  // key's slice of the list. Skipped (st.keys stays 0) when the list would exceed kMaxFusedRoaringList entries.
  void key_list(const ColumnData &c, const std::vector<int32_t> &ids, FilterStep &st) {
    int64_t total = 0;
    for (int32_t id : ids) total += c.inv_dir[id + 1] - c.inv_dir[id];
    if (total > kMaxFusedRoaringList) return;
    const int keys = (int)(((int64_t)seg_.num_docs + 65535) >> 16);
    std::vector<int32_t> dir(keys + 2, 0), list((size_t)std::max<int64_t>(total, 1));
    for (int32_t id : ids)
      for (int32_t j = c.inv_dir[id]; j < c.inv_dir[id + 1]; j++)
        if (c.inv_keys[j] < keys) dir[c.inv_keys[j] + 2]++;
    for (int k = 0; k < keys; k++) dir[k + 2] += dir[k + 1];
    for (int32_t id : ids)
      for (int32_t j = c.inv_dir[id]; j < c.inv_dir[id + 1]; j++)
        if (c.inv_keys[j] < keys) list[dir[c.inv_keys[j] + 1]++] = j;
    st.keys = keys;
    st.key_off = ar_.add(dir.data(), (size_t)(keys + 1) * 4);
    st.list_off = ar_.add(list.data(), list.size() * 4);
  }
  void scan_leaf(const ColumnData &c, const Evaluator &ev, FilterStep &st) {
    sp_.scan_leaves++;
    auto contiguous = [&](uint8_t want, int32_t &lo, int32_t &hi) {
      int32_t first = -1, last = -1;
      int64_t cnt = 0;
      for (int32_t i = 0; i < c.card; i++)
        if (ev.matching[i] == want) {
          if (first < 0) first = i;
          last = i;
          cnt++;
        }
      if (cnt == 0 || last - first + 1 != cnt) return false;
      lo = first;
      hi = last + 1;
      return true;
    };
    int32_t lo, hi;
    if (contiguous(1, lo, hi) || contiguous(0, lo, hi)) {
      st.leaf_kind = LEAF_RANGE;
      st.negate = ev.matching[lo] ? 0 : 1;
      st.lo = (uint32_t)lo;
      st.span = (uint32_t)(hi - lo);
    } else if (c.card <= 64) {
      st.leaf_kind = LEAF_LUT64;
      for (int32_t i = 0; i < c.card; i++)
        if (ev.matching[i]) st.lut64 |= 1ull << i;
    } else {
      std::vector<uint32_t> lut((c.card + 31) / 32 + 1, 0u);
      for (int32_t i = 0; i < c.card; i++)
        if (ev.matching[i]) lut[i >> 5] |= 1u << (i & 31);
      st.leaf_kind = LEAF_LUT;
      st.off = ar_.add(lut.data(), lut.size() * 4);
    }
  }

  int max_fused_bits_ = 32;
  int max_stack_ = kMaxFusedStack;
  Engine &e_;
  SegPlan &sp_;
  Arena &ar_;
  const SegmentData &seg_;
  int next_slot_ = 1;
};

struct QueryScratch {
  uint8_t *arena = nullptr;     // device copy of the query arena
  uint64_t *bitsets = nullptr;  // regions * slots * stride words
  int64_t stride = 0;
  int slots = 1;                // bitset slots per region
};

struct Timer {
  Engine &e;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> marks;
  size_t used = 0;
  explicit Timer(Engine &en) : e(en) {}
  std::pair<hipEvent_t, hipEvent_t> pair() {
    if (used * 2 + 2 > e.kev.size()) {
      hipEvent_t a, b;
      PINOT_HIP(hipEventCreate(&a));
      PINOT_HIP(hipEventCreate(&b));
      e.kev.push_back(a);
      e.kev.push_back(b);
    }
    auto p = std::make_pair(e.kev[used * 2], e.kev[used * 2 + 1]);
    used++;
    return p;
  }
  template <typename F>
  void timed(int kind, F f) {
    if (!e.timing) { f(); return; }
    auto p = pair();
    PINOT_HIP(hipEventRecord(p.first, e.stream));
    f();
    PINOT_HIP(hipEventRecord(p.second, e.stream));
    marks.push_back({kind, p});
  }
  void collect() {
    e.last_ms[0] = e.last_ms[1] = 0;
    e.last_launches[0] = e.last_launches[1] = 0;
    for (auto &m : marks) {
      float ms = 0;
      PINOT_HIP(hipEventElapsedTime(&ms, m.second.first, m.second.second));
      e.last_ms[m.first] += ms;
      e.last_launches[m.first]++;
    }
  }
};

// The star-tree plan's rewritten query: each function over its pre-aggregated pair column (COUNT sums count__*; AVG
// sums the AvgPair halves, "avg__x.sum" in its own slot and "avg__x.count" in a hidden slot after the query's).
struct StarQuery {
  std::vector<std::string> names;         // per slot: the star docs' column
  std::vector<pinot_agg_spec> specs;      // the query's slots, then the hidden AVG count slots
  std::vector<int> hidden;                // per query aggregation: its count slot (AVG) or -1
  pinot_query q{};                        // the query's slots only (stats, projections)
  pinot_query all{};                      // every slot
};

struct KeySpace {
  std::vector<int64_t> gcard;                          // global cardinality per group column
  std::vector<std::vector<std::vector<int32_t>>> remap;  // [segment][gcol] dictId -> global id (empty = identity)
  std::vector<std::vector<std::string>> gvalues;       // [gcol] global id -> string value
  int64_t G = 1;
  bool hashed = false;  // Π cardinalities > kDenseKeyLimit: keys are hash-table slots (G set by the plan)
};
constexpr int64_t kDenseKeyLimit = int64_t(1) << 27;

struct AdmissionPlan {
  bool active = false;           // some segment's holder or the inter-segment cap can drop keys
  bool cap_active = false;       // the 2 x limit inter-segment cap can bind
  std::vector<int64_t> upper;    // per segment: keys its holder admits (>= G: every present key)
  int64_t cap = 0;
};

struct AdmissionBuffers {
  uint32_t *first_doc = nullptr;  // [S][G]
  uint32_t *bitmaps = nullptr;    // [S][words]
  int64_t words = 0;
  void *scratch = nullptr;
  size_t scratch_bytes = 0;
};

struct GroupAccs {
  std::vector<int> acc_kind;    // per agg
  std::vector<size_t> acc_bytes_per_key;
};

// Fused group-by: ONE k_group_query launch (or COUNT / EMIT / reduce for the partitioned plan) over all
// segments, device compaction of the non-empty keys, device per-group outputs, one D2H of the arrays.
// Multi-GPU partial arrays in the partial layout: `po` = write them (pinot_gpu_group_by_partial, the kernels
// stop before compaction), `pin` = finalize from them (pinot_gpu_group_by_finalize, no kernels: the same
// device compaction / outputs / lazy HLL registers as a one-GPU group-by).
struct PartialOut {
  int64_t *counts;
  void *const *accs;
  bool hll_sum_room = false;         // HLL arrays: u64 [G] after the registers for the ring plan's register sums
  bool *hll_sums_written = nullptr;  // set: the ring plan left them
};

// Dense accumulators of one key range [key_base, key_base + G) -> result (the one-GPU group-by's back half, and the
// owner finalize of a multi-GPU reduce-scatter slice): ordered compaction of the non-empty keys on the device
// (`extra` enqueues further D2H copies ahead of the one sync), per-group outputs incl. the exact HLL register
// sums, one D2H, host fill over the host's cores. HLL registers stay on the device until asked for.
struct DenseGroups {
  const pinot_query *q;
  const KeySpace *ks;
  const GroupAccs *ga, *gx;          // accumulator kinds per aggregation; gx: 5 where alias[i] shares another's
  const std::vector<int> *alias;
  unsigned long long *counts;
  std::vector<void *> accs;
  int64_t key_base;
  const GroupArgs *hashed;           // hashed key spaces: the query's args (slot -> global-id tuples)
  std::vector<const void *> hll_sum;  // per accumulator: the HLL's packed register sums (k_group_final kind 9), or null
};

// ---- functions shared across the executor sources
const uint64_t *run_filter(Engine &e, SegPlan &p, const QueryScratch &qs, Timer &t, int64_t region = 0);
void fill_stats(const pinot_query &q, const std::vector<SegPlan> &plans, const std::vector<int64_t> &counts,
                double ms, pinot_exec_stats *st);
QueryScratch prepare_scratch(Engine &e, const std::vector<SegPlan> &plans, const Arena &ar, bool per_segment,
                             size_t extra = 0);
void wait_stream(Engine &e);
void wait_flag(Engine &e, volatile uint32_t *flag, uint32_t seq);
void upload_arena(Engine &e, const Arena &ar);
std::pair<int64_t, int64_t> chunk_window(const SegPlan &p, const Arena &ar);
FusedStep fused_leaf_step(const SegmentData &s, const FilterStep &l, const uint8_t *arena);
std::vector<SegPlan> plan_all(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q, Arena &ar,
                              std::unique_ptr<FilterTreeInput> &tree);
QueryScratch prepare(Engine &e, std::vector<SegPlan> &plans, Arena &ar);
bool star_plan(const Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q);
void star_query(const pinot_query &q, StarQuery &sq);
void star_stats(const pinot_query &q2, const std::vector<SegmentData *> &segs, const std::vector<StarMatch> &m,
                float ms, pinot_exec_stats *st);
int64_t projected_columns(const pinot_query &q);
double decode_ordered(uint64_t o);
GroupAccs group_acc_kinds(const SegmentData &s, const pinot_query &q);
KeySpace build_key_space(const std::vector<SegmentData *> &segs, const pinot_query &q);
AdmissionPlan plan_admission(const std::vector<SegmentData *> &segs, const pinot_query &q, const Engine &e, int64_t G);
std::unique_ptr<GroupByResult> finalize_groups(Engine &e, const pinot_query &q, const GroupAccs &ga,
                                               const KeySpace &ks, GroupByProgram gp, const MvHash *mh = nullptr);
bool same_dictionary(const ColumnData &a, const ColumnData &b);
unsigned long long compact_dense(Engine &e, const unsigned long long *counts, int64_t G, long long *&keys_dev,
                                 const std::function<void(uint8_t *)> &extra, size_t extra_bytes = 0);
DenseOut dense_outputs(Engine &e, const DenseGroups &d, const long long *keys_dev, unsigned long long n,
                       bool gather_hll = true, bool compact_ok = true, bool serialize_hll = false);
std::unique_ptr<GroupByResult> dense_fetch(Engine &e, const pinot_query &q, const std::vector<int64_t> &gcard,
                                           const std::vector<std::vector<std::string>> &gvalues, const DenseOut &o,
                                           const GroupArgs *hashed);
void apply_inter_segment_cap(std::vector<uint32_t> &bm, size_t S, int64_t words, int64_t cap);
void accumulate_groups(Engine &e, std::vector<SegPlan> &plans, const QueryScratch &qs, const pinot_query &q,
                       const GroupAccs &ga, const KeySpace &ks, unsigned long long *counts, void *const *accs,
                       Timer &t, std::vector<int64_t> &seg_counts, bool apply_limit);
void init_accs(Engine &e, int64_t G, unsigned long long *counts, const GroupAccs &ga, void *const *accs);
int64_t count_docs(Engine &e, const uint64_t *bits, const SegmentData &s);
bool touches_mv_group_by(const std::vector<SegmentData *> &segs, const pinot_query &q);
std::vector<pinot_agg_spec> mv_extended_specs(const pinot_query &q, std::vector<int> &hidden);
void fold_mv_counts(GroupByResult &res, const pinot_query &q, const std::vector<int> &hidden);
const long long *device_trim(Engine &e, const DenseGroups &d, const long long *keys_dev, unsigned long long &n,
                             int32_t top_n, std::vector<std::vector<int64_t>> &kept, int64_t min_groups = -1,
                             std::vector<uint32_t> *flags_out = nullptr);
AdmissionBuffers admission_buffers(Engine &e, size_t S, int64_t G);
void build_admitted(Engine &e, const AdmissionPlan &ap, size_t S, int64_t G, const AdmissionBuffers &ab);
GroupByProgram make_group_program(Engine &e, SegmentData &s, const pinot_query &q, const GroupAccs &ga,
                                  const KeySpace &ks, size_t si, const std::vector<DeviceBuffer> &remaps,
                                  unsigned long long *counts, void *const *accs);
std::unique_ptr<GroupByResult> build_dense_result(Engine &e, const DenseGroups &d, const long long *keys_dev,
                                                  unsigned long long n, bool subset = false);
std::unique_ptr<GroupByResult> exec_group_by_fused(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q,
                                                   const KeySpace &ks_in, const GroupAccs &ga, pinot_exec_stats *stats,
                                                   int attempt = 0, const PartialOut *po = nullptr,
                                                   const PartialOut *pin = nullptr, bool allow_admission = false,
                                                   AdmissionIO *aio = nullptr);
std::unique_ptr<GroupByResult> exec_group_by_mv(Engine &e, const std::vector<SegmentData *> &segs,
                                                const pinot_query &q, pinot_exec_stats *stats,
                                                const MvPartial *mp = nullptr, int attempt = 0);
std::unique_ptr<GroupByResult> exec_group_by_star(Engine &e, const std::vector<SegmentData *> &segs,
                                                  const std::vector<bool> &on_star, const pinot_query &q,
                                                  pinot_exec_stats *stats);
bool is_mv_function(int f);
bool touches_mv_aggregation(const std::vector<SegmentData *> &segs, const pinot_query &q);

std::unique_ptr<GroupByResult> exec_group_by_legacy(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q,
                                                    pinot_exec_stats *stats);
// Runs fn(0..n-1) on the host task pool (at most host_threads() threads; the calling thread takes tasks too).
void parallel_tasks(size_t n, const std::function<void(size_t)> &fn);
size_t host_threads();

}  // namespace pinot
