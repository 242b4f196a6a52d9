// Query execution on one GPU: per-segment filter plans, aggregation, group-by, combine.
//
// Restates, for dictionary-encoded single-value columns (PC = pinot-core/src/main/java/org/apache/pinot/core):
//   FilterPlanNode / FilterOperatorUtils operator choice            PC/plan/FilterPlanNode.java:70-126
//   AggregationOperator.getNextBlock / DefaultAggregationExecutor   PC/operator/query/AggregationOperator.java:56-82
//   Count/Sum/Min/Max/Avg/DistinctCountHLL aggregation functions     PC/query/aggregation/function/
//   AggregationGroupByOperator / DefaultGroupByExecutor               PC/operator/query/AggregationGroupByOperator.java:64-94
//   DictionaryBasedGroupKeyGenerator (raw keys, holder choice, limit) PC/query/aggregation/groupby/DictionaryBasedGroupKeyGenerator.java:79-437
//   CombineOperator / CombineService.mergeTwoBlocks                   PC/operator/CombineOperator.java:75-196
//   CombineGroupByOperator                                            PC/operator/CombineGroupByOperator.java:104-228
//   ExecutionStatistics                                               PC/operator/ExecutionStatistics.java:24-90
//
// A filter tree becomes a sequence of streaming leaf launches that write / AND / OR into doc bitsets in
// HBM (slot 0 holds the final set). All segments of a query are planned on the host first; every small
// per-query table (sorted ranges, roaring id lists, IN/NOT_IN membership bitmaps) goes up in ONE
// host->device copy, the kernels of all segments run back to back on the engine's stream, and the
// reduced per-segment results come back in ONE device->host copy.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <chrono>
#include <cmath>
#include <cstring>
#include <map>
#include <tuple>
#include <numeric>
#include <set>
#include <thread>
#include <functional>

#include "engine.h"
#include "group_ring.h"
#include "mv_hash.h"
#include "trim.h"

namespace pinot {
// fused_group.hip: the k_group_query instance a launch of `a` runs (mode * 10000 + read path * 1000 + threads)
int group_query_instance(const GroupArgs &a);
// hll_serde.hip: HyperLogLog.getBytes of n groups' u8 register rows ([n][256] -> [n][180] B)
void launch_hll_getbytes(const uint8_t *regs, long long n, uint8_t *out, hipStream_t stream);

void check_deadline(const Engine &e, const char *phase) {
  if (e.has_deadline && std::chrono::steady_clock::now() >= e.deadline)
    throw Error(PINOT_ERR_TIMEOUT, std::string("query timed out during ") + phase);
}

DeadlineScope::DeadlineScope(Engine &en, int32_t timeout_ms) : e(en) {
  require(timeout_ms >= 0, PINOT_ERR_TIMEOUT, "query budget already spent before execution (scheduling wait >= timeout)");
  e.has_deadline = timeout_ms > 0;
  if (timeout_ms > 0) e.deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
}

namespace {

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

std::string agg_column(const pinot_agg_spec &a) {
  if (a.column == nullptr) return "*";
  return a.column;
}

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

// Device scratch of a query: arena capacity (arena + `extra` bytes the caller appends once device
// addresses are known) and bitset slots, one region for all segments (run one after the other) or one
// region per segment (fused path: every `pre` bitset must exist when the single kernel runs).
QueryScratch prepare_scratch(Engine &e, const std::vector<SegPlan> &plans, const Arena &ar, bool per_segment,
                             size_t extra = 0) {
  QueryScratch qs;
  int64_t max_words = 1;
  for (auto &p : plans) {
    qs.slots = std::max(qs.slots, p.slots);
    max_words = std::max<int64_t>(max_words, p.seg->nwords());
  }
  e.small.reserve(std::max<size_t>(ar.bytes.size() + extra + 64, 256));
  qs.arena = e.small.get<uint8_t>();
  qs.stride = (max_words + 31) / 32 * 32;  // 256-B aligned slots
  const size_t regions = per_segment ? plans.size() : 1;
  e.bitsets.reserve(regions * (size_t)qs.slots * qs.stride * 8 + 512);  // + a chunk of `pre` words over-read
  qs.bitsets = e.bitsets.get<uint64_t>();
  return qs;
}

// Waits for the engine stream: hipStreamSynchronize, or a busy poll (sync.poll=1) that avoids the
// runtime's sleep/wake-up latency on short queries. Under a query deadline the poll gives up at the deadline
// (PINOT_ERR_TIMEOUT; the queued device work still drains in stream order before the engine's next call).
void wait_stream(Engine &e) {
  if (!e.sync_poll && !e.has_deadline) {
    PINOT_HIP(hipStreamSynchronize(e.stream));
    return;
  }
  hipError_t st;
  while ((st = hipStreamQuery(e.stream)) == hipErrorNotReady) {
    if (e.has_deadline) {
      check_deadline(e, "device execution");
      std::this_thread::yield();
    }
  }
  PINOT_HIP(st);
}

constexpr size_t kCtlClockOff = 64;  // fused_ctl: u32 arrival counter at 0, u64 clock_start here, HLL from 256

// Spins on a completion sequence number the kernel's last block stores (system scope, release) into mapped
// host memory after its results: no wait for the runtime's end-of-kernel signal. Every 1024 spins the stream
// is queried, so a device error, or a kernel that ended without the flag, still surfaces; deadlines hold.
void wait_flag(Engine &e, volatile uint32_t *flag, uint32_t seq) {
  for (uint64_t spins = 1;; spins++) {
    if (*flag == seq) break;
    if ((spins & 1023) == 0) {
      const hipError_t st = hipStreamQuery(e.stream);
      if (st != hipSuccess && st != hipErrorNotReady) PINOT_HIP(st);
      if (st == hipSuccess && *flag != seq) throw Error(PINOT_ERR_DEVICE, "query kernel ended without its completion flag");
      if (e.has_deadline) check_deadline(e, "device execution");
    }
    __builtin_ia32_pause();
  }
  std::atomic_thread_fence(std::memory_order_acquire);
}

// One async H2D copy of the arena through pinned staging. A repeated query (same program bytes at the
// same device address, e.g. a prepared statement re-executed) skips the copy: the device copy is
// only ever written here, so equal bytes mean the device already holds them.
void upload_arena(Engine &e, const Arena &ar) {
  if (ar.bytes.empty()) return;
  if (e.arena_dev_valid && e.arena_dev_gen == e.small.generation() && e.arena_shadow == ar.bytes) return;
  e.host_arena.reserve(ar.bytes.size());
  memcpy(e.host_arena.get(), ar.bytes.data(), ar.bytes.size());
  PINOT_HIP(hipMemcpyAsync(e.small.get(), e.host_arena.get(), ar.bytes.size(), hipMemcpyHostToDevice, e.stream));
  e.arena_shadow = ar.bytes;
  e.arena_dev_gen = e.small.generation();
  e.arena_dev_valid = true;
}

QueryScratch prepare(Engine &e, std::vector<SegPlan> &plans, Arena &ar) {
  QueryScratch qs = prepare_scratch(e, plans, ar, false);
  upload_arena(e, ar);
  return qs;
}

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

// Runs the filter steps of one segment. Returns the final bitset (slot 0), or nullptr for MATCH_ALL.
const uint64_t *run_filter(Engine &e, SegPlan &p, const QueryScratch &qs, Timer &t, int64_t region = 0) {
  if (p.match_all) return nullptr;
  SegmentData &s = *p.seg;
  const int64_t nwords = s.nwords();
  auto slot = [&](int i) { return qs.bitsets + (region * qs.slots + i) * qs.stride; };
  for (const FilterStep &st : p.steps) {
    uint64_t *dst = slot(st.dst);
    switch (st.kind) {
      case FilterStep::SCAN: {
        const ColumnData &c = *s.cols[st.col];
        LeafArgs a{};
        a.fwd = c.fwd.get<uint8_t>();
        a.nwords = nwords;
        a.num_docs = s.num_docs;
        a.negate = st.negate;
        a.lo = st.lo;
        a.span = st.span;
        a.lut64 = st.lut64;
        a.lut = reinterpret_cast<const uint32_t *>(qs.arena + st.off);
        a.mode = st.mode;
        a.dst = dst;
        t.timed(0, [&] { launch_leaf(c.bits, st.leaf_kind, a, e.stream); });
        break;
      }
      case FilterStep::RANGES:
        launch_ranges_to_bitset(reinterpret_cast<const int32_t *>(qs.arena + st.off), st.n, nwords, s.num_docs,
                                st.mode, dst, e.stream);
        break;
      case FilterStep::ROARING: {
        const ColumnData &c = *s.cols[st.col];
        launch_roaring_expand(c.inv_payload.get<uint8_t>(), c.inv_containers.get<RoaringContainer>(),
                              c.inv_dir_dev.get<int32_t>(), reinterpret_cast<const int32_t *>(qs.arena + st.off),
                              st.n, st.negate, nwords, s.num_docs, st.mode, dst, e.stream);
        break;
      }
      case FilterStep::COMBINE:
        launch_bitset_combine(dst, slot(st.src), nwords, s.num_docs, st.mode, 0, e.stream);
        break;
      case FilterStep::MV_SCAN: {
        const ColumnData &c = *s.cols[st.col];
        MvLeafArgs a{};
        a.fwd = c.fwd.get<uint8_t>();
        a.offsets = c.mv_offsets.get<uint32_t>();
        a.bits = c.bits;
        a.all = st.negate;
        a.lut = reinterpret_cast<const uint32_t *>(qs.arena + st.off);
        a.nwords = nwords;
        a.num_docs = s.num_docs;
        a.mode = st.mode;
        a.dst = dst;
        t.timed(0, [&] { launch_mv_leaf(a, e.stream); });
        break;
      }
      case FilterStep::FILL:
        launch_bitset_combine(dst, nullptr, nwords, s.num_docs, st.mode, st.negate, e.stream);
        break;
      case FilterStep::FUSED_OP:  // only in fused programs, never in a launch sequence
        throw Error(PINOT_ERR_DEVICE, "fused program step in a filter launch sequence");
    }
    PINOT_HIP(hipGetLastError());
  }
  return slot(0);
}

std::vector<SegPlan> plan_all(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q, Arena &ar,
                              std::unique_ptr<FilterTreeInput> &tree) {
  if (q.num_filter_nodes > 0) tree = std::make_unique<FilterTreeInput>(decode_filter(q.num_filter_nodes, q.filter));
  std::vector<SegPlan> plans(segs.size());
  for (size_t i = 0; i < segs.size(); i++) {
    plans[i].seg = segs[i];
    Compiler(e, plans[i], ar).run(tree.get());
  }
  return plans;
}

int64_t projected_columns(const pinot_query &q) {
  // TransformPlanNode: distinct columns of the aggregation and group-by expressions (COUNT(*) projects none)
  std::set<std::string> cols;
  for (int i = 0; i < q.num_aggregations; i++) {
    std::string c = agg_column(q.aggregations[i]);
    if (c != "*") cols.insert(c);
  }
  for (int i = 0; i < q.num_group_by; i++) cols.insert(q.group_by[i]);
  return (int64_t)cols.size();
}

void fill_stats(const pinot_query &q, const std::vector<SegPlan> &plans, const std::vector<int64_t> &counts,
                double ms, pinot_exec_stats *st) {
  if (!st) return;
  memset(st, 0, sizeof(*st));
  for (size_t i = 0; i < plans.size(); i++) {
    st->num_docs_scanned += counts[i];
    st->num_total_raw_docs += plans[i].seg->num_docs;
    st->num_entries_scanned_in_filter += plans[i].scan_leaves * plans[i].seg->num_docs;
  }
  st->num_entries_scanned_post_filter = st->num_docs_scanned * projected_columns(q);
  st->num_segments_processed = (int64_t)plans.size();
  for (size_t i = 0; i < plans.size(); i++) st->num_segments_matched += counts[i] > 0;
  st->device_ms = ms;
}

}  // namespace

// ------------------------------------------------------------------ filter API
void exec_filter(Engine &e, SegmentData &s, const FilterTreeInput *tree, uint64_t *bitset_out, int64_t *count) {
  Arena ar;
  std::vector<SegPlan> plans(1);
  plans[0].seg = &s;
  Compiler(e, plans[0], ar).run(tree);
  QueryScratch qs = prepare(e, plans, ar);
  const int64_t nwords = s.nwords();
  Timer t(e);
  if (plans[0].empty || plans[0].match_all) {
    if (bitset_out) {
      for (int64_t w = 0; w < nwords; w++) {
        uint64_t v = plans[0].empty ? 0 : ~0ull;
        if (w == nwords - 1 && (s.num_docs & 63)) v &= (1ull << (s.num_docs & 63)) - 1;
        bitset_out[w] = v;
      }
    }
    if (count) *count = plans[0].empty ? 0 : s.num_docs;
    wait_stream(e);
    return;
  }
  const int grid = scan_grid(nwords);
  e.partials.reserve((size_t)grid * 8);
  e.reduced.reserve(64);
  const uint64_t *bits = run_filter(e, plans[0], qs, t);
  launch_popcount(bits, nwords, s.num_docs, e.partials.get<unsigned long long>(), e.stream);
  ReduceArgs ra{};
  ra.in = e.partials.get<unsigned long long>();
  ra.stride = grid;
  ra.grid = grid;
  ra.out = e.reduced.get<unsigned long long>();
  launch_reduce_slots(ra, 1, e.stream);
  unsigned long long hc = 0;
  PINOT_HIP(hipMemcpyAsync(&hc, ra.out, 8, hipMemcpyDeviceToHost, e.stream));
  if (bitset_out && nwords)
    PINOT_HIP(hipMemcpyAsync(bitset_out, bits, nwords * 8, hipMemcpyDeviceToHost, e.stream));
  wait_stream(e);
  t.collect();
  if (count) *count = (int64_t)hc;
}

// ------------------------------------------------------------------ aggregation-only
namespace {

// How one aggregation function is computed on one segment.
struct AggRoute {
  enum Kind { COUNT_ONLY, IDSUM, MINMAX, GATHER, HLL } kind;
  int col = -1;
  int gather_kind = GA_SUM_I32;
};

AggRoute route_agg(Engine &e, SegmentData &s, const pinot_agg_spec &spec) {
  AggRoute r{AggRoute::COUNT_ONLY};
  const int f = spec.function;
  if (f == PINOT_AGG_COUNT) return r;
  ColumnData &c = *s.column(agg_column(spec));
  r.col = s.by_name[c.name];
  if (f == PINOT_AGG_DISTINCTCOUNTHLL) {
    ensure_hll_lut(e, c);
    r.kind = AggRoute::HLL;
    return r;
  }
  require(c.numeric(), PINOT_ERR_UNSUPPORTED, "numeric aggregation over STRING column " + c.name);
  if (f == PINOT_AGG_MIN || f == PINOT_AGG_MAX) {
    r.kind = AggRoute::MINMAX;  // sorted dictionary: min/max value = value of the min/max dictId
  } else if (c.affine && e.use_affine) {
    r.kind = AggRoute::IDSUM;   // Σ value = base * count + step * Σ dictId
  } else {
    r.kind = AggRoute::GATHER;
    r.gather_kind = c.data_type == PINOT_INT ? GA_SUM_I32 : c.data_type == PINOT_LONG ? GA_SUM_I64 : GA_SUM_F64;
  }
  return r;
}

}  // namespace

namespace {

// Chunk window of a segment's fused program: a top-level term that is a single sorted-index leaf bounds
// the candidate docs to [first range start, last range end] (SortedInvertedIndexBasedFilterOperator's
// docId ranges), so the kernels only visit the 4096-doc chunks inside it.
std::pair<int64_t, int64_t> chunk_window(const SegPlan &p, const Arena &ar) {
  const int64_t nchunks = (p.seg->nwords() + 63) / 64;
  int64_t lo = 0, hi = nchunks;
  const auto &L = p.fused_leaves;
  for (size_t i = 0; i < L.size(); i++) {
    const bool single = L[i].join == JOIN_NEW && (i + 1 == L.size() || L[i + 1].join == JOIN_NEW);
    if (!single || L[i].kind != FilterStep::RANGES) continue;
    if (L[i].n == 0) return {0, 0};
    const int32_t *r = reinterpret_cast<const int32_t *>(ar.bytes.data() + L[i].off);
    lo = std::max<int64_t>(lo, (int64_t)r[0] / 4096);
    hi = std::min<int64_t>(hi, (int64_t)r[2 * (L[i].n - 1) + 1] / 4096 + 1);
  }
  return {lo, std::max(lo, hi)};
}

// A fused leaf (FilterStep) as the device step k_scan_query / k_group_query evaluate.
FusedStep fused_leaf_step(const SegmentData &s, const FilterStep &l, const uint8_t *arena) {
  FusedStep st{};
  st.join = l.join;
  st.negate = l.negate;
  if (l.kind == FilterStep::FUSED_OP) {  // no column: the close of a nested term
    st.kind = FK_OP;
    return st;
  }
  const ColumnData &c = *s.cols[l.col];
  switch (l.kind) {
    case FilterStep::RANGES:
      st.kind = FK_LEAF_RANGES;
      st.table = arena + l.off;
      st.lo = (uint32_t)l.n;
      break;
    case FilterStep::ROARING:
      st.kind = FK_LEAF_ROARING;
      st.fwd = c.inv_payload.get<uint8_t>();
      st.aux0 = c.inv_containers.get();
      st.aux1 = c.inv_dir_dev.get();
      st.table = arena + l.off;
      st.lo = (uint32_t)l.n;
      if (l.n > kMaxFusedRoaringIds) {  // the per-key container list (key_list)
        st.ops = 1;
        st.aux1 = arena + l.key_off;
        st.table = arena + l.list_off;
        st.lo = (uint32_t)l.keys;
      }
      break;
    default:
      st.fwd = c.fwd.get<uint8_t>();
      st.bits = c.bits;
      st.kind = l.leaf_kind == LEAF_RANGE ? FK_LEAF_RANGE : l.leaf_kind == LEAF_LUT64 ? FK_LEAF_LUT64 : FK_LEAF_LUT;
      st.lo = l.lo;
      st.span = l.span;
      st.lut64 = l.lut64;
      st.table = arena + l.off;
      break;
  }
  return st;
}

// Where the device left aggregation a of segment si: index into the reduced u64 results, and for
// DISTINCTCOUNTHLL the register set (256 u32) holding its merged registers.
struct AggResults {
  const unsigned long long *res = nullptr;  // [S][nres]
  const uint32_t *hll = nullptr;            // [sets][256]
  int nres = 0;
  std::vector<std::vector<int>> src;        // [si][a] -> slot within the segment's nres
  std::vector<int> hll_set;                 // [a]
};

// CombineService.mergeTwoBlocks over segments (in segment order), per function.
void merge_aggregates(const pinot_query &q, const std::vector<SegPlan> &plans,
                      const std::vector<std::vector<AggRoute>> &routes, const std::vector<int64_t> &counts,
                      const AggResults &R, pinot_agg_result *out) {
  const size_t S = plans.size();
  int64_t total = 0;
  for (auto c : counts) total += c;
  for (int a = 0; a < q.num_aggregations; a++) {
    pinot_agg_result &r = out[a];
    memset(&r, 0, sizeof(r));
    const int f = q.aggregations[a].function;
    r.count = total;
    auto raw_of = [&](size_t si) { return R.res[si * R.nres + R.src[si][a]]; };
    switch (f) {
      case PINOT_AGG_COUNT:
        break;
      case PINOT_AGG_SUM:
      case PINOT_AGG_AVG: {
        bool exact = true;
        __int128 isum = 0;
        double dsum = 0.0;
        for (size_t si = 0; si < S; si++) {
          if (plans[si].empty || counts[si] == 0) continue;
          const AggRoute &rt = routes[si][a];
          const ColumnData &c = *plans[si].seg->cols[rt.col];
          const unsigned long long raw = raw_of(si);
          if (rt.kind == AggRoute::IDSUM) {
            isum += (__int128)c.affine_base * counts[si] + (__int128)c.affine_step * (__int128)raw;
          } else if (rt.gather_kind == GA_SUM_I32) {
            isum += (__int128)(long long)raw;
          } else {
            double d;
            memcpy(&d, &raw, 8);
            dsum += d;
            exact = false;
          }
        }
        if (exact) {
          r.value = (double)isum;
          if (isum >= INT64_MIN && isum <= INT64_MAX) {
            r.exact_sum = (int64_t)isum;
            r.has_exact_sum = 1;
          }
        } else {
          r.value = dsum + (double)isum;
        }
        break;
      }
      case PINOT_AGG_MIN:
      case PINOT_AGG_MAX: {
        const bool is_min = f == PINOT_AGG_MIN;
        double v = is_min ? INFINITY : -INFINITY;  // Min/MaxAggregationFunction.DEFAULT_VALUE
        for (size_t si = 0; si < S; si++) {
          if (plans[si].empty || counts[si] == 0) continue;
          const ColumnData &c = *plans[si].seg->cols[routes[si][a].col];
          const unsigned long long raw = raw_of(si);
          const uint32_t id = is_min ? (uint32_t)raw : (uint32_t)(raw >> 32);
          if (id >= (uint32_t)c.card) continue;
          const double x = c.double_value((int32_t)id);
          v = is_min ? std::min(v, x) : std::max(v, x);
        }
        r.value = v;
        break;
      }
      case PINOT_AGG_DISTINCTCOUNTHLL: {
        const uint32_t *regs = R.hll + (size_t)R.hll_set[a] * 256;
        for (int j = 0; j < 256; j++) r.hll_registers[j] = (uint8_t)regs[j];
        r.hll_cardinality = hll_cardinality(r.hll_registers);
        break;
      }
    }
  }
}

// The query shape k_scan_query evaluates in one launch: every aggregation a fold over a dictId stream
// (COUNT, Σ dictId of an arithmetic-progression dictionary, Σ int32 dictionary values, min/max dictId,
// HLL registers via the per-dictId LUT), at most kMaxFusedFolds distinct columns and kMaxHll HLL columns.
bool fusable(const pinot_query &q, const std::vector<std::vector<AggRoute>> &routes, std::vector<std::string> &fold_cols,
             std::vector<std::string> &hll_cols) {
  for (const auto &per_seg : routes)
    for (const AggRoute &r : per_seg)
      if (r.kind == AggRoute::GATHER && r.gather_kind != GA_SUM_I32) return false;
  for (int a = 0; a < q.num_aggregations; a++) {
    if (q.aggregations[a].function == PINOT_AGG_COUNT) continue;
    const std::string c = agg_column(q.aggregations[a]);
    if (std::find(fold_cols.begin(), fold_cols.end(), c) == fold_cols.end()) fold_cols.push_back(c);
    if (q.aggregations[a].function == PINOT_AGG_DISTINCTCOUNTHLL &&
        std::find(hll_cols.begin(), hll_cols.end(), c) == hll_cols.end())
      hll_cols.push_back(c);
  }
  return (int)fold_cols.size() <= kMaxFusedFolds && (int)hll_cols.size() <= kMaxHll;
}

int index_of_name(const std::vector<std::string> &v, const std::string &x) {
  return (int)(std::find(v.begin(), v.end(), x) - v.begin());
}

// Fused path: pre bitsets (index leaves / OR subtrees) per segment, then ONE k_scan_query over all
// segments and ONE fixed-order reduction, ONE device->host copy.
// The host plan of a fused aggregation (filter compile per segment, the device program in the arena, grid and
// LDS shape). A repeated query over the same segments (a prepared statement re-executed) reuses it: only the
// per-segment `pre` bitsets, the launch and the merge run again.
struct FusedPlan {
  std::string key;                  // query shape + segment uids + engine config epoch
  uint64_t small_gen = 0, bitsets_gen = 0;
  std::vector<SegPlan> plans;
  std::vector<std::vector<AggRoute>> routes;
  std::vector<std::string> fold_cols, hll_cols;
  Arena ar;
  QueryScratch qs;
  FusedArgs fa{};                   // launch-invariant fields
  bool gathers = false, pipelined = false;
  int nres = 0;
  size_t off_hll = 0, off_tail = 0, red_bytes = 0, ctl_acc = 0, res_bytes = 0;
};

// Identity of a fused query: the query text as marshalled (filter nodes, aggregations), the segments' uids and
// the engine's configuration epoch.
std::string fused_plan_key(const Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q) {
  std::string k;
  auto put_i = [&k](int64_t v) { k.append(reinterpret_cast<const char *>(&v), sizeof(v)); };
  auto put_s = [&k, &put_i](const char *s) {
    const size_t n = s ? strlen(s) : 0;
    put_i(s ? (int64_t)n : -1);
    if (n) k.append(s, n);
  };
  put_i(e.config_epoch);
  put_i(q.num_filter_nodes);
  for (int i = 0; i < q.num_filter_nodes; i++) {
    const pinot_filter_node &nd = q.filter[i];
    put_i(nd.op);
    put_i(nd.num_children);
    put_s(nd.column);
    put_i(nd.num_values);
    for (int v = 0; v < nd.num_values; v++) put_s(nd.values ? nd.values[v] : nullptr);
  }
  put_i(q.num_aggregations);
  for (int i = 0; i < q.num_aggregations; i++) {
    put_i(q.aggregations[i].function);
    put_s(q.aggregations[i].column);
  }
  put_i((int64_t)segs.size());
  for (SegmentData *sg : segs) put_i((int64_t)sg->uid);
  return k;
}

void plan_fused(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q, FusedPlan &fp) {
  const int na = q.num_aggregations;
  const size_t S = segs.size();
  std::vector<std::vector<AggRoute>> &routes = fp.routes;
  const std::vector<std::string> &fold_cols = fp.fold_cols, &hll_cols = fp.hll_cols;
  Arena &ar = fp.ar;
  std::unique_ptr<FilterTreeInput> tree;
  if (q.num_filter_nodes > 0) tree = std::make_unique<FilterTreeInput>(decode_filter(q.num_filter_nodes, q.filter));
  std::vector<SegPlan> &plans = fp.plans;
  plans.assign(S, SegPlan{});
  for (size_t si = 0; si < S; si++) {
    plans[si].seg = segs[si];
    Compiler(e, plans[si], ar).run_fused(tree.get());
  }
  e.last_pre_segments = 0;
  for (auto &p : plans) e.last_pre_segments += p.has_pre && !p.empty;
  const int nfolds = (int)fold_cols.size();
  const int nslots = 1 + 2 * nfolds;
  // steps: per segment its leaves then its folds
  int max_bits = 1;
  size_t nsteps = 0;
  for (auto &p : plans) {
    nsteps += p.fused_leaves.size() + nfolds;
    for (auto &l : p.fused_leaves)
      if (l.kind == FilterStep::SCAN) max_bits = std::max(max_bits, p.seg->cols[l.col]->bits);
    for (auto &c : fold_cols) max_bits = std::max(max_bits, p.seg->column(c)->bits);
  }
  const size_t tab_bytes = S * sizeof(FusedSegment) + nsteps * sizeof(FusedStep) + 256;  // + alignment/padding of two adds
  fp.qs = prepare_scratch(e, plans, ar, true, tab_bytes);
  QueryScratch &qs = fp.qs;
  std::vector<FusedSegment> fsegs(S);
  std::vector<FusedStep> fsteps;
  fsteps.reserve(nsteps);
  for (size_t si = 0; si < S; si++) {
    SegPlan &p = plans[si];
    SegmentData &s = *p.seg;
    FusedSegment &fs = fsegs[si];
    fs.pre = p.has_pre ? qs.bitsets + (int64_t)si * qs.slots * qs.stride : nullptr;
    fs.nwords = p.empty ? 0 : s.nwords();
    fs.num_docs = s.num_docs;
    fs.first_step = (int32_t)fsteps.size();
    fs.n_leaves = (int32_t)p.fused_leaves.size();
    fs.n_folds = nfolds;
    std::tie(fs.ch_begin, fs.ch_end) = chunk_window(p, ar);
    for (const FilterStep &l : p.fused_leaves) fsteps.push_back(fused_leaf_step(s, l, qs.arena));
    for (int f = 0; f < nfolds; f++) {
      ColumnData &c = *s.column(fold_cols[f]);
      FusedStep st{};
      st.fwd = c.fwd.get<uint8_t>();
      st.bits = c.bits;
      st.kind = FK_FOLD;
      st.fold = f;
      for (int a = 0; a < na; a++) {
        if (q.aggregations[a].function == PINOT_AGG_COUNT || agg_column(q.aggregations[a]) != fold_cols[f]) continue;
        const AggRoute &r = routes[si][a];
        if (r.kind == AggRoute::IDSUM) st.ops |= FOLD_IDSUM;
        else if (r.kind == AggRoute::MINMAX) st.ops |= FOLD_MINMAX;
        else if (r.kind == AggRoute::GATHER) { st.ops |= FOLD_DICT32; st.table = c.dict_dev.get(); }
        else if (r.kind == AggRoute::HLL) {
          st.ops |= FOLD_HLL;
          st.hll_lut = c.hll_lut.get<uint16_t>();
          st.hll_set = index_of_name(hll_cols, fold_cols[f]);
        }
      }
      fsteps.push_back(st);
    }
  }
  // pipelined shape: every step of a chunk gets its own 1-KiB-piece region of the wave's LDS slot
  int slot_bytes = 0;
  for (size_t si = 0; si < S; si++) {
    int off = kPipePreBytes;
    for (int i = 0; i < fsegs[si].n_leaves + fsegs[si].n_folds; i++) {
      FusedStep &st = fsteps[fsegs[si].first_step + i];
      st.stage_off = off;
      off += staged_chunk_bytes(st.bits);
    }
    slot_bytes = std::max(slot_bytes, off);
  }
  fp.pipelined = e.use_pipe && slot_bytes <= kMaxPipeSlotBytes;
  const size_t off_segs = ar.add(fsegs.data(), fsegs.size() * sizeof(FusedSegment));
  const size_t off_steps = ar.add(fsteps.data(), fsteps.size() * sizeof(FusedStep));  // may be empty (COUNT(*))
  require(ar.bytes.size() <= e.small.size(), PINOT_ERR_DEVICE, "query arena overflow");

  // grid: one resident wave of blocks, split evenly over the segments (equal work per block)
  const int stage_bytes = fp.pipelined ? slot_bytes : staged_chunk_bytes(max_bits);
  int64_t max_chunks = 1;  // chunks in the largest segment window
  for (const FusedSegment &fs : fsegs) max_chunks = std::max<int64_t>(max_chunks, fs.ch_end - fs.ch_begin);
  bool gathers = false;
  for (const FusedStep &st : fsteps)
    gathers = gathers || st.kind == FK_LEAF_LUT || st.kind == FK_LEAF_RANGES || st.kind == FK_LEAF_ROARING ||
              (st.kind == FK_FOLD && (st.ops & (FOLD_DICT32 | FOLD_HLL)));
  fp.gathers = gathers;
  const int64_t resident = (int64_t)scan_query_blocks_per_cu(stage_bytes, gathers, fp.pipelined) * e.num_cus;
  int bps = (int)std::max<int64_t>(1, resident / (int64_t)S);
  bps = (int)std::min<int64_t>(bps, (max_chunks + 3) / 4);
  fp.nres = kMaxFusedSlots;
  fp.res_bytes = S * fp.nres * 8;
  fp.off_hll = (fp.res_bytes + 255) / 256 * 256;
  fp.off_tail = fp.off_hll + (size_t)kMaxHll * 256 * 4;  // {u32 seq, u32, u64 elapsed ticks}
  fp.red_bytes = fp.off_tail + 16;
  // arrival counter | HLL registers | per-segment accumulators: set to their identities once, the
  // kernel's last block restores them after every launch
  fp.ctl_acc = 256 + (size_t)kMaxHll * 256 * 4;
  FusedArgs &fa = fp.fa;
  fa = FusedArgs{};
  fa.segs = reinterpret_cast<const FusedSegment *>(qs.arena + off_segs);
  fa.steps = reinterpret_cast<const FusedStep *>(qs.arena + off_steps);
  fa.nsegs = (int32_t)S;
  fa.bps = bps;
  fa.nslots = nslots;
  fa.stage_bytes = stage_bytes;
  fa.n_hll = (int32_t)hll_cols.size();
  fa.nt = e.use_nt ? 1 : 0;
  fa.res_stride = fp.nres;
  fa.result_hll_off = (int64_t)fp.off_hll;
  fa.result_tail_off = (int64_t)fp.off_tail;
  fp.small_gen = e.small.generation();
  fp.bitsets_gen = e.bitsets.generation();
}

void run_fused(Engine &e, FusedPlan &fp, const pinot_query &q, pinot_agg_result *out, pinot_exec_stats *stats,
               std::chrono::steady_clock::time_point tq0) {
  const int na = q.num_aggregations;
  const size_t S = fp.plans.size();
  std::vector<SegPlan> &plans = fp.plans;
  e.fused_result.reserve(fp.red_bytes);
  if (e.fused_ctl.size() < fp.ctl_acc + fp.res_bytes) {
    const size_t nseg_cap = std::max<size_t>(S, 64);
    e.fused_ctl.alloc(fp.ctl_acc + nseg_cap * fp.nres * 8);
    std::vector<uint8_t> init(e.fused_ctl.size(), 0);
    memset(init.data() + kCtlClockOff, 0xFF, 8);  // clock_start: ~0 between launches
    auto *acc0 = reinterpret_cast<unsigned long long *>(init.data() + fp.ctl_acc);
    for (size_t i = 0; i < nseg_cap * fp.nres; i++) {
      const int sl = (int)(i % fp.nres);
      acc0[i] = (sl == 0 || (sl & 1)) ? 0ull : 0x00000000FFFFFFFFull;
    }
    PINOT_HIP(hipMemcpy(e.fused_ctl.get(), init.data(), init.size(), hipMemcpyHostToDevice));
  }

  const auto tp0 = std::chrono::steady_clock::now();
  check_deadline(e, "planning");
  // completion: spin on the flag the last block writes into mapped memory (sync.flag=1, not under timing=1,
  // whose HIP events need the runtime's completion), else the stream wait
  const bool flag = e.sync_flag && !e.timing;
  if (!flag) PINOT_HIP(hipEventRecord(e.ev_start, e.stream));
  upload_arena(e, fp.ar);
  Timer t(e);
  for (size_t si = 0; si < S; si++)
    if (plans[si].has_pre && !plans[si].empty) run_filter(e, plans[si], fp.qs, t, (int64_t)si);
  FusedArgs fa = fp.fa;
  fa.acc = reinterpret_cast<unsigned long long *>(e.fused_ctl.get<uint8_t>() + fp.ctl_acc);
  fa.hll_out = reinterpret_cast<uint32_t *>(e.fused_ctl.get<uint8_t>() + 256);
  fa.done = e.fused_ctl.get<uint32_t>();
  fa.result = e.fused_result.device<unsigned long long>();
  fa.clock_start = reinterpret_cast<unsigned long long *>(e.fused_ctl.get<uint8_t>() + kCtlClockOff);
  volatile uint32_t *seq_flag = reinterpret_cast<volatile uint32_t *>(e.fused_result.host<uint8_t>() + fp.off_tail);
  if (flag) {
    if (++e.fused_seq == 0) e.fused_seq = 1;
    fa.seq = e.fused_seq;
  }
  const auto tp1 = std::chrono::steady_clock::now();
  t.timed(0, [&] { launch_scan_query(fa, fp.gathers, fp.pipelined, e.stream); });
  PINOT_HIP(hipGetLastError());
  if (!flag) PINOT_HIP(hipEventRecord(e.ev_stop, e.stream));
  const auto tp2 = std::chrono::steady_clock::now();
  if (flag) wait_flag(e, seq_flag, fa.seq);
  else wait_stream(e);
  if (e.host_phases) {
    const auto tp3 = std::chrono::steady_clock::now();
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    fprintf(stderr, "[pinot_gpu] fused query host phases (us): plan %.1f, pre-launch %.1f, launch %.1f, sync %.1f\n",
            us(tq0, tp0), us(tp0, tp1), us(tp1, tp2), us(tp2, tp3));
  }
  const uint8_t *host = e.fused_result.host<uint8_t>();
  float ms = 0;
  if (flag) ms = (float)((double)reinterpret_cast<const volatile unsigned long long *>(host + fp.off_tail)[1] /
                         (double)e.wall_clock_khz);
  else PINOT_HIP(hipEventElapsedTime(&ms, e.ev_start, e.ev_stop));
  t.collect();

  AggResults R;
  R.res = reinterpret_cast<const unsigned long long *>(host);
  R.hll = reinterpret_cast<const uint32_t *>(host + fp.off_hll);
  R.nres = fp.nres;
  R.src.assign(S, std::vector<int>(na, 0));
  R.hll_set.assign(na, 0);
  std::vector<int64_t> counts(S, 0);
  for (size_t si = 0; si < S; si++) {
    counts[si] = plans[si].empty ? 0 : (int64_t)R.res[si * fp.nres];
    for (int a = 0; a < na; a++) {
      if (q.aggregations[a].function == PINOT_AGG_COUNT) continue;
      const int f = index_of_name(fp.fold_cols, agg_column(q.aggregations[a]));
      R.src[si][a] = fp.routes[si][a].kind == AggRoute::MINMAX ? 2 + 2 * f : 1 + 2 * f;
    }
  }
  for (int a = 0; a < na; a++)
    if (q.aggregations[a].function == PINOT_AGG_DISTINCTCOUNTHLL)
      R.hll_set[a] = index_of_name(fp.hll_cols, agg_column(q.aggregations[a]));
  merge_aggregates(q, plans, fp.routes, counts, R, out);
  fill_stats(q, plans, counts, ms, stats);
  if (e.host_phases)
    fprintf(stderr, "[pinot_gpu] fused query host phases (us): after sync %.1f\n",
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tp2).count());
}

}  // namespace

namespace {

// InstancePlanMakerImplV2.makeInnerSegmentPlan (PC/plan/maker/InstancePlanMakerImplV2.java:96-110,148-211): with no
// filter (and no group-by), all-COUNT queries take the metadata plan (MetadataBasedAggregationOperator: the
// segment's total docs) and all-MIN/MAX queries over dictionary columns the dictionary plan
// (DictionaryBasedAggregationOperator: dictionary value 0 / length - 1; immutable dictionaries are sorted). Both
// report numDocsScanned = totalRawDocs and no entries scanned (MetadataBasedAggregationOperator.java:74-77,
// DictionaryBasedAggregationOperator.java:99-102). Nothing runs on the device.
bool shortcut_aggregate(const std::vector<SegmentData *> &segs, const pinot_query &q, pinot_agg_result *out,
                        pinot_exec_stats *stats) {
  if (q.num_filter_nodes != 0 || q.num_group_by != 0) return false;
  bool all_count = true, all_minmax = true;
  std::vector<std::vector<const ColumnData *>> cols(q.num_aggregations);
  for (int a = 0; a < q.num_aggregations; a++) {
    const int f = q.aggregations[a].function;
    all_count = all_count && f == PINOT_AGG_COUNT;
    const bool mm = f == PINOT_AGG_MIN || f == PINOT_AGG_MAX;
    all_minmax = all_minmax && mm;
    if (!mm) continue;
    const std::string c = agg_column(q.aggregations[a]);
    for (SegmentData *sg : segs) {
      auto it = sg->by_name.find(c);
      const ColumnData *cd = it == sg->by_name.end() ? nullptr : sg->cols[it->second].get();
      // unknown / STRING columns: the regular plan reports it; raw columns have no dictionary to read the ends from
      // (InstancePlanMakerImplV2.isFitForDictionaryBasedPlan)
      if (!cd || !cd->numeric() || cd->raw) all_minmax = false;
      cols[a].push_back(cd);
    }
  }
  if (!all_count && !all_minmax) return false;
  int64_t total = 0;
  for (SegmentData *sg : segs) total += sg->num_docs;
  for (int a = 0; a < q.num_aggregations; a++) {
    pinot_agg_result &r = out[a];
    memset(&r, 0, sizeof(r));
    r.count = total;
    const int f = q.aggregations[a].function;
    if (f == PINOT_AGG_MIN || f == PINOT_AGG_MAX) {
      const bool is_min = f == PINOT_AGG_MIN;
      double v = is_min ? INFINITY : -INFINITY;
      for (const ColumnData *cd : cols[a]) {
        if (cd->card < 1 || cd->num_docs == 0) continue;
        const double x = cd->double_value(is_min ? 0 : cd->card - 1);
        v = is_min ? java_min(v, x) : java_max(v, x);
      }
      r.value = v;
    }
  }
  if (stats) {
    memset(stats, 0, sizeof(*stats));
    stats->num_docs_scanned = total;
    stats->num_total_raw_docs = total;
    stats->num_segments_processed = (int64_t)segs.size();
    for (auto *sg : segs) stats->num_segments_matched += sg->num_docs > 0;
  }
  return true;
}

}  // namespace

namespace {

bool is_mv_function(int f) { return f >= PINOT_AGG_COUNTMV && f <= PINOT_AGG_DISTINCTCOUNTHLLMV; }

// Does the query aggregate over a multi-value column (or with an MV function)? AggregationFunctionFactory pairs MV
// functions with MV columns; a single-value function over an MV column reads it as single-valued and fails.
bool touches_mv_aggregation(const std::vector<SegmentData *> &segs, const pinot_query &q) {
  bool mv = false;
  for (int a = 0; a < q.num_aggregations; a++) {
    const int f = q.aggregations[a].function;
    const std::string col = agg_column(q.aggregations[a]);
    bool col_mv = false;
    for (SegmentData *sg : segs) {
      auto it = sg->by_name.find(col);
      col_mv = col_mv || (it != sg->by_name.end() && sg->cols[it->second]->mv);
    }
    if (is_mv_function(f)) {
      require(col_mv || col == "*", PINOT_ERR_BAD_QUERY, "multi-value aggregation over single-value column " + col);
      mv = true;
    } else if (col_mv && f != PINOT_AGG_COUNT) {
      throw Error(PINOT_ERR_BAD_QUERY, "single-value aggregation over multi-value column " + col);
    }
  }
  return mv;
}

// Aggregation-only query with multi-value functions (CountMV / SumMV / MinMV / MaxMV / AvgMV / DistinctCountHLLMV,
// PC/query/aggregation/function/*MVAggregationFunction.java: aggregate() folds every entry of every matching doc),
// beside any single-value functions of the same query: per segment the filter's dense bitset (the launch sequence,
// MV scan leaves included) and ONE k_mv_aggregate over its docs; the segments' partials merged in segment order on
// the host (CombineService.mergeTwoBlocks).
void exec_aggregate_mv(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q, pinot_agg_result *out,
                       pinot_exec_stats *stats) {
  const int na = q.num_aggregations;
  const size_t S = segs.size();
  Arena ar;
  std::unique_ptr<FilterTreeInput> tree;
  std::vector<SegPlan> plans = plan_all(e, segs, q, ar, tree);
  QueryScratch qs = prepare(e, plans, ar);
  constexpr size_t kOut = 5 * kMaxAggs * 8, kHll = kMaxAggs * 256 * 4;
  e.fused_result.reserve(kOut + kHll + 64);
  uint8_t *dev = e.fused_result.device<uint8_t>();
  const uint8_t *host = e.fused_result.host<uint8_t>();
  std::vector<unsigned long long> init(5 * kMaxAggs, 0ull);
  for (int g = 0; g < kMaxAggs; g++) init[5 * g + 3] = ~0ull;
  PINOT_HIP(hipEventRecord(e.ev_start, e.stream));
  PINOT_HIP(hipMemsetAsync(dev + kOut, 0, kHll, e.stream));  // HyperLogLog registers: max over every segment
  upload_arena(e, ar);
  Timer t(e);
  struct Part {
    int64_t docs = 0;
    std::vector<unsigned long long> v;
    std::vector<uint32_t> hll;
  };
  std::vector<Part> parts(S);
  for (size_t si = 0; si < S; si++) {
    SegPlan &p = plans[si];
    SegmentData &sg = *p.seg;
    if (p.empty || sg.num_docs == 0) continue;
    const uint64_t *bits = run_filter(e, p, qs, t);
    MvAggArgs a{};
    a.bitset = bits;
    a.nwords = sg.nwords();
    a.num_docs = sg.num_docs;
    a.n = na;
    for (int g = 0; g < na; g++) {
      const int f = q.aggregations[g].function;
      MvAggSpec &sp = a.specs[g];
      if (f == PINOT_AGG_COUNT) {
        sp.kind = MVA_COUNT_DOCS;
        continue;
      }
      ColumnData &c = *sg.column(agg_column(q.aggregations[g]));
      sp.fwd = c.fwd.get<uint8_t>();
      sp.offsets = c.mv ? c.mv_offsets.get<uint32_t>() : nullptr;
      sp.dict = c.dict_dev.get();
      sp.bits = c.bits;
      sp.value_kind = c.value_kind();
      sp.numeric = c.numeric() ? 1 : 0;
      sp.kind = MVA_VALUES;
      if (f == PINOT_AGG_DISTINCTCOUNTHLL || f == PINOT_AGG_DISTINCTCOUNTHLLMV) {
        ensure_hll_lut(e, c);
        sp.hll_lut = c.hll_lut.get<uint16_t>();
        sp.kind = MVA_HLL;
      } else {
        require(c.numeric() || f == PINOT_AGG_COUNTMV, PINOT_ERR_BAD_QUERY,
                "numeric aggregation over STRING column " + c.name);
      }
    }
    a.out = reinterpret_cast<unsigned long long *>(dev);
    a.hll = reinterpret_cast<uint32_t *>(dev + kOut);
    a.docs = reinterpret_cast<unsigned long long *>(dev + kOut + kHll);
    PINOT_HIP(hipMemcpyAsync(dev, init.data(), kOut, hipMemcpyHostToDevice, e.stream));
    PINOT_HIP(hipMemsetAsync(dev + kOut, 0, kHll + 8, e.stream));
    t.timed(1, [&] { launch_mv_aggregate(a, e.stream); });
    PINOT_HIP(hipGetLastError());
    wait_stream(e);  // the result block is reused by the next segment
    Part &pt = parts[si];
    pt.docs = (int64_t)*reinterpret_cast<const volatile unsigned long long *>(host + kOut + kHll);
    pt.v.assign(reinterpret_cast<const unsigned long long *>(host),
                reinterpret_cast<const unsigned long long *>(host) + 5 * kMaxAggs);
    pt.hll.assign(reinterpret_cast<const uint32_t *>(host + kOut),
                  reinterpret_cast<const uint32_t *>(host + kOut) + kMaxAggs * 256);
  }
  PINOT_HIP(hipEventRecord(e.ev_stop, e.stream));
  wait_stream(e);
  float ms = 0;
  PINOT_HIP(hipEventElapsedTime(&ms, e.ev_start, e.ev_stop));
  t.collect();
  auto decode = [](unsigned long long o) {
    const unsigned long long u = (o & 0x8000000000000000ull) ? (o & ~0x8000000000000000ull) : ~o;
    double d;
    memcpy(&d, &u, 8);
    return d;
  };
  std::vector<int64_t> counts(S, 0);
  for (size_t si = 0; si < S; si++) counts[si] = parts[si].docs;
  for (int g = 0; g < na; g++) {
    pinot_agg_result &r = out[g];
    memset(&r, 0, sizeof(r));
    const int f = q.aggregations[g].function;
    const bool exact = true;
    __int128 isum = 0;
    double dsum = 0.0, mn = INFINITY, mx = -INFINITY;
    int64_t entries = 0, docs = 0;
    bool any_fp = false;
    uint8_t regs[256] = {};
    for (size_t si = 0; si < S; si++) {  // CombineService.mergeTwoBlocks, segment order
      const Part &pt = parts[si];
      if (pt.v.empty()) continue;
      docs += pt.docs;
      const unsigned long long *o = pt.v.data() + 5 * g;
      if (o[0] == 0) continue;
      entries += (int64_t)o[0];
      isum += (__int128)(long long)o[1];
      double d;
      memcpy(&d, &o[2], 8);
      if (plans[si].seg->column(agg_column(q.aggregations[g]))->value_kind() == 2) any_fp = true;
      dsum += d;
      mn = java_min(mn, decode(o[3]));
      mx = java_max(mx, decode(o[4]));
      for (int j = 0; j < 256; j++) regs[j] = std::max<uint8_t>(regs[j], (uint8_t)pt.hll[(size_t)g * 256 + j]);
    }
    (void)exact;
    switch (f) {
      case PINOT_AGG_COUNT: r.count = docs; break;
      case PINOT_AGG_COUNTMV: r.count = entries; r.value = (double)entries; break;
      case PINOT_AGG_SUM:
      case PINOT_AGG_SUMMV:
      case PINOT_AGG_AVG:
      case PINOT_AGG_AVGMV:
        r.count = (f == PINOT_AGG_AVG || f == PINOT_AGG_SUM) ? docs : entries;
        if (any_fp) {
          r.value = dsum + (double)isum;
        } else {
          r.value = (double)isum;
          if (isum >= INT64_MIN && isum <= INT64_MAX) {
            r.exact_sum = (int64_t)isum;
            r.has_exact_sum = 1;
          }
        }
        break;
      case PINOT_AGG_MIN:
      case PINOT_AGG_MINMV: r.count = docs; r.value = mn; break;
      case PINOT_AGG_MAX:
      case PINOT_AGG_MAXMV: r.count = docs; r.value = mx; break;
      default:  // DISTINCTCOUNTHLL(MV)
        r.count = docs;
        memcpy(r.hll_registers, regs, 256);
        r.hll_cardinality = hll_cardinality(r.hll_registers);
        break;
    }
  }
  fill_stats(q, plans, counts, ms, stats);
}

}  // namespace

// Per segment, as the reference plans each segment on its own (AggregationPlanNode / AggregationGroupByPlanNode:
// StarTreeUtils.isFitForStarTree over that segment's trees).
bool star_plan_fits(const Engine &e, const SegmentData &seg, const pinot_query &q) {
  if (!e.use_star_tree) return false;
  int slots = q.num_aggregations;  // each AVG adds its AvgPair count column
  for (int a = 0; a < q.num_aggregations; a++) slots += q.aggregations[a].function == PINOT_AGG_AVG;
  return slots <= kMaxAggs && star_tree_fits(seg, q);
}

namespace {

bool star_plan(const Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q) {
  for (SegmentData *s : segs)
    if (!star_plan_fits(e, *s, q)) return false;
  return true;
}

// The star-tree plan's rewritten query: each function over its pre-aggregated pair column (COUNT sums count__*; AVG
// sums the AvgPair halves, "avg__x.sum" in its own slot and "avg__x.count" in a hidden slot after the query's).
struct StarQuery {
  std::vector<std::string> names;         // per slot: the star docs' column
  std::vector<pinot_agg_spec> specs;      // the query's slots, then the hidden AVG count slots
  std::vector<int> hidden;                // per query aggregation: its count slot (AVG) or -1
  pinot_query q{};                        // the query's slots only (stats, projections)
  pinot_query all{};                      // every slot
};
void star_query(const pinot_query &q, StarQuery &sq) {
  const int na = q.num_aggregations;
  int nb = na;
  for (int a = 0; a < na; a++) nb += q.aggregations[a].function == PINOT_AGG_AVG;
  sq.names.assign(nb, "");
  sq.specs.assign(q.aggregations, q.aggregations + na);
  sq.hidden.assign(na, -1);
  for (int a = 0; a < na; a++) {
    const std::string p = star_pair_column(q.aggregations[a]);
    sq.names[a] = q.aggregations[a].function == PINOT_AGG_AVG ? p + ".sum" : p;
    if (sq.specs[a].function == PINOT_AGG_COUNT) sq.specs[a].function = PINOT_AGG_SUM;
    if (q.aggregations[a].function == PINOT_AGG_AVG) {
      const int h = (int)sq.specs.size();
      sq.names[h] = p + ".count";
      pinot_agg_spec hs = q.aggregations[a];
      hs.function = PINOT_AGG_SUM;
      sq.specs.push_back(hs);
      sq.hidden[a] = h;
    }
  }
  for (int b = 0; b < nb; b++) sq.specs[b].column = sq.names[b].c_str();
  sq.q = q;
  sq.q.aggregations = sq.specs.data();
  sq.q.num_filter_nodes = 0;
  sq.q.filter = nullptr;
  sq.all = sq.q;
  sq.all.num_aggregations = nb;
}

void star_stats(const pinot_query &q2, const std::vector<SegmentData *> &segs, const std::vector<StarMatch> &m,
                float ms, pinot_exec_stats *st) {
  if (!st) return;
  memset(st, 0, sizeof(*st));
  for (size_t i = 0; i < segs.size(); i++) {
    st->num_docs_scanned += m[i].docs;
    st->num_entries_scanned_in_filter += m[i].entries_in_filter;
    st->num_total_raw_docs += segs[i]->num_docs;
    st->num_segments_matched += m[i].docs > 0;
  }
  // StarTreeProjectionPlanNode: the pair columns and the group-by dimensions
  st->num_entries_scanned_post_filter = st->num_docs_scanned * projected_columns(q2);
  st->num_segments_processed = (int64_t)segs.size();
  st->device_ms = ms;
}

// Aggregation-only on the segments' star-trees (StarTreeAggregationExecutor): per segment the traversal's matched
// star docs uploaded as a bitset, one k_mv_aggregate over the pair columns, merged in segment order.
void exec_aggregate_star(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q,
                         pinot_agg_result *out, pinot_exec_stats *stats) {
  const int na = q.num_aggregations;
  StarQuery sq;
  star_query(q, sq);
  std::unique_ptr<FilterTreeInput> tree;
  if (q.num_filter_nodes > 0) tree = std::make_unique<FilterTreeInput>(decode_filter(q.num_filter_nodes, q.filter));
  const size_t S = segs.size();
  std::vector<StarMatch> m(S);
  for (size_t si = 0; si < S; si++) m[si] = star_tree_match(*segs[si], q, tree.get());
  e.star_answered.insert(e.star_answered.end(), segs.begin(), segs.end());
  constexpr size_t kOut = 5 * kMaxAggs * 8, kHll = kMaxAggs * 256 * 4;
  e.fused_result.reserve(kOut + kHll + 64);
  uint8_t *dev = e.fused_result.device<uint8_t>();
  const uint8_t *host = e.fused_result.host<uint8_t>();
  std::vector<unsigned long long> init(5 * kMaxAggs, 0ull);
  for (int g = 0; g < kMaxAggs; g++) init[5 * g + 3] = ~0ull;
  PINOT_HIP(hipEventRecord(e.ev_start, e.stream));
  // the HLL register block is max-merged across the segments: zero it once (the fused, MV and earlier star queries
  // leave their registers in the same buffer)
  PINOT_HIP(hipMemsetAsync(dev + kOut, 0, kHll, e.stream));
  std::vector<std::vector<unsigned long long>> parts(S);
  DeviceBuffer bits;
  for (size_t si = 0; si < S; si++) {
    if (m[si].empty || m[si].docs == 0) continue;
    SegmentData &sd = *segs[si]->star->docs;
    bits.reserve(m[si].bits.size() * 8 + 16);
    PINOT_HIP(hipMemcpyAsync(bits.get(), m[si].bits.data(), m[si].bits.size() * 8, hipMemcpyHostToDevice, e.stream));
    MvAggArgs a{};
    a.bitset = bits.get<uint64_t>();
    a.nwords = sd.nwords();
    a.num_docs = sd.num_docs;
    a.n = sq.all.num_aggregations;
    for (int g = 0; g < a.n; g++) {
      MvAggSpec &sp = a.specs[g];
      if (sq.specs[g].function == PINOT_AGG_DISTINCTCOUNTHLL) {  // register rows, max-merged
        sp = MvAggSpec{};
        sp.dict = segs[si]->star->regs.at(sq.names[g]).get();
        sp.kind = MVA_REGS;
        continue;
      }
      ColumnData &c = *sd.column(sq.names[g]);
      sp.fwd = c.fwd.get<uint8_t>();
      sp.offsets = nullptr;
      sp.dict = c.dict_dev.get();
      sp.bits = c.bits;
      sp.value_kind = c.value_kind();
      sp.numeric = 1;
      sp.kind = MVA_VALUES;
    }
    a.out = reinterpret_cast<unsigned long long *>(dev);
    a.hll = reinterpret_cast<uint32_t *>(dev + kOut);
    a.docs = reinterpret_cast<unsigned long long *>(dev + kOut + kHll);
    PINOT_HIP(hipMemcpyAsync(dev, init.data(), kOut, hipMemcpyHostToDevice, e.stream));
    PINOT_HIP(hipMemsetAsync(dev + kOut + kHll, 0, 8, e.stream));
    launch_mv_aggregate(a, e.stream);
    PINOT_HIP(hipGetLastError());
    wait_stream(e);
    parts[si].assign(reinterpret_cast<const unsigned long long *>(host),
                     reinterpret_cast<const unsigned long long *>(host) + 5 * kMaxAggs);
  }
  PINOT_HIP(hipEventRecord(e.ev_stop, e.stream));
  wait_stream(e);
  float ms = 0;
  PINOT_HIP(hipEventElapsedTime(&ms, e.ev_start, e.ev_stop));
  auto decode_ordered_u64 = [](unsigned long long o) {
    const unsigned long long u = (o & 0x8000000000000000ull) ? (o & ~0x8000000000000000ull) : ~o;
    double d;
    memcpy(&d, &u, 8);
    return d;
  };
  for (int g = 0; g < na; g++) {
    pinot_agg_result &r = out[g];
    memset(&r, 0, sizeof(r));
    const int f = q.aggregations[g].function;
    int64_t isum = 0, hcount = 0;
    double dsum = 0.0, mn = INFINITY, mx = -INFINITY;
    for (size_t si = 0; si < S; si++) {  // CombineService.mergeTwoBlocks, segment order
      if (parts[si].empty()) continue;
      const unsigned long long *o = parts[si].data() + 5 * g;
      if (sq.hidden[g] >= 0) hcount += (int64_t)parts[si][5 * sq.hidden[g] + 1];  // Σ avg__x.count (LONG)
      if (o[0] == 0) continue;
      isum = (int64_t)((uint64_t)isum + o[1]);
      double d;
      memcpy(&d, &o[2], 8);
      dsum += d;
      mn = java_min(mn, decode_ordered_u64(o[3]));
      mx = java_max(mx, decode_ordered_u64(o[4]));
    }
    switch (f) {
      case PINOT_AGG_COUNT: r.count = isum; r.value = (double)isum; break;  // Σ count__*
      case PINOT_AGG_SUM: r.value = dsum; break;                           // Σ sum__x (doubles)
      case PINOT_AGG_AVG: r.value = dsum; r.count = hcount; break;         // AvgPair(Σ sum, Σ count)
      case PINOT_AGG_DISTINCTCOUNTHLL: {                                   // addAll over the matched docs
        const uint32_t *h = reinterpret_cast<const uint32_t *>(host + kOut) + (size_t)g * 256;
        for (int j = 0; j < 256; j++) r.hll_registers[j] = (uint8_t)h[j];
        r.hll_cardinality = hll_cardinality(r.hll_registers);
        break;
      }
      case PINOT_AGG_MIN: r.value = mn; break;
      default: r.value = mx; break;
    }
  }
  star_stats(sq.q, segs, m, ms, stats);
}

}  // namespace

void exec_aggregate(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q, pinot_agg_result *out,
                    pinot_exec_stats *stats) {
  const int na = q.num_aggregations;
  require(na >= 1 && na <= kMaxAggs, PINOT_ERR_UNSUPPORTED, "1..8 aggregation functions per query");
  if (touches_mv_aggregation(segs, q)) {
    exec_aggregate_mv(e, segs, q, out, stats);
    return;
  }
  std::vector<SegmentData *> on_star, on_scan;
  for (SegmentData *s : segs) (star_plan_fits(e, *s, q) ? on_star : on_scan).push_back(s);
  if (!on_star.empty() && on_scan.empty()) {
    exec_aggregate_star(e, segs, q, out, stats);
    return;
  }
  if (!on_star.empty()) {  // mixed: each side on its plan, CombineService.mergeTwoBlocks over the two blocks
    std::vector<pinot_agg_result> p1(na), p2(na);
    pinot_exec_stats s1{}, s2{};
    exec_aggregate_star(e, on_star, q, p1.data(), &s1);
    exec_aggregate(e, on_scan, q, p2.data(), &s2);
    merge_agg_parts(q, {p1.data(), p2.data()}, out);
    if (stats) {
      memset(stats, 0, sizeof(*stats));
      for (const pinot_exec_stats *x : {&s1, &s2}) {
        stats->num_docs_scanned += x->num_docs_scanned;
        stats->num_entries_scanned_in_filter += x->num_entries_scanned_in_filter;
        stats->num_entries_scanned_post_filter += x->num_entries_scanned_post_filter;
        stats->num_total_raw_docs += x->num_total_raw_docs;
        stats->num_segments_processed += x->num_segments_processed;
        stats->num_segments_matched += x->num_segments_matched;
        stats->device_ms += x->device_ms;
      }
    }
    return;
  }
  if (e.use_shortcut_plans && shortcut_aggregate(segs, q, out, stats)) return;
  int n_hll = 0;
  for (int a = 0; a < na; a++) {
    const int f = q.aggregations[a].function;
    require(f >= PINOT_AGG_COUNT && f <= PINOT_AGG_DISTINCTCOUNTHLL, PINOT_ERR_UNSUPPORTED, "aggregation function");
    if (f == PINOT_AGG_DISTINCTCOUNTHLL) n_hll++;
  }
  require(n_hll <= kMaxHll, PINOT_ERR_UNSUPPORTED, "at most 4 DISTINCTCOUNTHLL per query");
  const size_t S = segs.size();
  const auto tq0 = std::chrono::steady_clock::now();
  if (e.use_fused && e.use_plan_cache) {  // a repeated fused query: its host plan as last time
    FusedPlan *fp = static_cast<FusedPlan *>(e.fused_plan.get());
    if (fp && fp->small_gen == e.small.generation() && fp->bitsets_gen == e.bitsets.generation() &&
        fp->key == fused_plan_key(e, segs, q)) {
      run_fused(e, *fp, q, out, stats, tq0);
      return;
    }
  }
  std::vector<std::vector<AggRoute>> routes(S);
  for (size_t si = 0; si < S; si++)
    for (int a = 0; a < na; a++) routes[si].push_back(route_agg(e, *segs[si], q.aggregations[a]));
  if (e.use_fused) {
    std::vector<std::string> fold_cols, hll_cols;
    if (fusable(q, routes, fold_cols, hll_cols)) {
      auto fp = std::make_shared<FusedPlan>();
      fp->routes = std::move(routes);
      fp->fold_cols = std::move(fold_cols);
      fp->hll_cols = std::move(hll_cols);
      plan_fused(e, segs, q, *fp);
      fp->key = fused_plan_key(e, segs, q);
      e.fused_plan = fp;
      run_fused(e, *fp, q, out, stats, tq0);
      return;
    }
  }
  Arena ar;
  std::unique_ptr<FilterTreeInput> tree;
  std::vector<SegPlan> plans = plan_all(e, segs, q, ar, tree);
  QueryScratch qs = prepare(e, plans, ar);
  int64_t max_words = 1;
  for (auto &p : plans) max_words = std::max<int64_t>(max_words, p.seg->nwords());
  const int grid = scan_grid(max_words);
  // per-segment result slots: [0] count, [1 + a] aggregation a, [na + 1] discarded duplicate counts;
  // then HLL registers [na][256] u32
  const int nres = na + 2;
  const size_t off_hll = ((S * nres * 8 + 255) / 256) * 256;
  const size_t red_bytes = off_hll + (size_t)na * 256 * 4;
  e.reduced.reserve(red_bytes);
  e.partials.reserve((size_t)grid * kMaxSlots * 8);
  uint8_t *red = e.reduced.get<uint8_t>();
  auto *res_dev = reinterpret_cast<unsigned long long *>(red);
  auto *hll_dev = reinterpret_cast<uint32_t *>(red + off_hll);
  auto *part = e.partials.get<unsigned long long>();

  PINOT_HIP(hipEventRecord(e.ev_start, e.stream));
  PINOT_HIP(hipMemsetAsync(red, 0, red_bytes, e.stream));
  Timer t(e);
  for (size_t si = 0; si < S; si++) {
    SegPlan &p = plans[si];
    SegmentData &s = *p.seg;
    if (p.empty) continue;
    const uint64_t *bits = run_filter(e, p, qs, t);
    const int64_t nwords = s.nwords();
    // partial slot p: part + p * grid ; slot kinds/targets for the reduction
    ReduceArgs ra{};
    ra.in = part;
    ra.stride = grid;
    ra.grid = scan_grid(nwords);  // this segment's launches: the blocks beyond it hold another segment's partials
    ra.out = res_dev + si * nres;
    int nslots = 0;
    auto new_slot = [&](int kind, int target) {
      ra.kinds[nslots] = kind;
      ra.out_index[nslots] = target;
      return part + (int64_t)(nslots++) * grid;
    };
    bool have_count = false;
    const int discard = na + 1;
    // one fold per column over its IDSUM / MINMAX aggregations
    std::map<int, std::vector<int>> by_col;
    for (int a = 0; a < na; a++)
      if (routes[si][a].kind == AggRoute::IDSUM || routes[si][a].kind == AggRoute::MINMAX)
        by_col[routes[si][a].col].push_back(a);
    for (auto &kv : by_col) {
      const ColumnData &c = *s.cols[kv.first];
      ColAggArgs ca{};
      ca.fwd = c.fwd.get<uint8_t>();
      ca.bitset = bits;
      ca.nwords = nwords;
      ca.num_docs = s.num_docs;
      // several aggregations of one kind on one column share the first one's slot (src below)
      int ops = 0;
      int a_sum = -1, a_mm = -1;
      for (int a : kv.second) {
        if (routes[si][a].kind == AggRoute::IDSUM) {
          ops |= COLAGG_IDSUM;
          if (a_sum < 0) a_sum = a;
        } else {
          ops |= COLAGG_MINMAX;
          if (a_mm < 0) a_mm = a;
        }
      }
      ca.out_count = new_slot(SLOT_SUM_U64, have_count ? discard : 0);
      have_count = true;
      if (ops & COLAGG_IDSUM) ca.out_idsum = new_slot(SLOT_SUM_U64, 1 + a_sum);
      if (ops & COLAGG_MINMAX) ca.out_minmax = new_slot(SLOT_MINMAX, 1 + a_mm);
      t.timed(1, [&] { launch_colagg(c.bits, ops, ca, e.stream); });
      PINOT_HIP(hipGetLastError());
    }
    // dictionary / LUT gathers
    GatherArgs ga{};
    ga.bitset = bits;
    ga.nwords = nwords;
    ga.num_docs = s.num_docs;
    int hslot = 0;
    for (int a = 0; a < na; a++) {
      const AggRoute &r = routes[si][a];
      if (r.kind != AggRoute::GATHER && r.kind != AggRoute::HLL) continue;
      ColumnData &c = *s.cols[r.col];
      GatherSpec &g = ga.specs[ga.n++];
      g.bits = c.bits;
      g.fwd = c.fwd.get<uint8_t>();
      if (r.kind == AggRoute::HLL) {
        g.kind = GA_HLL;
        g.table = c.hll_lut.get();
        g.hll_slot = hslot++;
        g.hll_out = hll_dev + a * 256;
      } else {
        g.kind = r.gather_kind;
        g.table = c.dict_dev.get();
        g.out = new_slot(r.gather_kind == GA_SUM_I32 ? SLOT_SUM_U64 : SLOT_SUM_F64, 1 + a);
      }
    }
    if (ga.n) {
      ga.out_count = new_slot(SLOT_SUM_U64, have_count ? discard : 0);
      have_count = true;
      t.timed(1, [&] { launch_gather_agg(ga, e.stream); });
      PINOT_HIP(hipGetLastError());
    }
    if (!have_count && bits) {
      launch_popcount(bits, nwords, s.num_docs, new_slot(SLOT_SUM_U64, 0), e.stream);
      PINOT_HIP(hipGetLastError());
    }
    require(nslots <= kMaxSlots, PINOT_ERR_UNSUPPORTED, "too many aggregation slots");
    // one fixed-order reduction launch for all slots; the next segment reuses `part` behind it in stream order
    launch_reduce_slots(ra, nslots, e.stream);
    PINOT_HIP(hipGetLastError());
  }
  PINOT_HIP(hipEventRecord(e.ev_stop, e.stream));
  e.host_result.reserve(red_bytes);
  uint8_t *host = e.host_result.get<uint8_t>();
  PINOT_HIP(hipMemcpyAsync(host, red, red_bytes, hipMemcpyDeviceToHost, e.stream));
  wait_stream(e);
  float ms = 0;
  PINOT_HIP(hipEventElapsedTime(&ms, e.ev_start, e.ev_stop));
  t.collect();

  AggResults R;
  R.res = reinterpret_cast<const unsigned long long *>(host);
  R.hll = reinterpret_cast<const uint32_t *>(host + off_hll);
  R.nres = nres;
  R.src.assign(S, std::vector<int>(na, 0));
  R.hll_set.resize(na);
  std::vector<int64_t> counts(S, 0);
  for (size_t si = 0; si < S; si++) {
    if (plans[si].empty) counts[si] = 0;
    else if (plans[si].match_all && R.res[si * nres] == 0) counts[si] = plans[si].seg->num_docs;
    else counts[si] = (int64_t)R.res[si * nres];
    // duplicates of one (IDSUM | MINMAX, column) share the first aggregation's slot
    for (int a = 0; a < na; a++) {
      int src = a;
      for (int b = 0; b < a; b++)
        if (routes[si][b].kind == routes[si][a].kind && routes[si][b].col == routes[si][a].col &&
            (routes[si][a].kind == AggRoute::IDSUM || routes[si][a].kind == AggRoute::MINMAX)) {
          src = b;
          break;
        }
      R.src[si][a] = 1 + src;
    }
  }
  for (int a = 0; a < na; a++) R.hll_set[a] = a;
  merge_aggregates(q, plans, routes, counts, R, out);
  fill_stats(q, plans, counts, ms, stats);
}

// ------------------------------------------------------------------ group-by
namespace {

struct KeySpace {
  std::vector<int64_t> gcard;                          // global cardinality per group column
  std::vector<std::vector<std::vector<int32_t>>> remap;  // [segment][gcol] dictId -> global id (empty = identity)
  std::vector<std::vector<std::string>> gvalues;       // [gcol] global id -> string value
  int64_t G = 1;
  bool hashed = false;  // Π cardinalities > kDenseKeyLimit: keys are hash-table slots (G set by the plan)
};
constexpr int64_t kDenseKeyLimit = int64_t(1) << 27;

bool same_dictionary(const ColumnData &a, const ColumnData &b) {
  if (a.data_type != b.data_type || a.card != b.card) return false;
  if (a.data_type == PINOT_INT || a.data_type == PINOT_LONG) {
    // arithmetic progressions are equal when their (base, step) are: no element-wise pass over 1M-entry
    // dictionaries on every query
    if (a.affine && b.affine) return a.affine_base == b.affine_base && a.affine_step == b.affine_step;
    return a.dict_int == b.dict_int;
  }
  if (a.data_type == PINOT_STRING) return a.dict_str == b.dict_str;
  return a.dict_dbl == b.dict_dbl;
}

// Global raw-key space over all segments (the reference merges per-segment results by string key,
// CombineGroupByOperator.java:142-161; a dense device merge needs one key space instead).
KeySpace build_key_space(const std::vector<SegmentData *> &segs, const pinot_query &q) {
  KeySpace ks;
  const int ng = q.num_group_by;
  ks.remap.assign(segs.size(), std::vector<std::vector<int32_t>>(ng));
  ks.gvalues.resize(ng);
  for (int j = 0; j < ng; j++) {
    const std::string name = q.group_by[j];
    const ColumnData &c0 = *segs[0]->column(name);
    bool same = true;
    for (size_t si = 1; si < segs.size(); si++) same = same && same_dictionary(c0, *segs[si]->column(name));
    if (same) {
      ks.gcard.push_back(c0.card);
      ks.gvalues[j].resize(c0.card);
      for (int32_t i = 0; i < c0.card; i++) ks.gvalues[j][i] = c0.string_value(i);
    } else {
      // union dictionary in value order
      const bool is_str = c0.data_type == PINOT_STRING;
      std::set<std::string> strs;
      std::map<std::pair<int64_t, double>, int> nmap;
      auto nkey = [](const ColumnData &c, int32_t i) {
        return std::make_pair(c.data_type <= PINOT_LONG ? c.dict_int[i] : (int64_t)0,
                              c.data_type <= PINOT_LONG ? 0.0 : c.dict_dbl[i]);
      };
      for (auto *s : segs) {
        const ColumnData &c = *s->column(name);
        require(c.data_type == c0.data_type, PINOT_ERR_BAD_QUERY, "group-by column type differs across segments");
        for (int32_t i = 0; i < c.card; i++) {
          if (is_str) strs.insert(c.dict_str[i]);
          else nmap[nkey(c, i)] = 0;
        }
      }
      if (is_str) {
        std::map<std::string, int> idx;
        int k = 0;
        for (auto &v : strs) { idx[v] = k++; ks.gvalues[j].push_back(v); }
        for (size_t si = 0; si < segs.size(); si++) {
          const ColumnData &c = *segs[si]->column(name);
          auto &m = ks.remap[si][j];
          m.resize(c.card);
          for (int32_t i = 0; i < c.card; i++) m[i] = idx[c.dict_str[i]];
        }
      } else {
        int k = 0;
        for (auto &kv : nmap) kv.second = k++;
        ks.gvalues[j].resize(nmap.size());
        for (size_t si = 0; si < segs.size(); si++) {
          const ColumnData &c = *segs[si]->column(name);
          auto &m = ks.remap[si][j];
          m.resize(c.card);
          for (int32_t i = 0; i < c.card; i++) {
            const int g = nmap[nkey(c, i)];
            m[i] = g;
            ks.gvalues[j][g] = c.string_value(i);
          }
        }
      }
      ks.gcard.push_back((int64_t)ks.gvalues[j].size());
    }
  }
  // dense raw keys up to kDenseKeyLimit; beyond (LONG_MAP / ARRAY_MAP holder shapes) the key space is
  // hashed: G becomes the number of hash slots, sized by the caller from the docs
  for (auto g : ks.gcard) {
    if (ks.G > kDenseKeyLimit / std::max<int64_t>(g, 1)) {
      ks.hashed = true;
      break;
    }
    ks.G *= g;
  }
  if (ks.hashed) ks.G = 0;
  return ks;
}

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

AdmissionPlan plan_admission(const std::vector<SegmentData *> &segs, const pinot_query &q, const Engine &e, int64_t G);
AdmissionBuffers admission_buffers(Engine &e, size_t S, int64_t G);
void build_admitted(Engine &e, const AdmissionPlan &ap, size_t S, int64_t G, const AdmissionBuffers &ab);

struct GroupAccs {
  std::vector<int> acc_kind;    // per agg
  std::vector<size_t> acc_bytes_per_key;
};

GroupAccs group_acc_kinds(const SegmentData &s, const pinot_query &q) {
  GroupAccs g;
  for (int a = 0; a < q.num_aggregations; a++) {
    const int f = q.aggregations[a].function, sf = sv_function(f);
    int kind = 5;
    size_t bytes = 0;
    if (f == PINOT_AGG_COUNTMV) {  // entries per group (an int64 sum)
      kind = 6;
      bytes = 8;
    } else if (f != PINOT_AGG_COUNT) {
      const ColumnData &c = *s.column(agg_column(q.aggregations[a]));
      if (sf == PINOT_AGG_DISTINCTCOUNTHLL) {
        kind = 4;
        bytes = 1024;
      } else {
        require(c.numeric(), PINOT_ERR_UNSUPPORTED, "numeric aggregation over STRING column " + c.name);
        if (sf == PINOT_AGG_MIN) kind = 2;
        else if (sf == PINOT_AGG_MAX) kind = 3;
        else kind = c.data_type == PINOT_INT ? 0 : 1;
        bytes = 8;
      }
    }
    g.acc_kind.push_back(kind);
    g.acc_bytes_per_key.push_back(bytes);
  }
  return g;
}

GroupByProgram make_group_program(Engine &e, SegmentData &s, const pinot_query &q, const GroupAccs &ga,
                                  const KeySpace &ks, size_t si, const std::vector<DeviceBuffer> &remaps,
                                  unsigned long long *counts, void *const *accs) {
  GroupByProgram gp{};
  gp.n_gcols = q.num_group_by;
  gp.n_aggs = q.num_aggregations;
  std::map<int, int> slots;
  auto slot = [&](const ColumnData &c) {
    int ci = s.by_name[c.name];
    auto it = slots.find(ci);
    if (it != slots.end()) return it->second;
    int k = (int)slots.size();
    require(k < kMaxProgramColumns, PINOT_ERR_UNSUPPORTED, "too many columns");
    slots[ci] = k;
    gp.cols[k] = c.dev();
    return k;
  };
  long long stride = 1;
  for (int j = 0; j < q.num_group_by; j++) {
    const ColumnData &c = *s.column(q.group_by[j]);
    gp.gcol[j] = slot(c);
    gp.remap[j] = ks.remap[si][j].empty() ? nullptr : remaps[si * q.num_group_by + j].get<int32_t>();
    gp.stride[j] = stride;
    stride *= ks.gcard[j];
  }
  gp.counts = counts;
  for (int a = 0; a < q.num_aggregations; a++) {
    gp.acc_kind[a] = ga.acc_kind[a];
    gp.acc[a] = accs[a];
    AggSpecDev &sd = gp.aggs[a];
    sd.kind = 0;
    if (ga.acc_kind[a] == 5) continue;
    ColumnData &c = *s.column(agg_column(q.aggregations[a]));
    sd.col = slot(c);
    sd.dict = c.dict_dev.get();
    gp.value_kind[a] = c.value_kind();
    if (ga.acc_kind[a] == 4) {
      ensure_hll_lut(e, c);
      sd.hll_lut = c.hll_lut.get<uint16_t>();
    }
  }
  gp.n_cols = (int)slots.size();
  return gp;
}

double decode_ordered(uint64_t o) {
  uint64_t u = (o & 0x8000000000000000ull) ? (o & ~0x8000000000000000ull) : ~o;
  double d;
  memcpy(&d, &u, 8);
  return d;
}

void parallel_tasks(size_t n, const std::function<void(size_t)> &fn);
size_t host_threads();

// Dense accumulators -> result arrays (bitset path and the multi-GPU partial finalize): ordered device
// compaction of the non-empty keys, one gather, D2H into grow-only engine buffers, host fill over 8 threads.
std::unique_ptr<GroupByResult> finalize_groups(Engine &e, const pinot_query &q, const GroupAccs &ga,
                                               const KeySpace &ks, GroupByProgram gp, const MvHash *mh = nullptr) {
  const int na = q.num_aggregations;
  const size_t cscr = compact_keys_scratch_bytes(ks.G);
  e.group_final.reserve(std::max<int64_t>(ks.G, 1) * 8 + 64 + cscr);
  auto *keys_dev = e.group_final.get<long long>();
  auto *n_dev = reinterpret_cast<unsigned long long *>(e.group_final.get<uint8_t>() + ks.G * 8);
  launch_compact_keys_ordered(ks.G, gp.counts, keys_dev, n_dev, e.group_final.get<uint8_t>() + ks.G * 8 + 64, cscr,
                              e.stream);
  PINOT_HIP(hipGetLastError());
  unsigned long long n = 0;
  PINOT_HIP(hipMemcpyAsync(&n, n_dev, 8, hipMemcpyDeviceToHost, e.stream));
  wait_stream(e);
  int n_hll = 0;
  for (int a = 0; a < na; a++) n_hll += ga.acc_kind[a] == 4;
  auto res = std::make_unique<GroupByResult>();
  res->num_columns = q.num_group_by;
  res->functions.resize(na);
  res->counts.assign(na, {});
  res->values.assign(na, {});
  res->hll.assign(na, {});
  res->hll_card.assign(na, {});
  res->gvalues = ks.gvalues;
  res->gcard = ks.gcard;
  for (int a = 0; a < na; a++) res->functions[a] = q.aggregations[a].function;
  if (n == 0) return res;
  // device layout == host layout: keys [n], counts [n], accs [na][n], HLL registers [n_hll][n][256]
  const size_t out_b = n * 8 * (2 + na) + (size_t)n_hll * n * 256 + 16;
  e.group_out.reserve(out_b);
  e.group_host.reserve(out_b);
  auto *o_keys = e.group_out.get<long long>();
  auto *o_cnt = reinterpret_cast<unsigned long long *>(o_keys + n);
  auto *o_acc = o_cnt + n;
  auto *o_hll = reinterpret_cast<uint8_t *>(o_acc + n * na);
  PINOT_HIP(hipMemcpyAsync(o_keys, keys_dev, n * 8, hipMemcpyDeviceToDevice, e.stream));
  launch_gather_groups(gp, keys_dev, (int64_t)n, o_cnt, o_acc, o_hll, e.stream);
  PINOT_HIP(hipGetLastError());
  DeviceBuffer ids;
  if (mh) {  // hashed key space: the groups are slots; their global-id tuples from the table
    ids.alloc(n * q.num_group_by * 4 + 16);
    launch_mv_hash_tuples(*mh, q.num_group_by, keys_dev, (long long)n, ids.get<int32_t>(), e.stream);
    PINOT_HIP(hipGetLastError());
    res->key_ids.resize(n * q.num_group_by);
    PINOT_HIP(hipMemcpyAsync(res->key_ids.data(), ids.get(), n * q.num_group_by * 4, hipMemcpyDeviceToHost, e.stream));
  }
  PINOT_HIP(hipMemcpyAsync(e.group_host.get(), e.group_out.get(), out_b, hipMemcpyDeviceToHost, e.stream));
  wait_stream(e);
  const auto *hkeys = e.group_host.get<long long>();
  const auto *hcnt = reinterpret_cast<const unsigned long long *>(hkeys + n);
  const auto *hacc = hcnt + n;
  const auto *hhll = reinterpret_cast<const uint8_t *>(hacc + n * na);
  res->raw_keys.assign(hkeys, hkeys + n);
  std::vector<int> hidx(na, -1);
  for (int a = 0, h = 0; a < na; a++) {
    res->counts[a].resize(n);
    res->values[a].resize(n);
    if (ga.acc_kind[a] == 4) {
      hidx[a] = h++;
      res->hll[a].resize(n * 256);
      res->hll_card[a].resize(n);
    }
  }
  const size_t nt = n >= (1u << 16) ? host_threads() : 1;
  parallel_tasks(nt, [&](size_t t) {
    const size_t lo = n * t / nt, hi = n * (t + 1) / nt;
    for (int a = 0; a < na; a++) {
      int64_t *cv = res->counts[a].data();
      double *vv = res->values[a].data();
      const int ak = ga.acc_kind[a];
      for (size_t i = lo; i < hi; i++) {
        cv[i] = (int64_t)hcnt[i];
        const uint64_t raw = hacc[(size_t)a * n + i];
        switch (ak) {
          case 0:
          case 6:
          case 7: vv[i] = (double)(int64_t)raw; break;
          case 1: { double d; memcpy(&d, &raw, 8); vv[i] = d; break; }
          case 2:
          case 3: vv[i] = decode_ordered(raw); break;
          case 4: {
            uint8_t *r = res->hll[a].data() + i * 256;
            memcpy(r, hhll + ((size_t)hidx[a] * n + i) * 256, 256);
            res->hll_card[a][i] = hll_cardinality(r);
            vv[i] = (double)res->hll_card[a][i];
            break;
          }
          default: vv[i] = (double)hcnt[i]; break;
        }
      }
    }
  });
  return res;
}

// Device count of the docs in a bitset (blocking; used only by the group-limit rule).
int64_t count_docs(Engine &e, const uint64_t *bits, const SegmentData &s) {
  if (!bits) return s.num_docs;
  const int grid = scan_grid(s.nwords());
  DeviceBuffer part((size_t)grid * 8 + 64);
  auto *p = part.get<unsigned long long>();
  launch_popcount(bits, s.nwords(), s.num_docs, p, e.stream);
  ReduceArgs ra{};
  ra.in = p;
  ra.stride = grid;
  ra.grid = grid;
  ra.out = p + grid;
  launch_reduce_slots(ra, 1, e.stream);
  unsigned long long c = 0;
  PINOT_HIP(hipMemcpyAsync(&c, p + grid, 8, hipMemcpyDeviceToHost, e.stream));
  wait_stream(e);
  return (int64_t)c;
}

// Accumulates every segment's group-by into the given device arrays (already initialised).
void accumulate_groups(Engine &e, std::vector<SegPlan> &plans, const QueryScratch &qs, const pinot_query &q,
                       const GroupAccs &ga, const KeySpace &ks, unsigned long long *counts, void *const *accs,
                       Timer &t, std::vector<int64_t> &seg_counts, bool apply_limit) {
  const size_t S = plans.size();
  std::vector<DeviceBuffer> remaps(S * q.num_group_by);
  for (size_t si = 0; si < S; si++)
    for (int j = 0; j < q.num_group_by; j++) {
      const auto &m = ks.remap[si][j];
      if (m.empty()) continue;
      remaps[si * q.num_group_by + j].alloc(m.size() * 4 + 16);
      PINOT_HIP(hipMemcpyAsync(remaps[si * q.num_group_by + j].get(), m.data(), m.size() * 4, hipMemcpyHostToDevice,
                               e.stream));
    }
  seg_counts.assign(S, 0);
  std::vector<SegmentData *> sv(S);
  for (size_t si = 0; si < S; si++) sv[si] = plans[si].seg;
  // num.groups.limit (per segment and the inter-segment cap): first doc per key of every segment, admitted bitmaps
  const AdmissionPlan ap = apply_limit ? plan_admission(sv, q, e, ks.G) : AdmissionPlan{};
  AdmissionBuffers ab;
  if (ap.active) {
    ab = admission_buffers(e, S, ks.G);
    PINOT_HIP(hipMemsetAsync(ab.first_doc, 0xFF, (size_t)S * ks.G * 4, e.stream));
    for (size_t si = 0; si < S; si++) {
      SegPlan &p = plans[si];
      if (p.empty) continue;
      const uint64_t *bits = run_filter(e, p, qs, t);
      GroupByProgram gp = make_group_program(e, *p.seg, q, ga, ks, si, remaps, counts, accs);
      launch_first_doc(gp, bits, p.seg->nwords(), p.seg->num_docs, ab.first_doc + si * ks.G, e.stream);
      PINOT_HIP(hipGetLastError());
    }
    build_admitted(e, ap, S, ks.G, ab);
  }
  for (size_t si = 0; si < S; si++) {
    SegPlan &p = plans[si];
    SegmentData &s = *p.seg;
    if (p.empty) continue;
    const uint64_t *bits = run_filter(e, p, qs, t);
    seg_counts[si] = count_docs(e, bits, s);
    GroupByProgram gp = make_group_program(e, s, q, ga, ks, si, remaps, counts, accs);
    if (ap.active) gp.admitted = ab.bitmaps + si * ab.words;
    t.timed(1, [&] { launch_group_by(gp, bits, s.nwords(), s.num_docs, e.stream); });
    PINOT_HIP(hipGetLastError());
  }
}

void init_accs(Engine &e, int64_t G, unsigned long long *counts, const GroupAccs &ga, void *const *accs) {
  PINOT_HIP(hipMemsetAsync(counts, 0, G * 8, e.stream));
  for (size_t a = 0; a < ga.acc_kind.size(); a++) {
    if (ga.acc_kind[a] == 5) continue;
    PINOT_HIP(hipMemsetAsync(accs[a], ga.acc_kind[a] == 2 ? 0xFF : 0, G * ga.acc_bytes_per_key[a], e.stream));
  }
}

}  // namespace

// Result-array pool: a 1 M-group result is ~48 MB of fresh host pages, and first-touching them cost more than
// filling them. Released results hand their arrays back; the next large result takes them (capacity kept).
namespace {
// Recycled host result arrays (a 1M-group result allocates several 8 MB arrays per query). Bounded: at most
// kPoolMaxBytes held in total; take = best fit, and an array more than twice the request stays pooled for a
// larger result instead of being handed to a small one.
struct ResultPool {
  std::mutex mu;
  std::vector<HostVec<int64_t>> i64;
  std::vector<HostVec<double>> f64;
  size_t bytes = 0;
};
ResultPool &result_pool() {
  static ResultPool *p = new ResultPool;  // never destroyed: results may be released during interpreter exit
  return *p;
}
constexpr size_t kPoolMinElems = 1u << 16, kPoolMaxArrays = 16, kPoolMaxBytes = 256ull << 20;
template <class T>
HostVec<T> take_pooled(ResultPool &rp, std::vector<HostVec<T>> &pool, size_t n) {
  size_t best = SIZE_MAX;
  for (size_t i = 0; i < pool.size(); i++) {
    const size_t cap = pool[i].capacity();
    if (cap >= n && cap <= 2 * std::max(n, kPoolMinElems) && (best == SIZE_MAX || cap < pool[best].capacity()))
      best = i;
  }
  if (best == SIZE_MAX) return {};
  HostVec<T> v = std::move(pool[best]);
  pool.erase(pool.begin() + best);
  rp.bytes -= v.capacity() * sizeof(T);
  return v;
}
}  // namespace

GroupByResult::~GroupByResult() {
  ResultPool &p = result_pool();
  std::lock_guard<std::mutex> lk(p.mu);
  auto put = [&p](auto &pool, auto &v) {
    const size_t b = v.capacity() * sizeof(v[0]);
    if (v.capacity() >= kPoolMinElems && pool.size() < kPoolMaxArrays && p.bytes + b <= kPoolMaxBytes) {
      // size kept: the next result's resize(n) then shrinks without touching the pages (clear() would make it
      // zero-fill n elements the fill overwrites anyway)
      pool.push_back(std::move(v));
      p.bytes += b;
    }
  };
  put(p.i64, raw_keys);
  for (auto &v : counts) put(p.i64, v);
  for (auto &v : hll_card) put(p.i64, v);
  for (auto &v : values) put(p.f64, v);
}

void group_by_hll_registers(const GroupByResult &r, int fn, uint8_t *registers, bool pinned_dst) {
  const size_t n = r.raw_keys.size();
  if (!n) return;
  if (r.hll_parts.empty()) {
    memcpy(registers, r.hll[fn].data(), n * 256);
    return;
  }
  // a caller's (pageable) buffer is never the copy target: the runtime would pin it in place, and its later unmap
  // stalls the GPU queues; the registers pass through a pinned, cached staging block instead
  HostVec<uint8_t> stage;
  uint8_t *dst = registers;
  if (!pinned_dst) {
    stage.resize(n * 256);
    dst = stage.data();
  }
  int caller_dev = 0;
  PINOT_HIP(hipGetDevice(&caller_dev));
  struct Restore {  // the caller's current device, whatever the parts' devices were
    int d;
    ~Restore() { (void)hipSetDevice(d); }
  } restore{caller_dev};
  for (const HllPart &p : r.hll_parts) {
    if (!p.num_groups) continue;
    PINOT_HIP(hipSetDevice(p.device));
    PINOT_HIP(hipMemcpy(dst + p.group_begin * 256, p.buf->get<uint8_t>() + p.off[fn], p.num_groups * 256,
                        hipMemcpyDeviceToHost));
  }
  if (!pinned_dst) memcpy(registers, dst, n * 256);
}

// DictionaryBasedGroupKeyGenerator.getGroupKey (:421-437): column 0 first, values '\t'-joined.
const std::string &GroupByResult::key(int64_t g) const {
  if (keys.size() != raw_keys.size()) {
    keys.assign(raw_keys.size(), std::string());
    key_built.assign(raw_keys.size(), 0);
  }
  if (!key_built[g]) {
    int64_t k = raw_keys[g];
    std::string s;
    const size_t nc = gcard.size();
    for (size_t j = 0; j < nc; j++) {
      if (j) s += '\t';
      if (!key_ids.empty()) {
        s += gvalues[j][key_ids[g * nc + j]];
      } else {
        s += gvalues[j][k % gcard[j]];
        k /= gcard[j];
      }
    }
    keys[g] = std::move(s);
    key_built[g] = 1;
  }
  return keys[g];
}

namespace {
void parallel_tasks(size_t n, const std::function<void(size_t)> &fn);
}

// Bulk key export: lengths of every key (mixed-radix digits -> dictionary strings), a prefix sum, then the
// bytes, each pass split over 8 threads for large results.
uint64_t GroupByResult::export_keys(char *buf, uint64_t buf_len, int64_t *offsets) const {
  const int64_t n = (int64_t)raw_keys.size();
  const size_t nc = gcard.size();
  const size_t nt = n >= (1 << 16) ? host_threads() : 1;
  auto digit = [&](int64_t g, size_t j, int64_t &k) -> const std::string & {
    if (!key_ids.empty()) return gvalues[j][key_ids[g * nc + j]];
    const std::string &v = gvalues[j][k % gcard[j]];
    k /= gcard[j];
    return v;
  };
  if ((int64_t)key_offsets.size() != n + 1) {
    std::vector<int64_t> off(n + 1, 0);
    std::vector<int64_t> part(nt + 1, 0);
    parallel_tasks(nt, [&](size_t t) {
      const int64_t lo = n * t / nt, hi = n * (t + 1) / nt;
      int64_t acc = 0;
      for (int64_t g = lo; g < hi; g++) {
        int64_t k = raw_keys[g], len = (int64_t)nc - 1;
        for (size_t j = 0; j < nc; j++) len += (int64_t)digit(g, j, k).size();
        off[g + 1] = len;
        acc += len;
      }
      part[t + 1] = acc;
    });
    for (size_t t = 0; t < nt; t++) part[t + 1] += part[t];
    parallel_tasks(nt, [&](size_t t) {
      const int64_t lo = n * t / nt, hi = n * (t + 1) / nt;
      int64_t run = part[t];
      for (int64_t g = lo; g < hi; g++) {
        run += off[g + 1];
        off[g + 1] = run;
      }
    });
    key_offsets.swap(off);
  }
  const uint64_t need = (uint64_t)key_offsets[n];
  if (offsets) memcpy(offsets, key_offsets.data(), (size_t)(n + 1) * 8);
  if (!buf || buf_len < need) return need;
  parallel_tasks(nt, [&](size_t t) {
    const int64_t lo = n * t / nt, hi = n * (t + 1) / nt;
    for (int64_t g = lo; g < hi; g++) {
      char *p = buf + key_offsets[g];
      int64_t k = raw_keys[g];
      for (size_t j = 0; j < nc; j++) {
        if (j) *p++ = '\t';
        const std::string &v = digit(g, j, k);
        memcpy(p, v.data(), v.size());
        p += v.size();
      }
    }
  });
  return need;
}

// AggregationGroupByTrimmingService.trimIntermediateResultsMap (:71-116) for one function: above
// 4 * max(5 * topN, 5000) groups, keep the trimSize best final values — ComparableSorter (COUNT / SUM / MIN / MAX /
// AVG: the intermediate value; AvgPair compares sum / count) or NonComparableSorter (DISTINCTCOUNTHLL: the final
// cardinality) — MIN ascending, every other function descending (getSorter :160-176). The reference's heap keeps
// an arbitrary member of a tie at the boundary; here the lower raw key wins.
std::vector<int64_t> GroupByResult::trim(int32_t top_n, int32_t fn) const {
  if (trimmed_top_n) {  // the device already kept each function's trimSize best groups
    require(top_n == trimmed_top_n, PINOT_ERR_BAD_ARG, "result was trimmed on the device for another TOP n");
    return fn_kept.at(fn);
  }
  const int64_t n = (int64_t)raw_keys.size();
  const int64_t trim_size = std::max<int64_t>(5 * (int64_t)top_n, 5000);
  std::vector<int64_t> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  if (n <= 4 * trim_size) return idx;
  const int f = sv_function(functions[fn]);
  const HostVec<int64_t> &cnt = counts[counts_shared ? 0 : fn];
  std::vector<double> v(n);
  for (int64_t g = 0; g < n; g++) {
    switch (f) {
      case PINOT_AGG_COUNT: v[g] = (double)cnt[g]; break;
      case PINOT_AGG_AVG: v[g] = cnt[g] ? values[fn][g] / (double)cnt[g] : -INFINITY; break;
      case PINOT_AGG_DISTINCTCOUNTHLL: v[g] = (double)hll_card[fn][g]; break;
      default: v[g] = values[fn][g]; break;
    }
  }
  const bool asc = f == PINOT_AGG_MIN;
  auto better = [&](int64_t a, int64_t b) {
    if (v[a] != v[b]) return asc ? v[a] < v[b] : v[a] > v[b];
    return a < b;
  };
  std::nth_element(idx.begin(), idx.begin() + trim_size, idx.end(), better);
  idx.resize(trim_size);
  std::sort(idx.begin(), idx.end());
  return idx;
}

std::unique_ptr<GroupByResult> exec_group_by_legacy(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q,
                                                    pinot_exec_stats *stats);

namespace {

// Runs fn(0..n-1) on up to n threads (the calling thread takes task 0).
namespace {
// Persistent host workers for the result fills (spawning threads per call cost ~0.1 ms per call, several calls per
// query). One job at a time: a second concurrent caller (another engine's thread in the multi-GPU server) runs its
// tasks on threads of its own instead of waiting. g_pool_spin: the pause instructions a pool thread spins after a job
// before it sleeps (engine key host.spin; process-wide, the pool is shared by every engine). Short by default, so an
// idle server's host cores sleep between queries.
std::atomic<int> g_pool_spin{2000};

class TaskPool {
 public:
  static TaskPool &get() {
    static TaskPool *p = new TaskPool();  // never destroyed: workers may outlive static destruction order
    return *p;
  }
  size_t threads() const { return workers_ + 1; }
  bool try_run(size_t n, const std::function<void(size_t)> &fn) {
    std::unique_lock<std::mutex> busy(job_mu_, std::try_to_lock);
    if (!busy.owns_lock()) return false;
    auto job = std::make_shared<Job>();
    job->fn = &fn;
    job->n = n;
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = job;
      gen_++;
      gen_seen_.store(gen_, std::memory_order_release);
    }
    cv_.notify_all();
    work(*job);  // the caller takes tasks too
    const int spin_n = g_pool_spin.load(std::memory_order_relaxed);
    for (int spin = 0; spin < spin_n && job->done.load(std::memory_order_acquire) != n; spin++) pause();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return job->done.load() == n; });
    job_.reset();
    return true;
  }

 private:
  struct Job {
    const std::function<void(size_t)> *fn = nullptr;
    size_t n = 0;
    std::atomic<size_t> next{0}, done{0};
  };
  TaskPool() {
    const unsigned hc = std::max(1u, std::thread::hardware_concurrency());
    workers_ = std::min<size_t>(15, hc > 1 ? hc - 1 : 0);
    for (size_t i = 0; i < workers_; i++) std::thread([this] { loop(); }).detach();
  }
  void work(Job &j) {
    for (;;) {
      const size_t i = j.next.fetch_add(1);
      if (i >= j.n) return;
      (*j.fn)(i);
      if (j.done.fetch_add(1) + 1 == j.n) {
        std::lock_guard<std::mutex> lk(mu_);
        done_cv_.notify_all();
      }
    }
  }
  // A worker that finished a job spins briefly before sleeping (host.spin pause instructions): the host phases issue
  // their parallel passes a few microseconds apart, and a condition-variable wake costs tens of microseconds per pass.
  static void pause() { __builtin_ia32_pause(); }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      const int spin_n = g_pool_spin.load(std::memory_order_relaxed);
      for (int spin = 0; spin < spin_n && gen_seen_.load(std::memory_order_acquire) == seen; spin++) pause();
      std::shared_ptr<Job> j;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        j = job_;
      }
      if (j) work(*j);
    }
  }
  size_t workers_ = 0;
  std::mutex job_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::shared_ptr<Job> job_;
  uint64_t gen_ = 0;
  std::atomic<uint64_t> gen_seen_{0};  // gen_, readable without the lock (the spin)
};
}  // namespace

size_t host_threads() { return std::min<size_t>(16, TaskPool::get().threads()); }

}  // namespace

void set_host_spin(int pauses) { g_pool_spin.store(std::max(0, pauses), std::memory_order_relaxed); }

namespace {

void parallel_tasks(size_t n, const std::function<void(size_t)> &fn) {
  if (n <= 1) {
    if (n == 1) fn(0);
    return;
  }
  if (TaskPool::get().try_run(n, fn)) return;
  std::vector<std::thread> th;
  struct Join {  // every started thread is joined, also when starting one throws or fn(0) throws
    std::vector<std::thread> &t;
    ~Join() {
      for (auto &x : t)
        if (x.joinable()) x.join();
    }
  } join{th};
  th.reserve(n - 1);
  for (size_t t = 1; t < n; t++) th.emplace_back(fn, t);
  fn(0);
}

// Fused group-by plan (GroupMode) chosen from the key space and the accumulators' per-key bytes.
struct GroupPlan {
  int mode = GB_GLOBAL;
  int shift = 0;        // partitioned: 2^shift keys per partition
  int split = 0;        // two-level: 2^split partitions per coarse run of the EMIT pass
  int64_t P = 0;
  int lds_acc_bytes = 0;
  std::vector<int> lds_off, field_shift, reduce_off;
  int reduce_bytes = 0;
  int reduce_wave_cnt_off = 0;
  int record_bits = 0;  // partitioned: local key + aggregated fields (the bucketed EMIT keeps bit 63 as a valid mark)
};

constexpr int kRingInstanceCode = 90000;  // group.last_instance of a ring-plan query

constexpr int kGroupMaxFusedLeafBits = 12;    // 16 wave stages x 6 KiB
constexpr int kGroupLdsAccBudget = 60 * 1024;  // GB_LDS accumulators / GB_COUNT-EMIT partition cursors
constexpr int kReduceLdsBudget = 152 * 1024;   // k_partition_reduce accumulators (one block per CU)
constexpr int64_t kMaxPartitions = 16384;       // 64 KiB of partition cursors beside 16 x 6 KiB wave stages

size_t lds_acc_bytes_per_key(int kind, bool lds_hll_u32) {
  if (kind == 5) return 0;
  if (kind == 4) return lds_hll_u32 ? 1024 : 256;
  return 8;
}

constexpr int64_t kCoarseRuns = 16;  // EMIT's live run cursors per block (16: fewest lines per scattered store, measured)

GroupPlan plan_group(const std::vector<SegmentData *> &segs, const pinot_query &q, const KeySpace &ks,
                     const GroupAccs &ga, const std::string &force, int force_split, int max_shift) {
  GroupPlan gp;
  const int na = q.num_aggregations;
  gp.lds_off.assign(na, 0);
  gp.field_shift.assign(na, 0);
  gp.reduce_off.assign(na, 0);
  // GB_LDS: counts u32 [G], then each accumulator array (8-byte aligned)
  size_t off = ((size_t)ks.G * 4 + 7) / 8 * 8;
  for (int a = 0; a < na; a++) {
    gp.lds_off[a] = (int)std::min<size_t>(off, INT32_MAX);
    off += (size_t)ks.G * lds_acc_bytes_per_key(ga.acc_kind[a], true);
  }
  if (off <= (size_t)kGroupLdsAccBudget && (force.empty() || force == "lds")) {
    gp.mode = GB_LDS;
    gp.lds_acc_bytes = (int)off;
    return gp;
  }
  // partitioned: identical aggregated dictionaries on every segment (records carry dictIds) and a record
  // (local key + each aggregated column's dictId) within 64 bits
  bool same = true;
  for (int a = 0; a < na && same; a++) {
    if (ga.acc_kind[a] == 5) continue;
    const ColumnData &c0 = *segs[0]->column(agg_column(q.aggregations[a]));
    for (size_t si = 1; si < segs.size(); si++) same = same && same_dictionary(c0, *segs[si]->column(c0.name));
  }
  size_t per_key = 4 + 16;  // shared count slot + 4 private count copies
  for (int a = 0; a < na; a++) per_key += lds_acc_bytes_per_key(ga.acc_kind[a], false);  // u8 HLL registers
  int shift = 0;
  while (shift < 12 && ((size_t)2 << shift) * per_key <= (size_t)kReduceLdsBudget) shift++;
  if (max_shift >= 0) shift = std::min(max_shift, 16);  // group.pshift: an explicit partition size (experiments)
  const int64_t K = int64_t(1) << shift;
  const int64_t P = (ks.G + K - 1) / K;
  // two-level: EMIT scatters into ceil(P / 2^split) coarse runs (few enough live lines per block to combine
  // in L2), k_partition_split then moves each run's records to their partitions
  int agg_bits = 0;
  {
    std::set<std::string> seen;
    for (int a = 0; a < na; a++)
      if (ga.acc_kind[a] != 5 && seen.insert(agg_column(q.aggregations[a])).second)
        agg_bits += segs[0]->column(agg_column(q.aggregations[a]))->bits;
  }
  int split = 0;
  if (force_split >= 0) split = force_split;
  else
    while (split < 8 && ((P + (int64_t(1) << split) - 1) >> split) > kCoarseRuns) split++;
  while (split > 0 && shift + split + agg_bits > 64) split--;
  // record layout: [shift + split bits local key | one field per distinct aggregated column]
  std::map<std::string, int> col_field;
  int bits = shift + split;
  for (int a = 0; a < na; a++) {
    if (ga.acc_kind[a] == 5) continue;
    const std::string c = agg_column(q.aggregations[a]);
    auto it = col_field.find(c);
    if (it == col_field.end()) {
      it = col_field.emplace(c, bits).first;
      bits += segs[0]->column(c)->bits;
    }
    gp.field_shift[a] = it->second;
  }
  const bool want_part = force.empty() ? ks.G >= 4 * K : force == "partition";
  if (same && bits <= 64 && P <= kMaxPartitions && want_part && force != "global") {
    gp.mode = GB_EMIT;  // COUNT + EMIT (+ split) + reduce
    gp.record_bits = bits;
    gp.shift = shift;
    gp.split = split;
    gp.P = P;
    size_t roff = ((size_t)K * 4 + 15) / 16 * 16;
    for (int a = 0; a < na; a++) {
      gp.reduce_off[a] = (int)roff;
      roff += ((size_t)K * lds_acc_bytes_per_key(ga.acc_kind[a], false) + 15) / 16 * 16;
    }
    gp.reduce_wave_cnt_off = (int)roff;
    roff += (size_t)K * 4 * 4;  // k_partition_reduce: 4 private count copies
    gp.reduce_bytes = (int)roff;
    return gp;
  }
  gp.mode = GB_GLOBAL;
  return gp;
}

// Ring plan (group_ring.hip): the partitioned plan without its histogram pass. Applies to dense key spaces whose
// partitions of K <= 1024 keys number at most kRingMaxPartitions (k_group_ring's LDS rings), read through the
// lane-owns-quarter decoder (<= 4 columns of <= 20 bits) with records of <= 53 bits.
constexpr size_t kRingReduceLds = 160 * 1024;
constexpr int kRingHllFieldBits = 13;  // register (8 bits, log2m = 8) << 5 | rank (<= 25)
struct RingPlan {
  bool on = false;
  int shift = 0;
  int64_t P = 0;
  int rec_bytes = 8;                     // 6 when the record fields fit 48 bits (group.ring_rec6)
  std::vector<int> field_shift, lds_off;
  std::vector<int> hll_form;             // per aggregation: 1 = the HLL whose field the scatter computes (at most one)
  int cnt_off = 0, hist_off = 0, exc_off = 0, lds_bytes = 0;
  uint32_t cap = 0;        // records per region the allocation holds
  int64_t nblk = 0;
  int64_t total_chunks = 0;
};

RingPlan plan_ring(const Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q, const KeySpace &ks,
                   const GroupAccs &gx, int64_t total_chunks) {
  RingPlan rp;
  const int na = q.num_aggregations;
  if (ks.G <= 0 || ks.G > (int64_t)UINT32_MAX || total_chunks <= 0) return rp;
  // columns: the group columns, then one slot per distinct accumulator (as the EMIT prefetch lists them)
  int nc = q.num_group_by;
  for (int a = 0; a < na; a++) nc += gx.acc_kind[a] != 5;
  if (nc > kGroupPfCols || q.num_group_by > kRingGroupCols || nc - q.num_group_by > kRingAggCols) return rp;
  for (auto *s : segs) {
    for (int j = 0; j < q.num_group_by; j++)
      if (s->column(q.group_by[j])->bits > kGroupLwMaxBits) return rp;
    for (int a = 0; a < na; a++)
      if (gx.acc_kind[a] != 5 && s->column(agg_column(q.aggregations[a]))->bits > kGroupLwMaxBits) return rp;
  }
  const size_t nblk = (size_t)e.num_cus;
  const size_t fixed = nblk * 4 + (4 + (size_t)ring_reduce_exceptions()) * 4 + 256;
  size_t per_key = 4;
  for (int a = 0; a < na; a++)
    if (gx.acc_kind[a] != 5) per_key += gx.acc_kind[a] == 4 ? 128 : 8;
  int s = 10;
  while (s > 0 && ((size_t)1 << s) * per_key + fixed > kRingReduceLds) s--;
  const int64_t need = (ks.G + kRingMaxPartitions - 1) / kRingMaxPartitions;  // K >= G / max partitions
  if (((int64_t)1 << s) < need) return rp;
  while (s > 5 && ((ks.G + ((int64_t)1 << (s - 1)) - 1) >> (s - 1)) <= kRingMaxPartitions &&
         ((ks.G + ((int64_t)1 << s) - 1) >> s) < 2 * (int64_t)nblk)
    s--;  // small key spaces: more, smaller partitions for the reduce's grid
  const int64_t K = (int64_t)1 << s;
  rp.P = (ks.G + K - 1) / K;
  if (rp.P > kRingMaxPartitions || ring_lds_bytes((int)rp.P) > kRingReduceLds) return rp;
  // HLL (register, rank) computed by the scatter's flushers (group.ring_hll): a column only HLL aggregations read,
  // over an affine INT / LONG dictionary (identical on every segment: plan_group's condition) with every value in
  // [0, 2^32) (the reduce's lo32 test), leaves the block as register << 5 | rank (13 bits) in its field (at least 13
  // bits wide) instead of its dictId, so the reduce does no hashing
  rp.hll_form.assign(na, 0);
  for (int a = 0; a < na && e.group_ring_hll; a++) {
    if (gx.acc_kind[a] != 4) continue;
    const std::string c = agg_column(q.aggregations[a]);
    bool only_hll = true;
    for (int b = 0; b < na; b++)
      if (gx.acc_kind[b] != 5 && gx.acc_kind[b] != 4 && agg_column(q.aggregations[b]) == c) only_hll = false;
    const ColumnData &cd = *segs[0]->column(c);
    if (!only_hll || !cd.affine || !e.use_affine || (cd.data_type != PINOT_INT && cd.data_type != PINOT_LONG) ||
        cd.bits > kGroupLwMaxBits)
      continue;
    const long long top = cd.affine_base + cd.affine_step * (long long)((1ull << cd.bits) - 1ull);
    const bool lo32 = cd.affine_base >= 0 && cd.affine_step >= 0 && cd.bits < 32 && top < (1ll << 32);
    if (lo32) {
      rp.hll_form[a] = 1;
      break;  // one such column per query (RingArgs.hll)
    }
  }
  // record layout: [s bits local key | one field per distinct aggregated column]
  rp.field_shift.assign(na, 0);
  std::map<std::string, int> col_field;
  int bits = s;
  for (int a = 0; a < na; a++) {
    if (gx.acc_kind[a] == 5) continue;
    const std::string c = agg_column(q.aggregations[a]);
    auto it = col_field.find(c);
    if (it == col_field.end()) {
      it = col_field.emplace(c, bits).first;
      bits += rp.hll_form[a] ? std::max(kRingHllFieldBits, segs[0]->column(c)->bits) : segs[0]->column(c)->bits;
    }
    rp.field_shift[a] = it->second;
  }
  if (bits > 53) return rp;
  rp.rec_bytes = bits <= 48 && e.group_ring_rec6 ? 6 : 8;
  // regions: every doc of the largest block matching, keys spread evenly (+ slack; beyond it the counted plan answers)
  const int64_t max_docs = (total_chunks + (int64_t)nblk - 1) / (int64_t)nblk * 4096;
  const uint32_t cap = ring_region_records((uint64_t)max_docs, K, ks.G, UINT32_MAX);
  if (cap > (1u << 20)) return rp;
  rp.cap = cap;
  // reduce LDS: accumulators (nibble HLL [K][128 B], 8-B others), counts u32 [K], hist row, exception list
  rp.lds_off.assign(na, 0);
  size_t off = 0;
  for (int a = 0; a < na; a++) {
    if (gx.acc_kind[a] == 5) continue;
    rp.lds_off[a] = (int)off;
    off += ((size_t)K * (gx.acc_kind[a] == 4 ? 128 : 8) + 15) / 16 * 16;
  }
  rp.cnt_off = (int)off;
  off += (size_t)K * 4;
  rp.hist_off = (int)off;
  off += (nblk * 4 + 15) / 16 * 16;
  rp.exc_off = (int)off;
  off += (4 + (size_t)ring_reduce_exceptions()) * 4;
  if (off > kRingReduceLds) return rp;
  rp.lds_bytes = (int)off;
  rp.shift = s;
  rp.nblk = (int64_t)nblk;
  rp.total_chunks = total_chunks;
  rp.on = true;
  return rp;
}

// num.groups.limit, per segment and across segments:
//   * DictionaryBasedGroupKeyGenerator (:79-126): a segment whose cardinality product exceeds
//     max.init.group.holder.capacity uses a map holder that gives group ids to the first
//     upper = min(product, limit) distinct keys in doc order (product > INT_MAX: limit); later keys get
//     INVALID_ID and are dropped (IntMapBasedHolder.getGroupId :293-302);
//   * CombineGroupByOperator (:61,147): a key enters the merged map only while it holds < 2 x limit keys.
// The reference merges segments on a thread pool, so which keys pass the inter-segment cap depends on timing;
// here it is the caller's segment order, ascending raw keys within a segment (the oracle's order).
AdmissionPlan plan_admission(const std::vector<SegmentData *> &segs, const pinot_query &q, const Engine &e, int64_t G) {
  AdmissionPlan ap;
  const int64_t limit = q.num_groups_limit > 0 ? q.num_groups_limit : e.num_groups_limit;
  const int64_t threshold = q.max_init_group_holder_capacity > 0 ? q.max_init_group_holder_capacity : 10000;
  int64_t possible = 0;
  for (auto *s : segs) {
    __int128 product = 1;
    for (int j = 0; j < q.num_group_by; j++) product *= s->column(q.group_by[j])->card;
    int64_t upper = INT64_MAX;
    if (product > threshold) upper = product <= INT32_MAX ? std::min<int64_t>((int64_t)product, limit) : limit;
    const int64_t reach = (int64_t)std::min<__int128>(std::min<__int128>(product, (__int128)s->num_docs), (__int128)G);
    if (upper < reach) ap.active = true;
    else upper = G;  // cannot bind: every present key
    ap.upper.push_back(upper);
    possible += std::min(upper, reach);
  }
  ap.cap = 2 * limit;
  if (std::min(possible, G) > ap.cap) ap.active = ap.cap_active = true;
  return ap;
}

// CombineGroupByOperator's inter-segment cap over the per-segment admitted bitmaps (host, [S][words] u32): keys
// enter in segment order, ascending within a segment, until `cap` distinct keys are in; every later new key is
// dropped from the segment that brings it.
void apply_inter_segment_cap(std::vector<uint32_t> &bm, size_t S, int64_t words, int64_t cap) {
  std::vector<uint32_t> merged(words, 0u);
  int64_t n = 0;
  bool full = false;
  for (size_t s = 0; s < S; s++) {
    uint32_t *b = bm.data() + s * words;
    for (int64_t w = 0; w < words; w++) {
      const uint32_t fresh = b[w] & ~merged[w];
      if (!fresh) continue;
      uint32_t kept = 0;
      if (!full) {
        const int64_t pc = __builtin_popcount(fresh);
        if (n + pc <= cap) {
          kept = fresh;
          n += pc;
        } else {
          uint32_t x = fresh;  // the lowest (cap - n) new keys of this word
          for (int64_t r = cap - n; r > 0; r--) {
            const uint32_t low = x & (0u - x);
            kept |= low;
            x ^= low;
          }
          n = cap;
        }
        if (n == cap) full = true;
      }
      merged[w] |= kept;
      b[w] = (b[w] & ~fresh) | kept;
    }
  }
}

// first_doc [S][G] (GB_FIRST / k_first_doc) -> admitted bitmaps [S][words] on the device, with the inter-segment
// cap applied on the host when it can bind. `buf` holds first docs, bitmaps and the sort scratch.
void build_admitted(Engine &e, const AdmissionPlan &ap, size_t S, int64_t G, const AdmissionBuffers &ab) {
  std::vector<long long> upper(ap.upper.begin(), ap.upper.end());
  launch_admission_bitmaps(ab.first_doc, (int)S, G, upper.data(), ab.bitmaps, ab.words, ab.scratch, ab.scratch_bytes,
                           e.stream);
  PINOT_HIP(hipGetLastError());
  if (!ap.cap_active) return;
  std::vector<uint32_t> bm(S * ab.words);
  PINOT_HIP(hipMemcpyAsync(bm.data(), ab.bitmaps, bm.size() * 4, hipMemcpyDeviceToHost, e.stream));
  wait_stream(e);
  apply_inter_segment_cap(bm, S, ab.words, ap.cap);
  e.host_arena.reserve(bm.size() * 4);  // pinned staging; the query arena is already on the device
  memcpy(e.host_arena.get(), bm.data(), bm.size() * 4);
  PINOT_HIP(hipMemcpyAsync(ab.bitmaps, e.host_arena.get(), bm.size() * 4, hipMemcpyHostToDevice, e.stream));
  wait_stream(e);  // host_arena is the staging of the next query's arena
}

AdmissionBuffers admission_buffers(Engine &e, size_t S, int64_t G) {
  AdmissionBuffers ab;
  ab.words = (G + 31) / 32 + 1;
  const size_t fd_b = ((size_t)S * G * 4 + 255) / 256 * 256, bm_b = ((size_t)S * ab.words * 4 + 255) / 256 * 256;
  ab.scratch_bytes = admission_scratch_bytes(G);
  const size_t need = fd_b + bm_b + ab.scratch_bytes;
  if (need > e.group_admit.size()) {
    size_t free_b = 0, total_b = 0;
    PINOT_HIP(hipMemGetInfo(&free_b, &total_b));
    require((double)need < 0.5 * (double)free_b, PINOT_ERR_UNSUPPORTED,
            "num.groups.limit admission state (first docs per segment and key) does not fit in HBM");
  }
  e.group_admit.reserve(need);
  ab.first_doc = e.group_admit.get<uint32_t>();
  ab.bitmaps = reinterpret_cast<uint32_t *>(e.group_admit.get<uint8_t>() + fd_b);
  ab.scratch = e.group_admit.get<uint8_t>() + fd_b + bm_b;
  return ab;
}

}  // namespace

// Fused group-by: ONE k_group_query launch (or COUNT / EMIT / reduce for the partitioned plan) over all
// segments, device compaction of the non-empty keys, device per-group outputs, one D2H of the arrays.
// Multi-GPU partial arrays in the partial layout: `po` = write them (pinot_gpu_group_by_partial, the kernels
// stop before compaction), `pin` = finalize from them (pinot_gpu_group_by_finalize, no kernels: the same
// device compaction / outputs / lazy HLL registers as a one-GPU group-by).
struct PartialOut {
  int64_t *counts;
  void *const *accs;
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

// extra(pinned) issues the caller's own small D2H reads into pinned[0, 4096) (read back after the wait).
unsigned long long compact_dense(Engine &e, const unsigned long long *counts, int64_t G, long long *&keys_dev,
                                 const std::function<void(uint8_t *)> &extra, size_t extra_bytes = 0) {
  const size_t cscr = compact_keys_scratch_bytes(G);
  e.group_final.reserve(G * 8 + 64 + cscr);
  keys_dev = e.group_final.get<long long>();
  auto *n_dev = reinterpret_cast<unsigned long long *>(e.group_final.get<uint8_t>() + G * 8);
  launch_compact_keys_ordered(G, counts, keys_dev, n_dev, e.group_final.get<uint8_t>() + G * 8 + 64, cscr, e.stream);
  PINOT_HIP(hipGetLastError());
  e.d2h_small.reserve(64 + std::max<size_t>(extra_bytes, 4096));
  auto *hn = e.d2h_small.get<unsigned long long>();
  PINOT_HIP(hipMemcpyAsync(hn, n_dev, 8, hipMemcpyDeviceToHost, e.stream));
  if (extra) extra(e.d2h_small.get<uint8_t>() + 64);
  wait_stream(e);
  return *hn;
}

// Device half of build_dense_result: the final arrays of the n non-empty groups in the host result's layout
// (k_group_final) and the HLL registers gathered per group, all on the device (no sync).
// compact_ok: the keys are every non-empty key of [0, G) (the compact read-back lists them from a bitmap of the
// counts); false for a subset (the device trim's kept union) or when only device arrays are wanted.
DenseOut dense_outputs(Engine &e, const DenseGroups &d, const long long *keys_dev, unsigned long long n,
                       bool gather_hll = true, bool compact_ok = true, bool serialize_hll = false) {
  const pinot_query &q = *d.q;
  const GroupAccs &ga = *d.ga, &gx = *d.gx;
  const std::vector<int> &alias = *d.alias;
  const int na = q.num_aggregations;
  DenseOut o;
  o.n = n;
  o.kind = ga.acc_kind;
  o.derive.assign(na, -1);  // -2: values from the HLL cardinalities; >= 0: copy of that function's values
  for (int i = 0; i < na; i++) {
    if (ga.acc_kind[i] == 4) o.derive[i] = -2;
    else if (alias[i] >= 0 && ga.acc_kind[i] == ga.acc_kind[alias[i]]) o.derive[i] = alias[i];
  }
  o.hll_off.assign(na, 0);
  o.values.assign(na, nullptr);
  o.cards.assign(na, nullptr);
  if (!n) return o;
  if (!e.hll_linear.size()) {
    e.hll_linear.alloc(257 * sizeof(double));
    PINOT_HIP(hipMemcpy(e.hll_linear.get(), hll_linear_counting_table(), 257 * sizeof(double), hipMemcpyHostToDevice));
  }
  int n_card = 0, n_hll = 0;
  for (int i = 0; i < na; i++) {
    n_card += ga.acc_kind[i] == 4;
    n_hll += gx.acc_kind[i] == 4;
  }
  const size_t n8 = n * 8;
  // compact read-back: keys as a bitmap over [0, G), counts / cardinalities as u32 (half the PCIe bytes)
  const bool compact = compact_ok && e.compact_d2h && !d.hashed && n >= (1u << 16) && d.ks->G > 0;
  const size_t key_words = compact ? (size_t)((d.ks->G + 63) / 64) : 0;
  const size_t compact_bytes = compact ? key_words * 8 + n * 4 * (1 + n_card) + 64 : 0;
  // a subset's keys also as per-column global ids (no division in the DataTable writer), after the arrays
  const int nc = q.num_group_by;
  const bool digits = serialize_hll && !d.hashed && nc <= kDigitsMaxCols && (size_t)d.ks->gcard.size() == (size_t)nc;
  const size_t digit_bytes = digits ? n * nc * 4 + 16 : 0;
  e.group_out.reserve(n8 * (2 + na + n_card) + 256 + compact_bytes + digit_bytes);
  GroupFinalArgs f{};
  f.n = na;
  f.out_keys = e.group_out.get<long long>();
  f.out_counts = f.out_keys + n;
  f.key_base = d.key_base;
  f.alpha_mm = hll_alpha_mm();
  f.linear = e.hll_linear.get<double>();
  {
    double *v = reinterpret_cast<double *>(f.out_counts + n);
    long long *c = reinterpret_cast<long long *>(v + n * na);
    for (int i = 0; i < na; i++) {
      const int src = alias[i] >= 0 ? alias[i] : i;  // the accumulator this aggregation reads
      f.kind[i] = ga.acc_kind[i];
      f.acc[i] = d.accs[src];
      if (ga.acc_kind[i] == 4 && (size_t)src < d.hll_sum.size() && d.hll_sum[src]) {
        f.kind[i] = 9;
        f.acc[i] = d.hll_sum[src];
      }
      f.out_values[i] = v + n * i;
      if (ga.acc_kind[i] == 4) {
        f.out_card[i] = c;
        c += n;
      }
    }
  }
  o.keys = f.out_keys;
  o.counts = f.out_counts;
  o.values.assign(f.out_values, f.out_values + na);
  o.cards.assign(f.out_card, f.out_card + na);
  o.cards32.assign(na, nullptr);
  if (compact) {
    uint8_t *cb = reinterpret_cast<uint8_t *>(f.out_counts + n) + n8 * (na + n_card);
    cb = reinterpret_cast<uint8_t *>(((uintptr_t)cb + 15) & ~(uintptr_t)15);
    uint64_t *kb = reinterpret_cast<uint64_t *>(cb);
    f.overflow = reinterpret_cast<unsigned int *>(kb + key_words);
    f.out_counts32 = f.overflow + 4;
    unsigned int *c32 = f.out_counts32 + n;
    for (int i = 0; i < na; i++)
      if (ga.acc_kind[i] == 4) {
        f.out_card32[i] = c32;
        c32 += n;
      }
    PINOT_HIP(hipMemsetAsync(f.overflow, 0, 4, e.stream));
    launch_key_bitmap(d.counts, d.ks->G, kb, e.stream);
    o.key_bits = kb;
    o.key_words = (int64_t)key_words;
    o.key_base = d.key_base;
    o.counts32 = f.out_counts32;
    o.cards32.assign(f.out_card32, f.out_card32 + na);
    o.overflow = f.overflow;
  }
  launch_group_final(d.counts, keys_dev, (long long)n, f, e.stream);
  PINOT_HIP(hipGetLastError());
  if (digits) {
    KeyDigits kd{};
    kd.nc = nc;
    for (int j = 0; j < nc; j++) kd.card[j] = d.ks->gcard[j];
    o.key_ids = reinterpret_cast<int32_t *>(reinterpret_cast<uint8_t *>(f.out_counts + n) + n8 * (na + n_card));
    launch_key_digits(keys_dev, (long long)n, d.key_base, kd, o.key_ids, e.stream);
    PINOT_HIP(hipGetLastError());
  }
  if (n_hll && gather_hll) {  // registers stay on the device until asked for; buffers are recycled once released
    const size_t need = (size_t)n_hll * n * 256 + 16;
    for (auto &b : e.hll_pool)
      if (b.use_count() == 1 && b->size() >= need) { o.hll = b; break; }
    if (!o.hll) {
      o.hll = std::make_shared<DeviceBuffer>(need + need / 4);
      if (e.hll_pool.size() < 4) e.hll_pool.push_back(o.hll);
    }
    int h = 0;
    for (int i = 0; i < na; i++)
      if (gx.acc_kind[i] == 4) {
        o.hll_off[i] = (size_t)h * n * 256;
        launch_gather_hll(static_cast<const uint8_t *>(d.accs[i]), keys_dev, (long long)n, o.hll->get<uint8_t>() + o.hll_off[i],
                          e.stream);
        h++;
      }
    for (int i = 0; i < na; i++)
      if (alias[i] >= 0 && ga.acc_kind[i] == 4) o.hll_off[i] = o.hll_off[alias[i]];
    if (serialize_hll) {  // HyperLogLog.getBytes of every listed group, for the DataTable (hll_serde.hip)
      const size_t need = (size_t)n_hll * n * 180 + 16;
      if (!e.hll_ser || e.hll_ser.use_count() > 1 || e.hll_ser->size() < need)
        e.hll_ser = std::make_shared<DeviceBuffer>(need + need / 4);
      o.hll_ser = e.hll_ser;
      o.hll_ser_off.assign(na, 0);
      int s = 0;
      for (int i = 0; i < na; i++)
        if (gx.acc_kind[i] == 4) {
          o.hll_ser_off[i] = (size_t)s * n * 180;
          launch_hll_getbytes(o.hll->get<uint8_t>() + o.hll_off[i], (long long)n, o.hll_ser->get<uint8_t>() + o.hll_ser_off[i],
                              e.stream);
          s++;
        }
      for (int i = 0; i < na; i++)
        if (alias[i] >= 0 && ga.acc_kind[i] == 4) o.hll_ser_off[i] = o.hll_ser_off[alias[i]];
    }
    PINOT_HIP(hipGetLastError());
  }
  return o;
}

// The compact read-back: the key bitmap, u32 counts / cardinalities and the values straight into the result arrays,
// then the keys listed and the u32 arrays widened over the host threads. False (nothing filled) when a count or a
// cardinality did not fit 32 bits: the caller then reads the 64-bit arrays.
bool compact_fetch(Engine &e, GroupByResult *res, const DenseOut &o, int na) {
  const unsigned long long n = o.n;
  const size_t n8 = n * 8;
  e.compact_host.reserve((size_t)o.key_words * 8 + n * 4 * (1 + na) + 64);
  uint8_t *h = e.compact_host.get<uint8_t>();
  uint64_t *hbits = reinterpret_cast<uint64_t *>(h);
  unsigned int *hover = reinterpret_cast<unsigned int *>(hbits + o.key_words);
  unsigned int *hc32 = hover + 4;
  std::vector<unsigned int *> hcard(na, nullptr);
  unsigned int *p = hc32 + n;
  for (int i = 0; i < na; i++)
    if (o.cards32[i]) {
      hcard[i] = p;
      p += n;
    }
  PINOT_HIP(hipMemcpyAsync(hbits, o.key_bits, (size_t)o.key_words * 8, hipMemcpyDeviceToHost, e.stream));
  PINOT_HIP(hipMemcpyAsync(hover, o.overflow, 4, hipMemcpyDeviceToHost, e.stream));
  PINOT_HIP(hipMemcpyAsync(hc32, o.counts32, n * 4, hipMemcpyDeviceToHost, e.stream));
  for (int i = 0; i < na; i++) {
    if (o.derive[i] == -1) PINOT_HIP(hipMemcpyAsync(res->values[i].data(), o.values[i], n8, hipMemcpyDeviceToHost, e.stream));
    if (hcard[i]) PINOT_HIP(hipMemcpyAsync(hcard[i], o.cards32[i], n * 4, hipMemcpyDeviceToHost, e.stream));
  }
  wait_stream(e);
  if (*hover) return false;
  const size_t nt = host_threads();
  const size_t W = (size_t)o.key_words;
  std::vector<size_t> base(nt + 1, 0);
  parallel_tasks(nt, [&](size_t t) {  // set bits per word range
    size_t c = 0;
    for (size_t w = W * t / nt; w < W * (t + 1) / nt; w++) c += __builtin_popcountll(hbits[w]);
    base[t + 1] = c;
  });
  for (size_t t = 0; t < nt; t++) base[t + 1] += base[t];
  require(base[nt] == n, PINOT_ERR_DEVICE, "key bitmap disagrees with the compacted key count");
  int64_t *keys = res->raw_keys.data();
  parallel_tasks(nt, [&](size_t t) {
    size_t i = base[t];
    for (size_t w = W * t / nt; w < W * (t + 1) / nt; w++)
      for (uint64_t x = hbits[w]; x; x &= x - 1) keys[i++] = (int64_t)(w * 64 + __builtin_ctzll(x)) + o.key_base;
    const size_t lo = n * t / nt, hi = n * (t + 1) / nt;
    int64_t *cv = res->counts[0].data();
    for (size_t g = lo; g < hi; g++) cv[g] = hc32[g];
    for (int f = 0; f < na; f++) {
      if (!hcard[f]) continue;
      int64_t *card = res->hll_card[f].data();
      for (size_t g = lo; g < hi; g++) card[g] = hcard[f][g];
    }
    for (int f = 0; f < na; f++) {
      if (o.derive[f] == -1) continue;
      double *v = res->values[f].data();
      if (o.derive[f] == -2) {
        const int64_t *c = res->hll_card[f].data();
        for (size_t g = lo; g < hi; g++) v[g] = (double)c[g];
      } else {
        memcpy(v + lo, res->values[o.derive[f]].data() + lo, (hi - lo) * 8);
      }
    }
  });
  return true;
}

// Host half: one D2H per array straight into the (pinned, pooled) result arrays — only what the host cannot
// derive: keys, counts, each primary's values, cardinalities; an alias's values (AVG(x) beside SUM(x)) and an HLL
// function's values (= its cardinalities) are filled on the host. HLL registers stay on the device (one part).
std::unique_ptr<GroupByResult> dense_fetch(Engine &e, const pinot_query &q, const std::vector<int64_t> &gcard,
                                           const std::vector<std::vector<std::string>> &gvalues, const DenseOut &o,
                                           const GroupArgs *hashed) {
  const int na = q.num_aggregations;
  const unsigned long long n = o.n;
  auto res = std::make_unique<GroupByResult>();
  res->num_columns = q.num_group_by;
  res->functions.resize(na);
  for (int i = 0; i < na; i++) res->functions[i] = q.aggregations[i].function;
  res->counts.assign(na, {});
  res->values.assign(na, {});
  res->hll.assign(na, {});
  res->hll_card.assign(na, {});
  res->gvalues = gvalues;
  res->gcard = gcard;
  res->counts_shared = true;  // every aggregation counts the same docs per group
  if (!n) return res;
  const auto tb0 = std::chrono::steady_clock::now();
  if (o.hll) {
    HllPart part;
    part.device = e.device;
    part.group_begin = 0;
    part.num_groups = (int64_t)n;
    part.off = o.hll_off;
    part.buf = o.hll;
    res->hll_parts.push_back(std::move(part));
  }
  DeviceBuffer ids;
  if (hashed) {  // group ordinals are hash slots: fetch each group's global-id tuple
    ids.alloc(n * q.num_group_by * 4 + 16);
    launch_hash_tuples(*hashed, o.keys, (long long)n, ids.get<int32_t>(), e.stream);
    PINOT_HIP(hipGetLastError());
    res->key_ids.resize(n * q.num_group_by);
    PINOT_HIP(hipMemcpyAsync(res->key_ids.data(), ids.get(), n * q.num_group_by * 4, hipMemcpyDeviceToHost, e.stream));
  }
  // the result arrays (pinned, recycled from released results where possible) are sized while the device works
  if (n >= kPoolMinElems) {
    ResultPool &rp = result_pool();
    std::lock_guard<std::mutex> lk(rp.mu);
    res->raw_keys = take_pooled(rp, rp.i64, n);
    res->counts[0] = take_pooled(rp, rp.i64, n);
    for (int i = 0; i < na; i++) {
      res->values[i] = take_pooled(rp, rp.f64, n);
      if (o.kind[i] == 4) res->hll_card[i] = take_pooled(rp, rp.i64, n);
    }
  }
  res->raw_keys.resize(n);
  res->counts[0].resize(n);
  for (int i = 0; i < na; i++) {
    res->values[i].resize(n);
    if (o.kind[i] == 4) res->hll_card[i].resize(n);
  }
  if (o.hll_ser) {  // the serialized HLL rows, in the same stream ahead of the arrays' copies and their wait
    res->hll_bytes.assign(na, {});
    for (int i = 0; i < na; i++)
      if (o.kind[i] == 4) {
        res->hll_bytes[i].resize(n * 180);
        PINOT_HIP(hipMemcpyAsync(res->hll_bytes[i].data(), o.hll_ser->get<uint8_t>() + o.hll_ser_off[i], n * 180,
                                 hipMemcpyDeviceToHost, e.stream));
      }
  }
  const auto tb1 = std::chrono::steady_clock::now();
  const size_t n8 = n * 8;
  if (o.key_bits && compact_fetch(e, res.get(), o, na)) {
    if (e.host_phases)
      fprintf(stderr, "[pinot_gpu] group-by outputs (us): sizing %.1f, compact D2H + widen %.1f\n",
              std::chrono::duration<double, std::micro>(tb1 - tb0).count(),
              std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tb1).count());
    return res;
  }
  // the arrays' D2H copies fanned out over d2h.streams streams (each its own copy queue), all after the final-array
  // kernels: one queue alone leaves PCIe half idle on a 32 MB result
  std::vector<std::pair<void *, const void *>> copies;
  copies.emplace_back(res->raw_keys.data(), o.keys);
  copies.emplace_back(res->counts[0].data(), o.counts);
  for (int i = 0; i < na; i++) {
    if (o.derive[i] == -1) copies.emplace_back(res->values[i].data(), o.values[i]);
    if (o.kind[i] == 4) copies.emplace_back(res->hll_card[i].data(), o.cards[i]);
  }
  const size_t id_bytes = o.key_ids ? n * (size_t)q.num_group_by * 4 : 0;
  if (o.key_ids) res->key_ids.resize(n * (size_t)q.num_group_by);
  if (n8 < (1u << 20)) {  // small arrays are pageable (HostVec): one copy of the arrays' device span into pinned
                          // staging, then host copies (a pageable D2H target is a staged, synchronous copy apiece)
    const uint8_t *lo = static_cast<const uint8_t *>(copies[0].second), *hi = lo;
    for (auto &c : copies) {
      lo = std::min(lo, static_cast<const uint8_t *>(c.second));
      hi = std::max(hi, static_cast<const uint8_t *>(c.second) + n8);
    }
    if (o.key_ids) {  // right after the arrays (dense_outputs)
      lo = std::min(lo, reinterpret_cast<const uint8_t *>(o.key_ids));
      hi = std::max(hi, reinterpret_cast<const uint8_t *>(o.key_ids) + id_bytes);
    }
    e.group_host.reserve((size_t)(hi - lo));
    PINOT_HIP(hipMemcpyAsync(e.group_host.get(), lo, (size_t)(hi - lo), hipMemcpyDeviceToHost, e.stream));
    wait_stream(e);
    for (auto &c : copies)
      memcpy(c.first, e.group_host.get<uint8_t>() + (static_cast<const uint8_t *>(c.second) - lo), n8);
    if (o.key_ids)
      memcpy(res->key_ids.data(), e.group_host.get<uint8_t>() + (reinterpret_cast<const uint8_t *>(o.key_ids) - lo), id_bytes);
    copies.clear();
  }
  const int ns = (n8 >= (1u << 20)) ? std::min<int>(e.d2h_streams, (int)copies.size()) : 1;
  if (ns > 1) {
    while ((int)e.copy_streams.size() < ns - 1) {
      hipStream_t cs;
      PINOT_HIP(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
      e.copy_streams.push_back(cs);
    }
    if (!e.ev_copy) PINOT_HIP(hipEventCreateWithFlags(&e.ev_copy, hipEventDisableTiming));
    PINOT_HIP(hipEventRecord(e.ev_copy, e.stream));
    for (int k = 0; k < ns - 1; k++) PINOT_HIP(hipStreamWaitEvent(e.copy_streams[k], e.ev_copy, 0));
  }
  for (size_t j = 0; j < copies.size(); j++) {
    const int k = (int)(j % (size_t)ns);
    hipStream_t st = k == 0 ? e.stream : e.copy_streams[k - 1];
    PINOT_HIP(hipMemcpyAsync(copies[j].first, copies[j].second, n8, hipMemcpyDeviceToHost, st));
  }
  if (o.key_ids && !copies.empty())
    PINOT_HIP(hipMemcpyAsync(res->key_ids.data(), o.key_ids, id_bytes, hipMemcpyDeviceToHost, e.stream));
  for (int k = 0; k < ns - 1; k++) PINOT_HIP(hipStreamSynchronize(e.copy_streams[k]));
  wait_stream(e);
  bool any_derived = false;
  for (int i = 0; i < na; i++) any_derived = any_derived || o.derive[i] != -1;
  if (any_derived) {
    const size_t nt = n >= (1u << 16) ? host_threads() : 1;
    auto fill = [&](size_t t) {
      const size_t lo = n * t / nt, hi = n * (t + 1) / nt;
      for (int i = 0; i < na; i++) {
        if (o.derive[i] == -1) continue;
        double *v = res->values[i].data();
        if (o.derive[i] == -2) {
          const int64_t *c = res->hll_card[i].data();
          for (size_t g = lo; g < hi; g++) v[g] = (double)c[g];
        } else {
          memcpy(v + lo, res->values[o.derive[i]].data() + lo, (hi - lo) * 8);
        }
      }
    };
    if (nt > 1) parallel_tasks(nt, fill);
    else fill(0);
  }
  if (e.host_phases)
    fprintf(stderr, "[pinot_gpu] group-by outputs (us): sizing %.1f, D2H wait %.1f\n",
            std::chrono::duration<double, std::micro>(tb1 - tb0).count(),
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tb1).count());
  return res;
}

std::unique_ptr<GroupByResult> build_dense_result(Engine &e, const DenseGroups &d, const long long *keys_dev,
                                                  unsigned long long n, bool subset = false) {
  const DenseOut o = dense_outputs(e, d, keys_dev, n, true, !subset, subset);
  return dense_fetch(e, *d.q, d.ks->gcard, d.ks->gvalues, o, d.hashed);
}

// CombineGroupByOperator's trim (AggregationGroupByTrimmingService.trimIntermediateResultsMap :71-116) on the device,
// before anything leaves it: above 4 x trimSize groups (trimSize = max(5 * TOP, 5000)) every function keeps its
// trimSize best groups (getSorter :160-176: MIN ascending, the others descending; AVG by sum / count, HLL by
// cardinality; ties in ascending raw key order); the result holds the union of the kept groups and each function's
// list. Returns the union's keys (device) and sets n to its size; `kept` stays empty when nothing is trimmed.
// min_groups >= 0: trim above that many groups instead of 4 x trimSize (a server rank's pre-trim of its own key range,
// server.cpp); flags_out: each kept group's bit mask of the functions that keep it.
const long long *device_trim(Engine &e, const DenseGroups &d, const long long *keys_dev, unsigned long long &n,
                             int32_t top_n, std::vector<std::vector<int64_t>> &kept, int64_t min_groups = -1,
                             std::vector<uint32_t> *flags_out = nullptr) {
  const int64_t T = std::max<int64_t>(5 * (int64_t)top_n, 5000);
  if ((int64_t)n <= (min_groups >= 0 ? min_groups : 4 * T) || d.hashed) return keys_dev;
  const pinot_query &q = *d.q;
  const int na = q.num_aggregations;
  const DenseOut o = dense_outputs(e, d, keys_dev, n, false, false);  // comparable values of every group, no registers
  const size_t scr = std::max(trim_scratch_bytes((long long)n), trim_radix_scratch_bytes((long long)n, na));
  const size_t a8 = ((size_t)n * 8 + 255) / 256 * 256, a4 = ((size_t)n * 4 + 255) / 256 * 256;
  e.group_trim.reserve(a8 + 2 * a4 + 256 + scr);
  uint8_t *p = e.group_trim.get<uint8_t>();
  auto *ukeys = reinterpret_cast<long long *>(p);
  auto *flags = reinterpret_cast<uint32_t *>(p + a8);
  auto *uflags = reinterpret_cast<uint32_t *>(p + a8 + a4);
  auto *n_dev = reinterpret_cast<unsigned long long *>(p + a8 + 2 * a4);
  void *tmp = p + a8 + 2 * a4 + 256;
  require(na <= kTrimMaxFns, PINOT_ERR_DEVICE, "trim over more functions than the selection holds");
  TrimFn fns[kTrimMaxFns];
  for (int i = 0; i < na; i++) {
    const int f = sv_function(q.aggregations[i].function);
    fns[i] = TrimFn{o.values[i], f == PINOT_AGG_AVG, f == PINOT_AGG_MIN};
  }
  launch_trim_radix(fns, na, o.counts, (long long)n, T, flags, tmp, scr, e.stream);  // every function's kept groups
  launch_trim_union(flags, keys_dev, (long long)n, ukeys, uflags, n_dev, tmp, scr, e.stream);
  PINOT_HIP(hipGetLastError());
  // the union holds at most na x T groups: its count and flags in one round trip
  const size_t max_u = std::min<size_t>((size_t)n, (size_t)na * (size_t)T);
  e.d2h_small.reserve(64 + max_u * 4);
  auto *pin = e.d2h_small.get<uint8_t>();
  PINOT_HIP(hipMemcpyAsync(pin, n_dev, 8, hipMemcpyDeviceToHost, e.stream));
  PINOT_HIP(hipMemcpyAsync(pin + 64, uflags, max_u * 4, hipMemcpyDeviceToHost, e.stream));
  wait_stream(e);
  const unsigned long long nu = *reinterpret_cast<const unsigned long long *>(pin);
  const uint32_t *hf = reinterpret_cast<const uint32_t *>(pin + 64);
  require(nu <= max_u, PINOT_ERR_DEVICE, "trim union larger than its functions' lists");
  kept.assign(na, {});
  for (int i = 0; i < na; i++) kept[i].reserve((size_t)T);
  for (unsigned long long g = 0; g < nu; g++)
    for (uint32_t x = hf[g]; x; x &= x - 1u) kept[__builtin_ctz(x)].push_back((int64_t)g);
  if (flags_out) flags_out->assign(hf, hf + nu);
  n = nu;
  return ukeys;
}

std::unique_ptr<GroupByResult> exec_group_by_fused(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q,
                                                   const KeySpace &ks_in, const GroupAccs &ga, pinot_exec_stats *stats,
                                                   int attempt = 0, const PartialOut *po = nullptr,
                                                   const PartialOut *pin = nullptr, bool allow_admission = false,
                                                   AdmissionIO *aio = nullptr) {
  const auto tg0 = std::chrono::steady_clock::now();
  const int na = q.num_aggregations;
  const size_t S = segs.size();
  KeySpace ks = ks_in;
  // aggregations repeating an earlier one's (accumulator kind, column) — SUM(x) and AVG(x) — share its
  // accumulator: the device program accumulates it once (kind 5 for the duplicate)
  std::vector<int> alias(na, -1);
  GroupAccs gx = ga;
  for (int a = 0; a < na; a++) {
    if (ga.acc_kind[a] == 5) continue;
    for (int b = 0; b < a; b++)
      if (alias[b] < 0 && ga.acc_kind[b] == ga.acc_kind[a] &&
          agg_column(q.aggregations[b]) == agg_column(q.aggregations[a])) {
        alias[a] = b;
        gx.acc_kind[a] = 5;
        break;
      }
  }
  int64_t hcap = 0;
  if (ks.hashed) {  // slots: a power of two >= 2 x the docs that can match
    int64_t docs = 0;
    for (auto *sg : segs) docs += sg->num_docs;
    hcap = 1024;
    while (hcap < 2 * docs) hcap <<= 1;
    ks.G = hcap;
  }
  const GroupPlan gp = plan_group(segs, q, ks, gx, ks.hashed ? std::string("global") : e.group_mode, e.group_split,
                                    e.group_pshift);
  // num.groups.limit: per-segment first-appearance admission and the inter-segment cap (plan_admission)
  AdmissionPlan adm = pin ? AdmissionPlan{} : plan_admission(segs, q, e, ks.G);
  if (aio && !pin) {  // the server applies the inter-segment cap across ranks (AdmissionIO): every segment's keys
    adm.active = true;
    adm.cap_active = false;
  }
  require(!(po && adm.active && (!allow_admission || adm.cap_active)), PINOT_ERR_UNSUPPORTED,
          "multi-GPU partials with num.groups.limit admission: use the engine's own multi-device group-by");
  const AdmissionBuffers ab = adm.active ? admission_buffers(e, S, ks.G) : AdmissionBuffers{};
  Arena ar;
  std::unique_ptr<FilterTreeInput> tree;
  if (q.num_filter_nodes > 0) tree = std::make_unique<FilterTreeInput>(decode_filter(q.num_filter_nodes, q.filter));
  std::vector<SegPlan> plans(S);
  for (size_t si = 0; si < S; si++) {
    plans[si].seg = segs[si];
    Compiler(e, plans[si], ar).run_fused(tree.get(), kGroupMaxFusedLeafBits, kMaxFusedStackGroup);
  }
  e.last_pre_segments = 0;
  for (auto &p : plans) e.last_pre_segments += p.has_pre && !p.empty;
  // chunk windows (a single sorted leaf bounds the chunks a segment's program visits), concatenated: the ring plan's
  // blocks split the global chunk list evenly
  std::vector<std::pair<int64_t, int64_t>> windows(S);
  std::vector<int64_t> cstart(S + 1, 0);
  for (size_t si = 0; si < S; si++) {
    windows[si] = chunk_window(plans[si], ar);
    const int64_t nch = plans[si].empty ? 0 : (plans[si].seg->nwords() + 63) / 64;
    const int64_t n = std::max<int64_t>(0, std::min(nch, windows[si].second) - windows[si].first);
    cstart[si + 1] = cstart[si] + n;
  }
  RingPlan rp;
  if (e.group_ring && gp.mode == GB_EMIT && !ks.hashed && !adm.active && !pin && e.group_prefetch &&
      e.group_lw == 2 && e.group_bucket && e.group_pshift < 0)
    rp = plan_ring(e, segs, q, ks, gx, cstart[S]);
  // a ring region overflowed (keys skewed beyond the regions' slack) or a bound tripped: the counted plan answers
  auto ring_fallback = [&]() {
    e.ring_fallbacks++;
    struct Restore {
      Engine &e;
      bool v;
      ~Restore() { e.group_ring = v; }
    } restore{e, e.group_ring};
    e.group_ring = false;
    return exec_group_by_fused(e, segs, q, ks_in, ga, stats, attempt, po, pin, allow_admission, aio);
  };
  const auto tga = std::chrono::steady_clock::now();
  // remaps (dictId -> global id) travel in the arena
  std::vector<std::vector<size_t>> remap_off(S, std::vector<size_t>(q.num_group_by, SIZE_MAX));
  for (size_t si = 0; si < S; si++)
    for (int j = 0; j < q.num_group_by; j++)
      if (!ks.remap[si][j].empty()) remap_off[si][j] = ar.add(ks.remap[si][j].data(), ks.remap[si][j].size() * 4);
  size_t n_leaves = 0;
  for (auto &p : plans) n_leaves += p.fused_leaves.size();
  const size_t tab_bytes = (S + 1) * 8 + 32 + S * sizeof(GroupSegment) + n_leaves * sizeof(FusedStep) +
                           S * q.num_group_by * sizeof(GroupColDev) + S * na * sizeof(GroupAggDev) + 512;
  QueryScratch qs = prepare_scratch(e, plans, ar, true, tab_bytes);

  const auto tgb = std::chrono::steady_clock::now();
  // dense accumulators: counts u64 [G], then one array per aggregation (HLL: u8 [G][256])
  std::vector<size_t> acc_bytes(na, 0);
  size_t per_key = 8;
  for (int a = 0; a < na; a++) {
    acc_bytes[a] = gx.acc_kind[a] == 5 ? 0 : gx.acc_kind[a] == 4 ? 256 : 8;
    per_key += acc_bytes[a] + (gx.acc_kind[a] == 4 ? 8 : 0);  // HLL: + the ring reduce's packed sums u64 [G]
  }
  const size_t head = 256 + (S * 8 + 255) / 256 * 256;  // matched [S] + verify flag, 256-B aligned arrays after
  const size_t scratch_b = ks.G * per_key + head + 256 * (size_t)(na + 1);
  if (scratch_b > e.group_scratch.size()) {  // growing: check the free HBM first (hipMemGetInfo is a syscall)
    size_t free_b = 0, total_b = 0;
    PINOT_HIP(hipMemGetInfo(&free_b, &total_b));
    require((double)ks.G * per_key < 0.5 * (double)free_b, PINOT_ERR_UNSUPPORTED, "dense group-by accumulators do not fit in HBM");
  }
  e.group_scratch.reserve(scratch_b);
  uint8_t *base = e.group_scratch.get<uint8_t>();
  auto *matched = reinterpret_cast<unsigned long long *>(base);
  auto *counts = reinterpret_cast<unsigned long long *>(base + head);
  std::vector<void *> accs(na, nullptr);
  {
    uint8_t *p = reinterpret_cast<uint8_t *>(counts) + (ks.G * 8 + 255) / 256 * 256;
    for (int a = 0; a < na; a++) {
      if (!acc_bytes[a]) continue;
      accs[a] = p;
      p += (ks.G * (acc_bytes[a] + (gx.acc_kind[a] == 4 ? 8 : 0)) + 255) / 256 * 256;
    }
    for (int a = 0; a < na; a++)
      if (alias[a] >= 0) accs[a] = accs[alias[a]];
  }
  if (pin) {  // merged partials: u64 counts, 8-byte accumulators and u8 HLL registers, as the fused sinks write them
    counts = reinterpret_cast<unsigned long long *>(pin->counts);
    for (int a = 0; a < na; a++) accs[a] = pin->accs[a];
  }
  if (po) {  // partials: the sinks write the caller's dense arrays directly (an alias's array is copied after)
    counts = reinterpret_cast<unsigned long long *>(po->counts);
    for (int a = 0; a < na; a++)
      if (acc_bytes[a]) accs[a] = po->accs[a];
    for (int a = 0; a < na; a++)
      if (alias[a] >= 0) accs[a] = accs[alias[a]];
  }

  const auto tgc = std::chrono::steady_clock::now();
  // device program
  std::vector<GroupSegment> gsegs(S);
  std::vector<FusedStep> leaves;
  std::vector<GroupColDev> gcols;
  std::vector<GroupAggDev> gaggs;
  int max_leaf_bits = 1;
  for (size_t si = 0; si < S; si++) {
    SegPlan &p = plans[si];
    SegmentData &s = *p.seg;
    GroupSegment &g = gsegs[si];
    g.pre = p.has_pre ? qs.bitsets + (int64_t)si * qs.slots * qs.stride : nullptr;
    g.nwords = p.empty ? 0 : s.nwords();
    g.num_docs = s.num_docs;
    g.first_leaf = (int32_t)leaves.size();
    g.n_leaves = (int32_t)p.fused_leaves.size();
    g.first_gcol = (int32_t)gcols.size();
    g.first_agg = (int32_t)gaggs.size();
    g.admitted = adm.active ? ab.bitmaps + si * ab.words : nullptr;
    std::tie(g.ch_begin, g.ch_end) = windows[si];
    for (const FilterStep &l : p.fused_leaves) {
      leaves.push_back(fused_leaf_step(s, l, qs.arena));
      max_leaf_bits = std::max(max_leaf_bits, leaves.back().bits);
    }
    long long stride = 1;
    for (int j = 0; j < q.num_group_by; j++) {
      const ColumnData &c = *s.column(q.group_by[j]);
      GroupColDev gc{};
      gc.fwd = c.fwd.get<uint8_t>();
      gc.remap = remap_off[si][j] == SIZE_MAX ? nullptr : reinterpret_cast<const int32_t *>(qs.arena + remap_off[si][j]);
      gc.stride = stride;
      gc.bits = c.bits;
      gcols.push_back(gc);
      stride *= ks.gcard[j];
    }
    for (int a = 0; a < na; a++) {
      GroupAggDev ag{};
      ag.acc_kind = gx.acc_kind[a];
      ag.acc = accs[a];
      if (ag.acc_kind != 5) {
        ColumnData &c = *s.column(agg_column(q.aggregations[a]));
        ag.fwd = c.fwd.get<uint8_t>();
        ag.dict = c.dict_dev.get();
        ag.bits = c.bits;
        ag.value_kind = c.value_kind();
        if (ag.acc_kind == 4) {
          ensure_hll_lut(e, c);
          ag.hll_lut = c.hll_lut.get<uint16_t>();
        }
        if (c.affine && e.use_affine && (c.data_type == PINOT_INT || c.data_type == PINOT_LONG)) {
          ag.affine = 1;
          ag.affine_base = c.affine_base;
          ag.affine_step = c.affine_step;
        }
      }
      ag.field_shift = rp.on ? rp.field_shift[a] : gp.field_shift[a];
      ag.lds_off = gp.lds_off[a];
      gaggs.push_back(ag);
    }
  }
  const size_t off_segs = ar.add(gsegs.data(), gsegs.size() * sizeof(GroupSegment));
  const size_t off_leaves = ar.add(leaves.data(), leaves.size() * sizeof(FusedStep));
  const size_t off_gcols = ar.add(gcols.data(), gcols.size() * sizeof(GroupColDev));
  const size_t off_aggs = ar.add(gaggs.data(), gaggs.size() * sizeof(GroupAggDev));
  const size_t off_cstart = ar.add(cstart.data(), cstart.size() * 8);
  require(ar.bytes.size() <= e.small.size(), PINOT_ERR_DEVICE, "query arena overflow");

  GroupArgs a{};
  a.segs = reinterpret_cast<const GroupSegment *>(qs.arena + off_segs);
  a.leaves = reinterpret_cast<const FusedStep *>(qs.arena + off_leaves);
  a.gcols = reinterpret_cast<const GroupColDev *>(qs.arena + off_gcols);
  a.aggs = reinterpret_cast<const GroupAggDev *>(qs.arena + off_aggs);
  a.nsegs = (int32_t)S;
  a.n_gcols = q.num_group_by;
  a.n_aggs = na;
  a.stage_bytes = staged_chunk_bytes(max_leaf_bits);
  a.G = ks.G;
  a.counts = counts;
  a.matched = matched;
  a.lds_acc_bytes = gp.lds_acc_bytes;
  a.shift = gp.shift;
  a.P = (int32_t)gp.P;
  a.mode = gp.mode == GB_EMIT ? GB_COUNT : gp.mode;
  a.nt_store = e.group_nt_store;
  // the prefetched column list: GB_EMIT's record fields, or GB_LDS's lane-owns-quarter reads (group.lw=2)
  if ((gp.mode == GB_EMIT || (gp.mode == GB_LDS && e.group_lw == 2)) &&
      !ks.hashed && e.group_prefetch) {
    int nc = q.num_group_by;
    for (int i = 0; i < na && nc <= kGroupPfCols; i++)
      if (gx.acc_kind[i] != 5) {
        if (nc < kGroupPfCols) a.pf_agg[nc] = i;
        nc++;
      }
    a.pf_nc = nc <= kGroupPfCols ? nc : 0;
    // lane-owns-word reads: u32 keys, every read column within the decoder's widths
    bool lw = e.group_lw && a.pf_nc > 0 && ks.G <= (long long)UINT32_MAX;
    for (const GroupColDev &gc : gcols) lw = lw && gc.bits <= kGroupLwMaxBits;
    for (size_t i = 0; i < gaggs.size(); i++)
      if (gx.acc_kind[i % na] != 5) lw = lw && gaggs[i].bits <= kGroupLwMaxBits;
    a.lw = lw ? e.group_lw : 0;
  }
  unsigned long long *htable = nullptr, *reps = nullptr;
  if (ks.hashed) {
    e.group_hash.reserve((size_t)hcap * 16 + 256);
    htable = e.group_hash.get<unsigned long long>();
    reps = htable + hcap;
    a.hashed = 1;
    a.htable = htable;
    a.reps = reps;
    a.hcap = hcap;
    a.hseed = 0x5EEDF00Dull + 0x9E3779B97F4A7C15ull * (unsigned long long)attempt;
    a.verify_err = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(matched) + S * 8 + 16);
  }
  if (gp.mode == GB_LDS) a.emit_block = e.group_lds_block;  // block size of the lane-owns-quarter GB_LDS instance
  int64_t max_chunks = 1;  // chunks in the largest segment window
  for (const GroupSegment &g : gsegs) max_chunks = std::max<int64_t>(max_chunks, g.ch_end - g.ch_begin);
  const int64_t resident = (int64_t)group_query_blocks_per_cu(a) * e.num_cus;
  a.bps = (int)std::max<int64_t>(1, std::min<int64_t>(resident / (int64_t)S, (max_chunks + 15) / 16));
  const int64_t nblk = (int64_t)S * a.bps;
  // GB_LDS on the lane-owns-quarter path: the count packed into an affine dictId sum when both fields fit 64 bits
  // (a block's docs < 2^cbits; Σ dictId < 2^(bits + cbits))
  a.lds_pack = -1;
  if (gp.mode == GB_LDS && a.lw == 2 && a.pf_nc > 0 && !pin) {
    const int64_t blk_docs = ((max_chunks + 16 * a.bps - 1) / (16 * a.bps)) * 16 * 4096;
    const int cbits = 64 - __builtin_clzll((unsigned long long)blk_docs);
    for (int c = q.num_group_by; c < a.pf_nc && a.lds_pack < 0; c++) {
      const int i = a.pf_agg[c];
      if (gx.acc_kind[i] != 0) continue;
      bool affine = true;
      int bits = 0;
      for (size_t si = 0; si < S; si++) {
        affine = affine && gaggs[si * na + i].affine;
        bits = std::max(bits, gaggs[si * na + i].bits);
      }
      if (affine && bits + 2 * cbits <= 64) {
        a.lds_pack = i;
        a.lds_sbits = bits + cbits;
      }
    }
  }

  const auto tgp = std::chrono::steady_clock::now();
  check_deadline(e, "planning");
  PINOT_HIP(hipEventRecord(e.ev_start, e.stream));
  upload_arena(e, ar);
  Timer t(e);
  for (size_t si = 0; si < S && !pin; si++)
    if (plans[si].has_pre && !plans[si].empty) run_filter(e, plans[si], qs, t, (int64_t)si);
  PINOT_HIP(hipMemsetAsync(matched, 0, S * 8, e.stream));
  if (ks.hashed && !pin && (adm.active || gp.mode != GB_EMIT)) {  // before any pass inserts keys
    PINOT_HIP(hipMemsetAsync(htable, 0, (size_t)hcap * 8, e.stream));
    PINOT_HIP(hipMemsetAsync(reps, 0xFF, (size_t)hcap * 8, e.stream));
    PINOT_HIP(hipMemsetAsync(a.verify_err, 0, 4, e.stream));
  }
  if (adm.active && aio && aio->mode == 2) {  // the server's capped bitmaps for these segments
    require(aio->words == ab.words && aio->bitmaps.size() == S * (size_t)ab.words, PINOT_ERR_DEVICE,
            "admitted bitmaps of another shape");
    e.host_arena.reserve(aio->bitmaps.size() * 4);
    memcpy(e.host_arena.get(), aio->bitmaps.data(), aio->bitmaps.size() * 4);
    PINOT_HIP(hipMemcpyAsync(ab.bitmaps, e.host_arena.get(), aio->bitmaps.size() * 4, hipMemcpyHostToDevice, e.stream));
    wait_stream(e);  // host_arena stages the next query's arena
  } else if (adm.active) {  // first matching doc per (segment, key) -> admitted bitmaps (+ inter-segment cap)
    PINOT_HIP(hipMemsetAsync(ab.first_doc, 0xFF, (size_t)S * ks.G * 4, e.stream));
    GroupArgs af = a;
    af.mode = GB_FIRST;
    af.first_doc = ab.first_doc;
    launch_group_query(af, e.stream);
    PINOT_HIP(hipGetLastError());
    build_admitted(e, adm, S, ks.G, ab);
    if (aio && aio->mode == 1) {  // export for the server's cap; no group-by here
      aio->words = ab.words;
      aio->bitmaps.assign(S * (size_t)ab.words, 0u);
      PINOT_HIP(hipMemcpyAsync(aio->bitmaps.data(), ab.bitmaps, aio->bitmaps.size() * 4, hipMemcpyDeviceToHost, e.stream));
      wait_stream(e);
      return nullptr;
    }
  }
  const auto tgu = std::chrono::steady_clock::now();
  uint32_t *ring_status = nullptr;  // ring plan: [0] status bits, [1] region records (k_group_ring)
  if (pin) {
  } else if (rp.on) {  // [GB_FILTER ->] k_group_ring -> k_ring_reduce (group_ring.hip): every key written, no memset
    const size_t nblk = (size_t)rp.nblk;
    const size_t hist_n = (size_t)rp.P * nblk;
    const size_t hist_b = (hist_n * 4 + 255) / 256 * 256;
    e.group_part.reserve(hist_b + 256);
    uint8_t *pb = e.group_part.get<uint8_t>();
    auto *hist = reinterpret_cast<uint32_t *>(pb);
    ring_status = reinterpret_cast<uint32_t *>(pb + hist_b);
    e.group_records.reserve((size_t)rp.P * nblk * rp.cap * rp.rec_bytes + 64);
    // the filter: a top-level conjunction of <= kRingMaxQuarterLeaves scan leaves (RANGE / LUT, <= 20 bits) is
    // evaluated by the ring kernel itself on each quarter; any other program runs first as GB_FILTER
    int nf = 0;
    for (size_t si = 0; si < S && nf >= 0; si++) {
      const GroupSegment &g = gsegs[si];
      if (g.nwords == 0) continue;
      if (g.n_leaves > kRingMaxQuarterLeaves) nf = -1;
      for (int i = 0; i < g.n_leaves && nf >= 0; i++) {
        const FusedStep &l = leaves[g.first_leaf + i];
        const bool ok = l.join == JOIN_NEW && l.bits <= kGroupLwMaxBits &&
                        (l.kind == FK_LEAF_RANGE || l.kind == FK_LEAF_LUT64 || l.kind == FK_LEAF_LUT);
        nf = ok ? std::max(nf, g.n_leaves) : -1;
      }
    }
    if (!e.group_ring_qfilter) nf = -1;
    GroupArgs af = a;
    int64_t fstride = 0;
    if (nf < 0) {
      for (auto *sg : segs) fstride = std::max<int64_t>(fstride, sg->nwords());
      fstride = (fstride + 63) / 64 * 64;
      e.group_filter.reserve((size_t)S * fstride * 8 + 512);
      af.mode = GB_FILTER;
      af.filter_out = e.group_filter.get<uint64_t>();
      af.filter_stride = fstride;
    }
    RingArgs ra{};
    ra.segs = a.segs;
    ra.gcols = a.gcols;
    ra.aggs = a.aggs;
    ra.leaves = a.leaves;
    ra.cstart = reinterpret_cast<const int64_t *>(qs.arena + off_cstart);
    ra.filter = nf < 0 ? af.filter_out : nullptr;
    ra.filter_stride = fstride;
    ra.total_chunks = rp.total_chunks;
    ra.G = ks.G;
    ra.nsegs = (int32_t)S;
    ra.n_gcols = q.num_group_by;
    ra.nc = a.pf_nc;
    for (int i = 0; i < 4; i++) ra.pf_agg[i] = a.pf_agg[i];
    ra.P = (int32_t)rp.P;
    ra.shift = rp.shift;
    ra.nblk = (int32_t)nblk;
    ra.cap = rp.cap;
    ra.nf = nf;
    ra.records = e.group_records.get<uint8_t>();
    ra.rec_bytes = rp.rec_bytes;
    for (int i = 0; i < na; i++)
      if (rp.hll_form[i]) {  // the flushers' HLL field (segment 0's dictionary: identical on every segment)
        ra.hll = 1;
        ra.hll_shift = rp.field_shift[i];
        ra.hll_bits = gaggs[i].bits;
        ra.hll_base = (uint32_t)gaggs[i].affine_base;
        ra.hll_step = (uint32_t)gaggs[i].affine_step;
      }
    ra.hist = hist;
    ra.status = ring_status;
    ra.region = ring_status + 1;
    ra.matched = matched;  // the quarter-form filter counts each segment's matching docs (GB_FILTER does otherwise)
    RingReduceArgs rr{};
    rr.records = ra.records;
    rr.rec_bytes = rp.rec_bytes;
    rr.hist = hist;
    rr.region = ra.region;
    rr.P = (int32_t)rp.P;
    rr.shift = rp.shift;
    rr.n_aggs = na;
    rr.nblk = (int32_t)nblk;
    rr.lds_bytes = rr.lds_zero_bytes = rp.lds_bytes;
    rr.cnt_off = rp.cnt_off;
    rr.hist_off = rp.hist_off;
    rr.exc_off = rp.exc_off;
    rr.G = ks.G;
    rr.counts = counts;
    rr.status = ring_status;
    rr.hll_sums = po ? 0 : 1;  // the engine's HLL arrays have room for the sums; a caller's partial arrays do not
    for (int i = 0; i < na; i++) {
      rr.aggs[i] = gaggs[i];  // segment 0's dictionary / LUT: identical on every segment (checked by plan_group)
      rr.aggs[i].lds_off = rp.lds_off[i];
      if (rp.hll_form[i]) {
        rr.hll_pre |= 1 << i;
        rr.aggs[i].bits = kRingHllFieldBits;
      }
    }
    require(a.pf_nc > 0, PINOT_ERR_DEVICE, "ring plan without its column list");
    PINOT_HIP(hipMemsetAsync(ring_status, 0, 256, e.stream));
    e.ring_queries++;
    if (nf >= 0) e.ring_qfilter_queries++;
    e.ring_last_rec_bytes = rp.rec_bytes;
    e.ring_last_hll_slot = ra.hll;
    e.last_group_instance = kRingInstanceCode;
    t.timed(1, [&] {
      if (nf < 0) launch_group_query(af, e.stream);
      launch_group_ring(ra, e.stream);
      launch_ring_reduce(rr, e.stream);
    });
    PINOT_HIP(hipGetLastError());
  } else if (gp.mode != GB_EMIT) {  // identities: counts / sums 0, min all-ones, max 0, HLL 0
    PINOT_HIP(hipMemsetAsync(counts, 0, ks.G * 8, e.stream));
    for (int i = 0; i < na; i++)
      if (acc_bytes[i]) PINOT_HIP(hipMemsetAsync(accs[i], gx.acc_kind[i] == 2 ? 0xFF : 0, ks.G * acc_bytes[i], e.stream));
    e.last_group_instance = group_query_instance(a);
    t.timed(1, [&] { launch_group_query(a, e.stream); });
    PINOT_HIP(hipGetLastError());
    if (ks.hashed) {  // every doc's tuple == its slot representative's tuple, or the fingerprints collided
      GroupArgs av = a;
      av.mode = GB_VERIFY;
      launch_group_query(av, e.stream);
      PINOT_HIP(hipGetLastError());
    }
  } else {
    const size_t hist_n = (size_t)gp.P * nblk;
    int64_t max_records = 0;
    for (auto *sg : segs) max_records += sg->num_docs;
    const size_t scan_tmp = exclusive_sum_u32(nullptr, nullptr, (long long)hist_n, nullptr, 0, e.stream);
    const size_t hist_b = (hist_n * 4 + 255) / 256 * 256, pstart_b = ((size_t)gp.P * 4 + 4 + 255) / 256 * 256;
    e.group_part.reserve(3 * hist_b + pstart_b + scan_tmp + 256);
    uint8_t *pb = e.group_part.get<uint8_t>();
    auto *hist = reinterpret_cast<uint32_t *>(pb);
    auto *offsets = reinterpret_cast<uint32_t *>(pb + hist_b);
    auto *pstart = reinterpret_cast<uint32_t *>(pb + 2 * hist_b);
    auto *padded = reinterpret_cast<uint32_t *>(pb + 2 * hist_b + pstart_b);
    void *tmp = pb + 3 * hist_b + pstart_b;
    // bucketed plan: COUNT keeps the filter words, GB_EMIT2 writes whole LDS buckets into the final layout; the
    // lane-owns-quarter sink pads every (partition, block) run to whole 64-B buckets (aligned flushes)
    const bool bucket = e.group_bucket && a.pf_nc > 0 && gp.P <= kBucketMaxPartitions &&
                        gp.record_bits <= kRecPartShift && gp.P <= (int64_t(1) << (63 - kRecPartShift));
    const bool aligned = bucket && a.lw == 2 && e.group_aligned;
    const int64_t pad_records = aligned ? (int64_t)hist_n * (kBucketRecs - 1) : 0;
    require(max_records + pad_records < (int64_t)UINT32_MAX, PINOT_ERR_UNSUPPORTED,
            "partitioned group-by over > 4G docs per GPU");
    e.group_records.reserve((size_t)(max_records + pad_records) * 8 + 64);
    if (gp.split && !bucket) e.group_runs.reserve((size_t)max_records * 8 + 64);
    int64_t fstride = 0;
    if (bucket) {
      for (auto *sg : segs) fstride = std::max<int64_t>(fstride, sg->nwords());
      fstride = (fstride + 63) / 64 * 64;
      e.group_filter.reserve((size_t)S * fstride * 8 + 512);
      a.filter_out = e.group_filter.get<uint64_t>();
      a.filter_stride = fstride;
    }
    a.hist = hist;
    a.offsets = offsets;
    a.pstart = pstart;
    a.emit = gp.split && !bucket ? e.group_runs.get<unsigned long long>() : e.group_records.get<unsigned long long>();
    PartitionReduceArgs ra{};
    ra.records = e.group_records.get<unsigned long long>();
    ra.pstart = pstart;
    ra.P = (int32_t)gp.P;
    ra.shift = gp.shift;
    ra.n_aggs = na;
    ra.lds_bytes = gp.reduce_bytes;
    ra.wave_cnt_off = gp.reduce_wave_cnt_off;
    ra.skip_invalid = aligned ? 1 : 0;
    a.aligned_runs = aligned ? 1 : 0;
    a.emit_block = e.group_emit_block;
    ra.G = ks.G;
    ra.counts = counts;
    for (int i = 0; i < na; i++) {
      ra.aggs[i] = gaggs[i];  // segment 0's dictionary / LUT: identical on every segment (checked)
      ra.aggs[i].lds_off = gp.reduce_off[i];
    }
    t.timed(1, [&] {
      launch_group_query(a, e.stream);
      if (aligned) launch_pad_counts(hist, (long long)hist_n, padded, e.stream);
      exclusive_sum_u32(aligned ? padded : hist, offsets, (long long)hist_n, tmp, scan_tmp, e.stream);
      launch_partition_starts(offsets, aligned ? padded : hist, (int32_t)gp.P, (int32_t)nblk, pstart, e.stream);
      GroupArgs a2 = a;
      if (bucket) {
        a2.mode = GB_EMIT2;
        a2.stage_bytes = 0;  // no filter re-evaluation: the COUNT pass's words
        e.last_group_instance = group_query_instance(a2);
        launch_group_query(a2, e.stream);
      } else {
        a2.mode = GB_EMIT;
        a2.split = gp.split;
        e.last_group_instance = group_query_instance(a2);
        launch_group_query(a2, e.stream);
        launch_partition_split(hist, offsets, pstart, (int32_t)gp.P, (int32_t)nblk, gp.shift, gp.split, a.emit,
                               e.group_records.get<unsigned long long>(), e.group_nt_store, e.stream);
      }
      launch_partition_reduce(ra, e.stream);
    });
    PINOT_HIP(hipGetLastError());
  }

  if (po) {  // partial: the dense accumulators are the caller's (u8 HLL registers included), no compaction
    for (int i = 0; i < na; i++)
      if (alias[i] >= 0 && ga.acc_kind[i] != 5 && po->accs[i] != po->accs[alias[i]])
        PINOT_HIP(hipMemcpyAsync(po->accs[i], po->accs[alias[i]], ks.G * (ga.acc_kind[i] == 4 ? 256 : 8),
                                 hipMemcpyDeviceToDevice, e.stream));
    PINOT_HIP(hipGetLastError());
    std::vector<unsigned long long> hm(S);
    uint32_t rs[4] = {0, 0, 0, 0};
    PINOT_HIP(hipMemcpyAsync(hm.data(), matched, S * 8, hipMemcpyDeviceToHost, e.stream));
    if (ring_status) PINOT_HIP(hipMemcpyAsync(rs, ring_status, 16, hipMemcpyDeviceToHost, e.stream));
    PINOT_HIP(hipEventRecord(e.ev_stop, e.stream));
    wait_stream(e);
    if (rs[0]) {
      e.ring_last_status = rs[0];
      return ring_fallback();
    }
    float pms = 0;
    PINOT_HIP(hipEventElapsedTime(&pms, e.ev_start, e.ev_stop));
    t.collect();
    std::vector<int64_t> seg_counts(S);
    for (size_t si = 0; si < S; si++) seg_counts[si] = plans[si].empty ? 0 : (int64_t)hm[si];
    fill_stats(q, plans, seg_counts, pms, stats);
    return nullptr;
  }

  const auto tg1 = std::chrono::steady_clock::now();
  if (e.host_phases) wait_stream(e);
  const auto tg2 = std::chrono::steady_clock::now();
  // finalize: ordered non-empty keys, per-group outputs, one D2H
  std::vector<unsigned long long> hmatched(S);
  uint32_t verify_err = 0;
  long long *keys_dev = nullptr;
  uint32_t rs[4] = {0, 0, 0, 0};
  uint8_t *small = nullptr;
  const unsigned long long n = compact_dense(e, counts, ks.G, keys_dev, [&](uint8_t *pin) {
    small = pin;  // [0, 8S) matched, then 16 B of ring status, then the verify flag
    PINOT_HIP(hipMemcpyAsync(pin, matched, S * 8, hipMemcpyDeviceToHost, e.stream));
    if (ring_status) PINOT_HIP(hipMemcpyAsync(pin + S * 8, ring_status, 16, hipMemcpyDeviceToHost, e.stream));
    if (ks.hashed) PINOT_HIP(hipMemcpyAsync(pin + S * 8 + 16, a.verify_err, 4, hipMemcpyDeviceToHost, e.stream));
  }, S * 8 + 32);
  memcpy(hmatched.data(), small, S * 8);
  if (ring_status) memcpy(rs, small + S * 8, 16);
  if (ks.hashed) memcpy(&verify_err, small + S * 8 + 16, 4);
  if (rs[0]) {
    e.ring_last_status = rs[0];
    return ring_fallback();
  }
  if (verify_err) {  // 64-bit fingerprint collision: retry with another seed
    require(attempt < 3, PINOT_ERR_DEVICE, "group-key fingerprint collisions persist");
    return exec_group_by_fused(e, segs, q, ks_in, ga, stats, attempt + 1);
  }
  const auto tg3 = std::chrono::steady_clock::now();
  DenseGroups dg{&q, &ks, &ga, &gx, &alias, counts, accs, 0, ks.hashed ? &a : nullptr};
  if (ring_status) {  // the ring reduce wrote each HLL's packed register sums after its registers
    dg.hll_sum.assign(na, nullptr);
    for (int i = 0; i < na; i++)
      if (gx.acc_kind[i] == 4) dg.hll_sum[i] = static_cast<const uint8_t *>(accs[i]) + (size_t)ks.G * 256;
  }
  std::vector<std::vector<int64_t>> kept;
  unsigned long long nres = n;
  const long long *rkeys = keys_dev;
  if (e.trim_top_n > 0) rkeys = device_trim(e, dg, keys_dev, nres, e.trim_top_n, kept);
  auto res = build_dense_result(e, dg, rkeys, nres, rkeys != keys_dev);
  res->merged_groups = (int64_t)n;  // before the trim: CombineGroupByOperator's numGroupsLimitReached test
  if (!kept.empty()) {
    res->trimmed_top_n = e.trim_top_n;
    res->fn_kept = std::move(kept);
  }
  const auto tg4 = std::chrono::steady_clock::now();
  PINOT_HIP(hipEventRecord(e.ev_stop, e.stream));
  wait_stream(e);
  if (e.host_phases) {
    const auto tg5 = std::chrono::steady_clock::now();
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    fprintf(stderr, "[pinot_gpu] group-by plan (us): compile %.1f, remap+scratch %.1f, accumulators %.1f, program %.1f\n",
            us(tg0, tga), us(tga, tgb), us(tgb, tgc), us(tgc, tgp));
    fprintf(stderr, "[pinot_gpu] group-by host phases (us): plan %.1f, upload %.1f, launch %.1f, kernels %.1f, "
            "compact+sync %.1f, outputs+D2H %.1f, host finalize %.1f (%llu groups)\n", us(tg0, tgp), us(tgp, tgu),
            us(tgu, tg1), us(tg1, tg2), us(tg2, tg3), us(tg3, tg4), us(tg4, tg5), (unsigned long long)n);
  }
  float ms = 0;
  PINOT_HIP(hipEventElapsedTime(&ms, e.ev_start, e.ev_stop));
  t.collect();
  std::vector<int64_t> seg_counts(S);
  for (size_t si = 0; si < S; si++) seg_counts[si] = plans[si].empty ? 0 : (int64_t)hmatched[si];
  fill_stats(q, plans, seg_counts, ms, stats);
  return res;
}

bool touches_mv_group_by(const std::vector<SegmentData *> &segs, const pinot_query &q) {
  bool mv = touches_mv_aggregation(segs, q);
  for (int j = 0; j < q.num_group_by; j++)
    for (SegmentData *sg : segs) {
      auto it = sg->by_name.find(q.group_by[j]);
      mv = mv || (it != sg->by_name.end() && sg->cols[it->second]->mv);
    }
  return mv;
}


std::vector<pinot_agg_spec> mv_extended_specs(const pinot_query &q, std::vector<int> &hidden) {
  const int na = q.num_aggregations;
  std::vector<pinot_agg_spec> specs(q.aggregations, q.aggregations + na);
  hidden.assign(na, -1);
  for (int a = 0; a < na; a++)
    if (q.aggregations[a].function == PINOT_AGG_AVGMV) {
      require((int)specs.size() < kMaxAggs, PINOT_ERR_UNSUPPORTED, "too many aggregations with AVGMV (8 at most)");
      pinot_agg_spec h = q.aggregations[a];
      h.function = PINOT_AGG_COUNTMV;
      hidden[a] = (int)specs.size();
      specs.push_back(h);
    }
  return specs;
}

void fold_mv_counts(GroupByResult &res, const pinot_query &q, const std::vector<int> &hidden) {
  const int na = q.num_aggregations;
  if (res.counts_shared) {  // one count vector for every function: split it before the MV functions take theirs
    res.counts.resize(res.functions.size());
    for (size_t a = 1; a < res.counts.size(); a++) res.counts[a] = res.counts[0];
    res.counts_shared = false;
  }
  for (int a = 0; a < na; a++) {
    const int f = q.aggregations[a].function;
    const int src = f == PINOT_AGG_COUNTMV ? a : hidden[a];
    if (src < 0) continue;
    HostVec<int64_t> &cv = res.counts[a];
    const HostVec<double> &sv = res.values[src];
    cv.resize(sv.size());
    for (size_t i = 0; i < cv.size(); i++) cv[i] = (int64_t)sv[i];
  }
  res.functions.resize(na);
  res.counts.resize(na);
  res.values.resize(na);
  res.hll.resize(na);
  res.hll_card.resize(na);
  for (HllPart &part : res.hll_parts) part.off.resize(na);
}

namespace {

// Group-by with multi-value group columns or MV functions: per segment the filter's bitset and one k_group_by_mv
// (every doc's cartesian product of group keys, DictionaryBasedGroupKeyGenerator's MV branch) into dense
// accumulators over the global key space, then the bitset path's finalisation. AvgMV needs its entry count beside
// its sum: a hidden CountMV accumulator per AvgMV, folded into the function's counts after finalisation. num.groups.limit:
// first-appearance admission per segment, then the 2 x limit cap (here, or the server's across ranks: `mp`).
std::unique_ptr<GroupByResult> exec_group_by_mv(Engine &e, const std::vector<SegmentData *> &segs,
                                                const pinot_query &q, pinot_exec_stats *stats,
                                                const MvPartial *mp = nullptr, int attempt = 0) {
  std::vector<int> hidden;
  std::vector<pinot_agg_spec> specs = mv_extended_specs(q, hidden);
  pinot_query q2 = q;
  q2.aggregations = specs.data();
  q2.num_aggregations = (int32_t)specs.size();
  const int nb = q2.num_aggregations;
  Arena ar;
  std::unique_ptr<FilterTreeInput> tree;
  std::vector<SegPlan> plans = plan_all(e, segs, q2, ar, tree);
  KeySpace ks;
  if (mp) {  // the server's global key space (union dictionaries over every rank)
    ks.gcard = *mp->gcard;
    ks.gvalues = *mp->gvalues;
    ks.remap = *mp->remap;
    ks.G = 1;
    for (auto g : ks.gcard) ks.G *= g;
  } else {
    ks = build_key_space(segs, q2);
  }
  const int64_t limit = q.num_groups_limit > 0 ? q.num_groups_limit : e.num_groups_limit;
  require(!(ks.hashed && mp), PINOT_ERR_UNSUPPORTED, "multi-GPU partials of a multi-value group-by over a hashed key space");
  const size_t S = segs.size();
  QueryScratch qs = prepare(e, plans, ar);
  Timer t(e);
  // hashed key space (LONG_MAP / ARRAY_MAP holder shapes, mv_hash.h): slots = a power of two >= 2 x the keys the
  // matching docs yield, counted on the device
  int64_t hcap = 0;
  if (ks.hashed) {
    DeviceBuffer tot(64);
    PINOT_HIP(hipMemsetAsync(tot.get(), 0, 8, e.stream));
    for (size_t si = 0; si < S; si++) {
      SegPlan &pl = plans[si];
      if (pl.empty || pl.seg->num_docs == 0) continue;
      MvGroupArgs c{};
      c.n_gcols = q.num_group_by;
      for (int j = 0; j < q.num_group_by; j++) {
        const ColumnData &col = *pl.seg->column(q.group_by[j]);
        c.goff[j] = col.mv ? col.mv_offsets.get<uint32_t>() : nullptr;
      }
      c.bitset = run_filter(e, pl, qs, t);
      c.nwords = pl.seg->nwords();
      c.num_docs = pl.seg->num_docs;
      launch_mv_key_count(c, tot.get<unsigned long long>(), e.stream);
      PINOT_HIP(hipGetLastError());
    }
    unsigned long long keys = 0;
    PINOT_HIP(hipMemcpyAsync(&keys, tot.get(), 8, hipMemcpyDeviceToHost, e.stream));
    wait_stream(e);
    hcap = 1024;
    while (hcap < 2 * (int64_t)keys) hcap <<= 1;
    ks.G = hcap;
  }
  // num.groups.limit (DictionaryBasedGroupKeyGenerator :79-126, IntMapBasedHolder.processMultiValue :282-300): a segment
  // whose cardinality product exceeds max.init.group.holder.capacity admits the first min(product, limit) distinct keys
  // in doc order, each doc's keys in getIntRawKeys order; then CombineGroupByOperator's 2 x limit cap in segment order
  AdmissionPlan adm;
  {
    const int64_t threshold = q.max_init_group_holder_capacity > 0 ? q.max_init_group_holder_capacity : 10000;
    int64_t possible = 0;
    for (auto *sg : segs) {
      __int128 product = 1;
      for (int j = 0; j < q.num_group_by; j++) product *= sg->column(q.group_by[j])->card;
      int64_t upper = INT64_MAX;
      if (product > threshold) upper = product <= INT32_MAX ? std::min<int64_t>((int64_t)product, limit) : limit;
      const int64_t reach = (int64_t)std::min<__int128>(product, (__int128)ks.G);  // a doc yields several keys
      if (upper < reach) adm.active = true;
      else upper = ks.G;
      adm.upper.push_back(upper);
      possible += std::min(upper, reach);
    }
    adm.cap = 2 * limit;
    if (std::min(possible, ks.G) > adm.cap) adm.active = adm.cap_active = true;
    if (mp && mp->aio) {  // the server applies the cap across ranks
      adm.active = true;
      adm.cap_active = false;
    } else if (mp) {
      require(!adm.cap_active, PINOT_ERR_DEVICE, "multi-GPU MV group-by partial without the server's cap exchange");
    }
  }
  GroupAccs ga;
  for (int a = 0; a < nb; a++) {
    const int f = specs[a].function;
    int kind = 5;
    size_t bytes = 0;
    if (f != PINOT_AGG_COUNT) {
      const ColumnData &c = *segs[0]->column(agg_column(specs[a]));
      bytes = 8;
      if (f == PINOT_AGG_COUNTMV) {
        kind = 6;
      } else if (f == PINOT_AGG_DISTINCTCOUNTHLL || f == PINOT_AGG_DISTINCTCOUNTHLLMV) {
        kind = 4;
        bytes = 1024;
      } else {
        require(c.numeric(), PINOT_ERR_BAD_QUERY, "numeric aggregation over STRING column " + c.name);
        const int sf = sv_function(f);
        kind = sf == PINOT_AGG_MIN ? 2 : sf == PINOT_AGG_MAX ? 3 : c.data_type == PINOT_INT ? 0 : 1;
      }
    }
    ga.acc_kind.push_back(kind);
    ga.acc_bytes_per_key.push_back(bytes);
  }
  size_t per_key = 8 + (ks.hashed ? 8 + 4 * (size_t)q.num_group_by : 0);  // (+ the table's fingerprint and tuple)
  for (auto b : ga.acc_bytes_per_key) per_key += b;
  size_t free_b = 0, total_b = 0;
  PINOT_HIP(hipMemGetInfo(&free_b, &total_b));
  require((double)ks.G * per_key < 0.5 * (double)free_b, PINOT_ERR_UNSUPPORTED,
          "dense group-by accumulators do not fit in HBM");
  MvHash mh{};
  if (ks.hashed) {
    e.group_hash.reserve((size_t)hcap * (8 + 4 * (size_t)q.num_group_by) + 256);
    mh.htable = e.group_hash.get<unsigned long long>();
    mh.tuples = reinterpret_cast<int32_t *>(mh.htable + hcap);
    mh.verify_err = reinterpret_cast<uint32_t *>(e.group_hash.get<uint8_t>() + (size_t)hcap * (8 + 4 * (size_t)q.num_group_by));
    mh.hcap = hcap;
    mh.hseed = 0x5EEDF00Dull + 0x9E3779B97F4A7C15ull * (unsigned long long)(attempt + 1);
    PINOT_HIP(hipMemsetAsync(mh.htable, 0, (size_t)hcap * 8, e.stream));
    PINOT_HIP(hipMemsetAsync(mh.verify_err, 0, 4, e.stream));
  }
  e.group_scratch.reserve(ks.G * per_key + 64);
  uint8_t *base = e.group_scratch.get<uint8_t>();
  auto *counts = reinterpret_cast<unsigned long long *>(base);
  std::vector<void *> accs(nb, nullptr);
  uint8_t *p = base + ks.G * 8;
  for (int a = 0; a < nb; a++) {
    if (ga.acc_kind[a] == 5) continue;
    accs[a] = p;
    p += ks.G * ga.acc_bytes_per_key[a];
  }
  if (mp && mp->accs) {  // partial: the server's arrays (HLL registers accumulate as u32 here, narrowed into its u8
                         // layout); the admission export (no arrays) keeps the scratch ones
    counts = reinterpret_cast<unsigned long long *>(mp->counts);
    for (int a = 0; a < nb; a++)
      if (ga.acc_kind[a] != 5 && ga.acc_kind[a] != 4) accs[a] = mp->accs[a];
  }
  PINOT_HIP(hipEventRecord(e.ev_start, e.stream));
  if (!(mp && !mp->accs)) init_accs(e, ks.G, counts, ga, accs.data());  // (the admission export: no arrays)
  std::vector<DeviceBuffer> remaps(S * q.num_group_by);
  std::vector<int64_t> seg_counts(S, 0);
  auto mv_args = [&](size_t si, const uint64_t *bits) {
    SegmentData &sg = *plans[si].seg;
    MvGroupArgs a{};
    a.n_gcols = q.num_group_by;
    a.n_aggs = nb;
    long long stride = 1;
    for (int j = 0; j < q.num_group_by; j++) {
      const ColumnData &c = *sg.column(q.group_by[j]);
      a.gfwd[j] = c.fwd.get<uint8_t>();
      a.goff[j] = c.mv ? c.mv_offsets.get<uint32_t>() : nullptr;
      a.gbits[j] = c.bits;
      const auto &m = ks.remap[si][j];
      if (!m.empty()) {
        DeviceBuffer &rb = remaps[si * q.num_group_by + j];
        if (!rb.size()) {  // uploaded once per query (the admission pass and the accumulation pass share it)
          rb.alloc(m.size() * 4 + 16);
          PINOT_HIP(hipMemcpyAsync(rb.get(), m.data(), m.size() * 4, hipMemcpyHostToDevice, e.stream));
        }
        a.remap[j] = rb.get<int32_t>();
      }
      a.stride[j] = stride;
      stride *= ks.gcard[j];
    }
    for (int g = 0; g < nb; g++) {
      a.acc_kind[g] = ga.acc_kind[g];
      a.acc[g] = accs[g];
      if (ga.acc_kind[g] == 5) continue;
      ColumnData &c = *sg.column(agg_column(specs[g]));
      a.afwd[g] = c.fwd.get<uint8_t>();
      a.aoff[g] = c.mv ? c.mv_offsets.get<uint32_t>() : nullptr;
      a.abits[g] = c.bits;
      a.dict[g] = c.dict_dev.get();
      a.value_kind[g] = c.value_kind();
      if (ga.acc_kind[g] == 4) {
        ensure_hll_lut(e, c);
        a.hll_lut[g] = c.hll_lut.get<uint16_t>();
      }
    }
    a.counts = counts;
    a.bitset = bits;
    a.nwords = sg.nwords();
    a.num_docs = sg.num_docs;
    return a;
  };
  if (ks.hashed)  // the table: every matching doc's keys
    for (size_t si = 0; si < S; si++) {
      SegPlan &pl = plans[si];
      if (pl.empty || pl.seg->num_docs == 0) continue;
      launch_mv_hash_insert(mv_args(si, run_filter(e, pl, qs, t)), mh, e.stream);
      PINOT_HIP(hipGetLastError());
    }
  // admission: every segment's first-appearance bitmap (first positions, one radix sort each), then the cap
  DeviceBuffer adm_buf;
  int64_t words = 0;
  AdmissionIO *aio = mp ? mp->aio : nullptr;
  if (adm.active && aio && aio->mode == 2) {  // the server's capped bitmaps for these segments
    words = (ks.G + 31) / 32 + 1;
    require(aio->words == words && aio->bitmaps.size() == S * (size_t)words, PINOT_ERR_DEVICE,
            "admitted bitmaps of another shape");
    const size_t fp_b = ((size_t)ks.G * 8 + 255) / 256 * 256;
    adm_buf.alloc(fp_b + aio->bitmaps.size() * 4 + 256);
    PINOT_HIP(hipMemcpyAsync(adm_buf.get<uint8_t>() + fp_b, aio->bitmaps.data(), aio->bitmaps.size() * 4,
                             hipMemcpyHostToDevice, e.stream));
    wait_stream(e);
  } else if (adm.active) {
    words = (ks.G + 31) / 32 + 1;
    const size_t fp_b = ((size_t)ks.G * 8 + 255) / 256 * 256, bm_b = ((size_t)S * words * 4 + 255) / 256 * 256;
    const size_t scr = admission_scratch_bytes_u64(ks.G);
    adm_buf.alloc(fp_b + bm_b + scr);
    auto *first_pos = adm_buf.get<unsigned long long>();
    auto *bitmaps = reinterpret_cast<uint32_t *>(adm_buf.get<uint8_t>() + fp_b);
    PINOT_HIP(hipMemsetAsync(bitmaps, 0, (size_t)S * words * 4, e.stream));
    for (size_t si = 0; si < S; si++) {
      SegPlan &pl = plans[si];
      if (pl.empty || pl.seg->num_docs == 0) continue;
      const MvGroupArgs a = mv_args(si, run_filter(e, pl, qs, t));
      PINOT_HIP(hipMemsetAsync(first_pos, 0xFF, (size_t)ks.G * 8, e.stream));
      if (ks.hashed) launch_first_pos_mv_hashed(a, mh, first_pos, e.stream);
      else launch_first_pos_mv(a, first_pos, e.stream);
      launch_admission_bitmap_u64(first_pos, ks.G, adm.upper[si], bitmaps + si * words, words,
                                  adm_buf.get<uint8_t>() + fp_b + bm_b, scr, e.stream);
      PINOT_HIP(hipGetLastError());
    }
    if (aio && aio->mode == 1) {  // export for the server's cap: no accumulation here
      aio->words = words;
      aio->bitmaps.assign(S * (size_t)words, 0u);
      PINOT_HIP(hipMemcpyAsync(aio->bitmaps.data(), bitmaps, aio->bitmaps.size() * 4, hipMemcpyDeviceToHost, e.stream));
      wait_stream(e);
      return nullptr;
    }
    if (adm.cap_active) {
      std::vector<uint32_t> bm(S * words);
      PINOT_HIP(hipMemcpyAsync(bm.data(), bitmaps, bm.size() * 4, hipMemcpyDeviceToHost, e.stream));
      wait_stream(e);
      apply_inter_segment_cap(bm, S, words, adm.cap);
      PINOT_HIP(hipMemcpyAsync(bitmaps, bm.data(), bm.size() * 4, hipMemcpyHostToDevice, e.stream));
      wait_stream(e);
    }
  }
  for (size_t si = 0; si < S; si++) {
    SegPlan &pl = plans[si];
    SegmentData &sg = *pl.seg;
    if (pl.empty || sg.num_docs == 0) continue;
    const uint64_t *bits = run_filter(e, pl, qs, t);
    seg_counts[si] = count_docs(e, bits, sg);
    MvGroupArgs a = mv_args(si, bits);
    if (adm.active)
      a.admitted = reinterpret_cast<const uint32_t *>(adm_buf.get<uint8_t>() + ((size_t)ks.G * 8 + 255) / 256 * 256) +
                   si * words;
    t.timed(1, [&] {
      if (ks.hashed) launch_group_by_mv_hashed(a, mh, e.stream);
      else launch_group_by_mv(a, e.stream);
    });
    PINOT_HIP(hipGetLastError());
  }
  if (ks.hashed) {  // a fingerprint collision: retry with another seed
    uint32_t verify_err = 0;
    PINOT_HIP(hipMemcpyAsync(&verify_err, mh.verify_err, 4, hipMemcpyDeviceToHost, e.stream));
    wait_stream(e);
    if (verify_err) {
      require(attempt < 3, PINOT_ERR_DEVICE, "group-key fingerprint collisions persist");
      return exec_group_by_mv(e, segs, q, stats, mp, attempt + 1);
    }
  }
  if (mp) {  // partial: the u32 registers into the server's u8 layout, the statistics, no finalisation
    for (int a = 0; a < nb; a++)
      if (ga.acc_kind[a] == 4) launch_narrow_u32(static_cast<const uint32_t *>(accs[a]), ks.G * 256,
                                                 static_cast<uint8_t *>(mp->accs[a]), e.stream);
    PINOT_HIP(hipGetLastError());
    PINOT_HIP(hipEventRecord(e.ev_stop, e.stream));
    wait_stream(e);
    float ms = 0;
    PINOT_HIP(hipEventElapsedTime(&ms, e.ev_start, e.ev_stop));
    t.collect();
    fill_stats(q, plans, seg_counts, ms, stats);
    return nullptr;
  }
  GroupByProgram gp{};
  gp.n_aggs = nb;
  gp.counts = counts;
  for (int a = 0; a < nb; a++) { gp.acc[a] = accs[a]; gp.acc_kind[a] = ga.acc_kind[a]; }
  auto res = finalize_groups(e, q2, ga, ks, gp, ks.hashed ? &mh : nullptr);
  PINOT_HIP(hipEventRecord(e.ev_stop, e.stream));
  wait_stream(e);
  float ms = 0;
  PINOT_HIP(hipEventElapsedTime(&ms, e.ev_start, e.ev_stop));
  t.collect();
  // CountMV: the entry count is the function's count; AvgMV: its hidden CountMV's values
  fold_mv_counts(*res, q, hidden);
  fill_stats(q, plans, seg_counts, ms, stats);
  return res;
}

// Group-by on the segments' star-trees (StarTreeGroupByExecutor): the traversal's matched star docs per segment, then
// k_group_by_mv over the star docs' dimension columns (the segment's dictionaries, so the global key space and its
// remaps are the segments' own) with each function over its pair column; COUNT is Σ count__* per group (exact int64).
// Segments whose tree does not fit (on_star[si] false) run their own filter and fold their columns into the same
// accumulators (COUNT and AVG's count: +1 per doc; SUM / AVG as doubles, as the pair columns hold them; HLL by value
// hash) — each segment on its own plan, as InstancePlanMakerImplV2 plans them. Runs while the key space fits
// num.groups.limit (no admission); otherwise the caller takes the regular plan.
std::unique_ptr<GroupByResult> exec_group_by_star(Engine &e, const std::vector<SegmentData *> &segs,
                                                  const std::vector<bool> &on_star, const pinot_query &q,
                                                  pinot_exec_stats *stats) {
  const int na = q.num_aggregations;
  KeySpace ks = build_key_space(segs, q);
  const int64_t limit = q.num_groups_limit > 0 ? q.num_groups_limit : e.num_groups_limit;
  if (ks.hashed || ks.G > limit) return nullptr;
  StarQuery sq;
  star_query(q, sq);
  std::unique_ptr<FilterTreeInput> tree;
  if (q.num_filter_nodes > 0) tree = std::make_unique<FilterTreeInput>(decode_filter(q.num_filter_nodes, q.filter));
  const size_t S = segs.size();
  std::vector<StarMatch> m(S);
  std::vector<SegmentData *> star_segs, scan_segs;
  std::vector<StarMatch> star_m;
  const SegmentData *first_star = nullptr;
  for (size_t si = 0; si < S; si++) {
    if (!on_star[si]) {
      scan_segs.push_back(segs[si]);
      continue;
    }
    m[si] = star_tree_match(*segs[si], q, tree.get());
    star_segs.push_back(segs[si]);
    star_m.push_back(m[si]);
    if (!first_star) first_star = segs[si];
  }
  require(first_star != nullptr, PINOT_ERR_BAD_ARG, "star-tree group-by without a star-tree segment");
  const int nb = sq.all.num_aggregations;
  GroupAccs ga;
  for (int a = 0; a < nb; a++) {
    if (sq.specs[a].function == PINOT_AGG_DISTINCTCOUNTHLL) {  // u32 registers per key (the kernel's kind 8)
      ga.acc_kind.push_back(4);
      ga.acc_bytes_per_key.push_back(1024);
      continue;
    }
    const ColumnData &c = *first_star->star->docs->column(sq.names[a]);
    const int f = sq.specs[a].function;  // COUNT is already SUM over count__*
    // a LONG column sums exactly in int64 (kind 7, or kind 0 over an int32 dictionary); DOUBLE in f64 (kind 1)
    ga.acc_kind.push_back(f == PINOT_AGG_MIN ? 2 : f == PINOT_AGG_MAX ? 3
                          : c.value_kind() == 0 ? 0 : c.value_kind() == 1 ? 7 : 1);
    ga.acc_bytes_per_key.push_back(8);
  }
  for (int a = 0; a < na; a++)  // the scan side adds exactly one per doc where the star side adds counts
    if (q.aggregations[a].function == PINOT_AGG_COUNT || q.aggregations[a].function == PINOT_AGG_AVG) {
      const int slot = q.aggregations[a].function == PINOT_AGG_COUNT ? a : sq.hidden[a];
      if (!scan_segs.empty() && ga.acc_kind[slot] == 0) return nullptr;  // int32 count column: not this plan
    }
  size_t per_key = 8;
  for (auto b : ga.acc_bytes_per_key) per_key += b;
  size_t free_b = 0, total_b = 0;
  PINOT_HIP(hipMemGetInfo(&free_b, &total_b));
  if ((double)ks.G * per_key >= 0.5 * (double)free_b) return nullptr;  // the scan plan sizes its own sink
  // the scan side's filters (plans over its segments; bitsets produced per segment before its fold)
  Arena ar;
  std::unique_ptr<FilterTreeInput> scan_tree;
  std::vector<SegPlan> plans;
  QueryScratch qs;
  if (!scan_segs.empty()) {
    plans = plan_all(e, scan_segs, q, ar, scan_tree);
    qs = prepare(e, plans, ar);
  }
  e.star_answered.insert(e.star_answered.end(), star_segs.begin(), star_segs.end());
  e.group_scratch.reserve(ks.G * per_key + 64);
  uint8_t *base = e.group_scratch.get<uint8_t>();
  auto *counts = reinterpret_cast<unsigned long long *>(base);
  std::vector<void *> accs(nb, nullptr);
  uint8_t *ap = base + ks.G * 8;
  for (int a = 0; a < nb; a++) {
    accs[a] = ap;
    ap += ks.G * ga.acc_bytes_per_key[a];
  }
  PINOT_HIP(hipEventRecord(e.ev_start, e.stream));
  init_accs(e, ks.G, counts, ga, accs.data());
  Timer t(e);
  std::vector<DeviceBuffer> remaps(S * q.num_group_by);
  std::vector<DeviceBuffer> bits(S);
  std::vector<int64_t> seg_counts(scan_segs.size(), 0);
  size_t pi = 0;
  for (size_t si = 0; si < S; si++) {
    const bool star = on_star[si];
    const uint64_t *bitset = nullptr;
    SegPlan *pl = star ? nullptr : &plans[pi++];
    if (star) {
      if (m[si].empty || m[si].docs == 0) continue;
      bits[si].alloc(m[si].bits.size() * 8 + 16);
      PINOT_HIP(hipMemcpyAsync(bits[si].get(), m[si].bits.data(), m[si].bits.size() * 8, hipMemcpyHostToDevice,
                               e.stream));
      bitset = bits[si].get<uint64_t>();
    } else {
      if (pl->empty || pl->seg->num_docs == 0) continue;
      bitset = run_filter(e, *pl, qs, t);
      seg_counts[pi - 1] = count_docs(e, bitset, *pl->seg);
    }
    SegmentData &sd = star ? *segs[si]->star->docs : *segs[si];
    MvGroupArgs a{};
    a.n_gcols = q.num_group_by;
    a.n_aggs = nb;
    long long stride = 1;
    for (int j = 0; j < q.num_group_by; j++) {
      const ColumnData &c = *sd.column(q.group_by[j]);
      a.gfwd[j] = c.fwd.get<uint8_t>();
      a.goff[j] = nullptr;
      a.gbits[j] = c.bits;
      const auto &rm = ks.remap[si][j];
      if (!rm.empty()) {
        DeviceBuffer &rb = remaps[si * q.num_group_by + j];
        rb.alloc(rm.size() * 4 + 16);
        PINOT_HIP(hipMemcpyAsync(rb.get(), rm.data(), rm.size() * 4, hipMemcpyHostToDevice, e.stream));
        a.remap[j] = rb.get<int32_t>();
      }
      a.stride[j] = stride;
      stride *= ks.gcard[j];
    }
    for (int g = 0; g < nb; g++) {
      a.acc[g] = accs[g];
      const int f = g < na ? q.aggregations[g].function : PINOT_AGG_COUNT;  // hidden slots: AVG's counts
      if (!star && f == PINOT_AGG_COUNT) {
        a.acc_kind[g] = 6;  // one per doc (an SV row holds one entry)
        continue;
      }
      if (ga.acc_kind[g] == 4) {
        if (star) {  // the doc's register row (kind 8)
          a.acc_kind[g] = 8;
          a.dict[g] = segs[si]->star->regs.at(sq.names[g]).get();
          continue;
        }
        ColumnData &c = *sd.column(agg_column(q.aggregations[g]));
        ensure_hll_lut(e, c);
        a.acc_kind[g] = 4;
        a.afwd[g] = c.fwd.get<uint8_t>();
        a.abits[g] = c.bits;
        a.hll_lut[g] = c.hll_lut.get<uint16_t>();
        continue;
      }
      ColumnData &c = *sd.column(star ? sq.names[g] : agg_column(q.aggregations[g]));
      require(star || c.numeric(), PINOT_ERR_BAD_QUERY, "numeric aggregation over STRING column " + c.name);
      a.acc_kind[g] = ga.acc_kind[g];
      a.afwd[g] = c.fwd.get<uint8_t>();
      a.aoff[g] = nullptr;
      a.abits[g] = c.bits;
      a.dict[g] = c.dict_dev.get();
      a.value_kind[g] = c.value_kind();
    }
    a.counts = counts;
    a.bitset = bitset;
    a.nwords = sd.nwords();
    a.num_docs = sd.num_docs;
    launch_group_by_mv(a, e.stream);
    PINOT_HIP(hipGetLastError());
  }
  GroupByProgram gp{};
  gp.n_aggs = nb;
  gp.counts = counts;
  for (int a = 0; a < nb; a++) { gp.acc[a] = accs[a]; gp.acc_kind[a] = ga.acc_kind[a]; }
  auto res = finalize_groups(e, sq.all, ga, ks, gp);
  PINOT_HIP(hipEventRecord(e.ev_stop, e.stream));
  wait_stream(e);
  float ms = 0;
  PINOT_HIP(hipEventElapsedTime(&ms, e.ev_start, e.ev_stop));
  t.collect();
  for (int a = 0; a < na; a++) {
    const int f = q.aggregations[a].function;
    res->functions[a] = f;
    // COUNT: the groups' Σ count__*; AVG: Σ avg__x.count from its hidden slot
    const int src = f == PINOT_AGG_COUNT ? a : f == PINOT_AGG_AVG ? sq.hidden[a] : -1;
    if (src < 0) continue;
    HostVec<int64_t> &cv = res->counts[a];
    const HostVec<double> &v = res->values[src];
    for (size_t i = 0; i < cv.size(); i++) cv[i] = (int64_t)v[i];
  }
  res->functions.resize(na);
  res->counts.resize(na);
  res->values.resize(na);
  res->hll.resize(na);
  res->hll_card.resize(na);
  pinot_exec_stats s1{}, s2{};
  star_stats(sq.q, star_segs, star_m, ms, &s1);
  if (!scan_segs.empty()) fill_stats(q, plans, seg_counts, 0.0f, &s2);
  if (stats) {
    *stats = s1;
    stats->num_docs_scanned += s2.num_docs_scanned;
    stats->num_entries_scanned_in_filter += s2.num_entries_scanned_in_filter;
    stats->num_entries_scanned_post_filter += s2.num_entries_scanned_post_filter;
    stats->num_total_raw_docs += s2.num_total_raw_docs;
    stats->num_segments_processed += s2.num_segments_processed;
    stats->num_segments_matched += s2.num_segments_matched;
  }
  return res;
}

}  // namespace

std::unique_ptr<GroupByResult> exec_group_by(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q,
                                             pinot_exec_stats *stats) {
  const int na = q.num_aggregations;
  require(na >= 1 && na <= kMaxAggs, PINOT_ERR_UNSUPPORTED, "1..8 aggregation functions per query");
  require(q.num_group_by >= 1 && q.num_group_by <= kMaxGroupCols, PINOT_ERR_UNSUPPORTED, "1..16 group-by columns");
  if (touches_mv_group_by(segs, q)) return exec_group_by_mv(e, segs, q, stats);
  std::vector<bool> on_star(segs.size());
  bool any_star = false;
  for (size_t i = 0; i < segs.size(); i++) any_star |= (on_star[i] = star_plan_fits(e, *segs[i], q));
  if (any_star) {  // each segment on its own plan (star-tree where its tree fits)
    auto r = exec_group_by_star(e, segs, on_star, q, stats);
    if (r) return r;
  }
  if (e.use_fused) {
    const auto t0 = std::chrono::steady_clock::now();
    KeySpace ks = build_key_space(segs, q);
    GroupAccs ga = group_acc_kinds(*segs[0], q);
    if (e.host_phases)
      fprintf(stderr, "[pinot_gpu] group-by key space (us): %.1f\n",
              std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    return exec_group_by_fused(e, segs, q, ks, ga, stats);
  }
  return exec_group_by_legacy(e, segs, q, stats);
}

std::unique_ptr<GroupByResult> exec_group_by_legacy(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q,
                                                    pinot_exec_stats *stats) {
  const int na = q.num_aggregations;
  require(na >= 1 && na <= kMaxAggs, PINOT_ERR_UNSUPPORTED, "1..8 aggregation functions per query");
  require(q.num_group_by >= 1 && q.num_group_by <= kMaxGroupCols, PINOT_ERR_UNSUPPORTED, "1..8 group-by columns");
  Arena ar;
  std::unique_ptr<FilterTreeInput> tree;
  std::vector<SegPlan> plans = plan_all(e, segs, q, ar, tree);
  KeySpace ks = build_key_space(segs, q);
  require(!ks.hashed, PINOT_ERR_UNSUPPORTED,
          "group key space too large for the dense bitset group-by (LONG_MAP/ARRAY_MAP shapes need the fused path)");
  GroupAccs ga = group_acc_kinds(*segs[0], q);
  size_t per_key = 8;
  for (auto b : ga.acc_bytes_per_key) per_key += b;
  size_t free_b = 0, total_b = 0;
  PINOT_HIP(hipMemGetInfo(&free_b, &total_b));
  require((double)ks.G * per_key < 0.5 * (double)free_b, PINOT_ERR_UNSUPPORTED,
          "dense group-by accumulators do not fit in HBM");
  QueryScratch qs = prepare(e, plans, ar);
  e.group_scratch.reserve(ks.G * per_key + 64);
  uint8_t *base = e.group_scratch.get<uint8_t>();
  auto *counts = reinterpret_cast<unsigned long long *>(base);
  std::vector<void *> accs(na, nullptr);
  uint8_t *p = base + ks.G * 8;
  for (int a = 0; a < na; a++) {
    if (ga.acc_kind[a] == 5) continue;
    accs[a] = p;
    p += ks.G * ga.acc_bytes_per_key[a];
  }
  PINOT_HIP(hipEventRecord(e.ev_start, e.stream));
  init_accs(e, ks.G, counts, ga, accs.data());
  Timer t(e);
  std::vector<int64_t> seg_counts;
  accumulate_groups(e, plans, qs, q, ga, ks, counts, accs.data(), t, seg_counts, true);
  GroupByProgram gp{};
  gp.n_aggs = na;
  gp.counts = counts;
  for (int a = 0; a < na; a++) { gp.acc[a] = accs[a]; gp.acc_kind[a] = ga.acc_kind[a]; }
  auto res = finalize_groups(e, q, ga, ks, gp);
  PINOT_HIP(hipEventRecord(e.ev_stop, e.stream));
  wait_stream(e);
  float ms = 0;
  PINOT_HIP(hipEventElapsedTime(&ms, e.ev_start, e.ev_stop));
  t.collect();
  fill_stats(q, plans, seg_counts, ms, stats);
  return res;
}

// ------------------------------------------------------------------ multi-GPU partials
void exec_group_by_layout(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q,
                          pinot_partial_layout *layout) {
  (void)e;
  require(!segs.empty(), PINOT_ERR_BAD_ARG, "no segments");
  require(!touches_mv_group_by(segs, q), PINOT_ERR_UNSUPPORTED, "multi-GPU partials of a multi-value group-by");
  KeySpace ks = build_key_space(segs, q);
  require(!ks.hashed, PINOT_ERR_UNSUPPORTED, "partial group-by needs a dense key space");
  for (auto &per_seg : ks.remap)
    for (auto &m : per_seg)
      require(m.empty(), PINOT_ERR_UNSUPPORTED, "partial group-by needs identical group-by dictionaries");
  GroupAccs ga = group_acc_kinds(*segs[0], q);
  memset(layout, 0, sizeof(*layout));
  layout->num_keys = ks.G;
  layout->num_aggregations = q.num_aggregations;
  for (int a = 0; a < q.num_aggregations && a < 8; a++) layout->acc_kind[a] = ga.acc_kind[a];
  uint64_t fp = 0;
  for (int j = 0; j < q.num_group_by; j++) fp = fp * 1099511628211ull + dictionary_fingerprint(*segs[0]->column(q.group_by[j]));
  layout->group_dictionary_fingerprint = fp;
}

void exec_group_by_partial(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q,
                           int64_t *counts_dev, void *const *accs_dev, pinot_exec_stats *stats) {
  require(!segs.empty(), PINOT_ERR_BAD_ARG, "no segments");
  require(!touches_mv_group_by(segs, q), PINOT_ERR_UNSUPPORTED, "multi-GPU partials of a multi-value group-by");
  KeySpace ks = build_key_space(segs, q);
  require(!ks.hashed, PINOT_ERR_UNSUPPORTED, "partial group-by needs a dense key space");
  GroupAccs ga = group_acc_kinds(*segs[0], q);
  require(!plan_admission(segs, q, e, ks.G).active, PINOT_ERR_UNSUPPORTED,
          "multi-GPU partials with num.groups.limit admission: use the engine's own multi-device group-by");
  if (e.use_fused) {  // the fused sinks, stopped before compaction
    const PartialOut po{counts_dev, accs_dev};
    exec_group_by_fused(e, segs, q, ks, ga, stats, 0, &po);
    return;
  }
  Arena ar;
  std::unique_ptr<FilterTreeInput> tree;
  std::vector<SegPlan> plans = plan_all(e, segs, q, ar, tree);
  QueryScratch qs = prepare(e, plans, ar);
  // the bitset path keeps u32 HLL registers: accumulate them in scratch, narrow into the caller's u8 arrays
  std::vector<void *> accs(accs_dev, accs_dev + q.num_aggregations);
  std::vector<DeviceBuffer> hll_tmp(q.num_aggregations);
  for (int a = 0; a < q.num_aggregations; a++)
    if (ga.acc_kind[a] == 4) {
      hll_tmp[a].alloc((size_t)ks.G * 1024 + 16);
      accs[a] = hll_tmp[a].get();
    }
  PINOT_HIP(hipEventRecord(e.ev_start, e.stream));
  auto *counts = reinterpret_cast<unsigned long long *>(counts_dev);
  init_accs(e, ks.G, counts, ga, accs.data());
  Timer t(e);
  std::vector<int64_t> seg_counts;
  accumulate_groups(e, plans, qs, q, ga, ks, counts, accs.data(), t, seg_counts, false);
  for (int a = 0; a < q.num_aggregations; a++)
    if (ga.acc_kind[a] == 4)
      launch_narrow_u32(hll_tmp[a].get<uint32_t>(), ks.G * 256, static_cast<uint8_t *>(accs_dev[a]), e.stream);
  PINOT_HIP(hipGetLastError());
  PINOT_HIP(hipEventRecord(e.ev_stop, e.stream));
  wait_stream(e);
  float ms = 0;
  PINOT_HIP(hipEventElapsedTime(&ms, e.ev_start, e.ev_stop));
  t.collect();
  fill_stats(q, plans, seg_counts, ms, stats);
}

std::unique_ptr<GroupByResult> exec_group_by_finalize(Engine &e, const std::vector<SegmentData *> &segs,
                                                      const pinot_query &q, const int64_t *counts_dev,
                                                      void *const *accs_dev) {
  KeySpace ks = build_key_space(segs, q);
  require(!ks.hashed, PINOT_ERR_UNSUPPORTED, "partial group-by needs a dense key space");
  GroupAccs ga = group_acc_kinds(*segs[0], q);
  if (e.use_fused) {
    const PartialOut pin{const_cast<int64_t *>(counts_dev), accs_dev};
    pinot_exec_stats st{};
    return exec_group_by_fused(e, segs, q, ks, ga, &st, 0, nullptr, &pin);
  }
  GroupByProgram gp{};
  gp.n_aggs = q.num_aggregations;
  gp.counts = reinterpret_cast<unsigned long long *>(const_cast<int64_t *>(counts_dev));
  std::vector<DeviceBuffer> hll_tmp(q.num_aggregations);  // u8 partial registers -> the u32 layout finalize reads
  for (int a = 0; a < q.num_aggregations; a++) {
    gp.acc[a] = accs_dev ? accs_dev[a] : nullptr;
    gp.acc_kind[a] = ga.acc_kind[a];
    if (ga.acc_kind[a] == 4 && gp.acc[a]) {
      hll_tmp[a].alloc((size_t)ks.G * 1024 + 16);
      launch_widen_u8(static_cast<const uint8_t *>(gp.acc[a]), ks.G * 256, hll_tmp[a].get<int32_t>(), e.stream);
      gp.acc[a] = hll_tmp[a].get();
    }
  }
  PINOT_HIP(hipGetLastError());
  return finalize_groups(e, q, ga, ks, gp);
}

}  // namespace pinot

namespace pinot {

// ------------------------------------------------------------------ pieces of the multi-GPU server (server.cpp)
namespace {

uint64_t ordered_double_key(double d) {  // Double.compare order: -0.0 < 0.0, NaN last
  uint64_t u;
  memcpy(&u, &d, 8);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

struct DictList {  // one group-by column's sorted unique values (the exchange format of local_group_dictionaries)
  int32_t type = -1;                 // pinot_data_type; -1: this rank holds no segment
  std::vector<int64_t> ints;         // INT / LONG
  std::vector<double> dbls;          // FLOAT / DOUBLE (by ordered_double_key)
  std::vector<std::string> strs;     // STRING (by bytes)
  size_t size() const { return type < 0 ? 0 : type <= PINOT_LONG ? ints.size() : type == PINOT_STRING ? strs.size() : dbls.size(); }
};

void sort_unique(DictList &d) {
  if (d.type <= PINOT_LONG) {
    if (!std::is_sorted(d.ints.begin(), d.ints.end()) || std::adjacent_find(d.ints.begin(), d.ints.end()) != d.ints.end()) {
      std::sort(d.ints.begin(), d.ints.end());
      d.ints.erase(std::unique(d.ints.begin(), d.ints.end()), d.ints.end());
    }
  } else if (d.type == PINOT_STRING) {
    std::sort(d.strs.begin(), d.strs.end());
    d.strs.erase(std::unique(d.strs.begin(), d.strs.end()), d.strs.end());
  } else {
    auto lt = [](double a, double b) { return ordered_double_key(a) < ordered_double_key(b); };
    auto eq = [](double a, double b) { return ordered_double_key(a) == ordered_double_key(b); };
    std::sort(d.dbls.begin(), d.dbls.end(), lt);
    d.dbls.erase(std::unique(d.dbls.begin(), d.dbls.end(), eq), d.dbls.end());
  }
}

void put_u64(std::vector<uint8_t> &b, uint64_t v) { b.insert(b.end(), reinterpret_cast<uint8_t *>(&v), reinterpret_cast<uint8_t *>(&v) + 8); }

struct Reader {
  const std::vector<uint8_t> &b;
  size_t p = 0;
  uint64_t u64() {
    require(p + 8 <= b.size(), PINOT_ERR_DEVICE, "group-by dictionary exchange: truncated payload");
    uint64_t v;
    memcpy(&v, b.data() + p, 8);
    p += 8;
    return v;
  }
  std::string str(size_t n) {
    require(p + n <= b.size(), PINOT_ERR_DEVICE, "group-by dictionary exchange: truncated payload");
    std::string s(reinterpret_cast<const char *>(b.data() + p), n);
    p += n;
    return s;
  }
};

bool equals_list(const ColumnData &c, const DictList &u) {
  if ((size_t)c.card != u.size()) return false;
  if (c.data_type <= PINOT_LONG) return c.dict_int == u.ints;
  if (c.data_type == PINOT_STRING) return c.dict_str == u.strs;
  for (int32_t i = 0; i < c.card; i++)
    if (ordered_double_key(c.dict_dbl[i]) != ordered_double_key(u.dbls[i])) return false;
  return true;
}

}  // namespace

std::vector<uint8_t> local_group_dictionaries(const std::vector<SegmentData *> &segs, const pinot_query &q) {
  std::vector<uint8_t> out;
  for (int j = 0; j < q.num_group_by; j++) {
    DictList d;
    const std::string name = q.group_by[j];
    if (!segs.empty()) {
      const ColumnData &c0 = *segs[0]->column(name);
      d.type = c0.data_type;
      bool same = true;
      for (size_t si = 1; si < segs.size(); si++) {
        const ColumnData &c = *segs[si]->column(name);
        require(c.data_type == c0.data_type, PINOT_ERR_BAD_QUERY, "group-by column type differs across segments");
        same = same && same_dictionary(c0, c);
      }
      for (size_t si = 0; si < (same ? 1 : segs.size()); si++) {
        const ColumnData &c = *segs[si]->column(name);
        if (d.type <= PINOT_LONG) d.ints.insert(d.ints.end(), c.dict_int.begin(), c.dict_int.end());
        else if (d.type == PINOT_STRING) d.strs.insert(d.strs.end(), c.dict_str.begin(), c.dict_str.end());
        else d.dbls.insert(d.dbls.end(), c.dict_dbl.begin(), c.dict_dbl.end());
      }
      sort_unique(d);
    }
    put_u64(out, (uint64_t)(int64_t)d.type);
    put_u64(out, d.size());
    if (d.type < 0) continue;
    if (d.type <= PINOT_LONG) {
      for (int64_t v : d.ints) put_u64(out, (uint64_t)v);
    } else if (d.type == PINOT_STRING) {
      for (const std::string &s : d.strs) {
        put_u64(out, s.size());
        out.insert(out.end(), s.begin(), s.end());
      }
    } else {
      for (double v : d.dbls) {
        uint64_t u;
        memcpy(&u, &v, 8);
        put_u64(out, u);
      }
    }
  }
  return out;
}

GlobalKeySpace global_key_space(const std::vector<SegmentData *> &segs, const pinot_query &q,
                                const std::vector<std::vector<uint8_t>> &rank_dicts) {
  const int ng = q.num_group_by;
  std::vector<DictList> u(ng);
  for (const auto &blob : rank_dicts) {
    Reader r{blob};
    for (int j = 0; j < ng; j++) {
      const int32_t type = (int32_t)(int64_t)r.u64();
      const uint64_t n = r.u64();
      if (type < 0) continue;
      require(type <= PINOT_STRING, PINOT_ERR_DEVICE, "group-by dictionary exchange: bad type");
      require(u[j].type < 0 || u[j].type == type, PINOT_ERR_BAD_QUERY, "group-by column type differs across segments");
      u[j].type = type;
      for (uint64_t i = 0; i < n; i++) {
        if (type <= PINOT_LONG) {
          u[j].ints.push_back((int64_t)r.u64());
        } else if (type == PINOT_STRING) {
          const uint64_t len = r.u64();
          u[j].strs.push_back(r.str(len));
        } else {
          const uint64_t bits = r.u64();
          double v;
          memcpy(&v, &bits, 8);
          u[j].dbls.push_back(v);
        }
      }
    }
  }
  GlobalKeySpace ks;
  ks.gvalues.resize(ng);
  ks.remap.assign(segs.size(), std::vector<std::vector<int32_t>>(ng));
  uint64_t fp = 1469598103934665603ull;
  auto mix = [&fp](uint64_t v) {
    for (int i = 0; i < 8; i++) {
      fp ^= (v >> (8 * i)) & 0xFF;
      fp *= 1099511628211ull;
    }
  };
  for (int j = 0; j < ng; j++) {
    DictList &d = u[j];
    if (d.type >= 0) sort_unique(d);
    const size_t n = d.size();
    ks.gcard.push_back((int64_t)n);
    mix((uint64_t)(int64_t)d.type);
    mix(n);
    auto &gv = ks.gvalues[j];
    gv.resize(n);
    for (size_t i = 0; i < n; i++) {  // Dictionary.getStringValue of the value
      if (d.type <= PINOT_LONG) {
        gv[i] = std::to_string(d.ints[i]);
        mix((uint64_t)d.ints[i]);
      } else if (d.type == PINOT_STRING) {
        gv[i] = d.strs[i];
        for (char ch : d.strs[i]) mix((uint8_t)ch);
      } else {
        gv[i] = d.type == PINOT_FLOAT ? java_float_to_string((float)d.dbls[i]) : java_double_to_string(d.dbls[i]);
        mix(ordered_double_key(d.dbls[i]));
      }
    }
    const std::string name = q.group_by[j];
    for (size_t si = 0; si < segs.size(); si++) {
      const ColumnData &c = *segs[si]->column(name);
      if (equals_list(c, d)) continue;  // identity
      auto &m = ks.remap[si][j];
      m.resize(c.card);
      for (int32_t i = 0; i < c.card; i++) {
        size_t g;
        if (d.type <= PINOT_LONG) {
          g = std::lower_bound(d.ints.begin(), d.ints.end(), c.dict_int[i]) - d.ints.begin();
        } else if (d.type == PINOT_STRING) {
          g = std::lower_bound(d.strs.begin(), d.strs.end(), c.dict_str[i]) - d.strs.begin();
        } else {
          const uint64_t key = ordered_double_key(c.dict_dbl[i]);
          g = std::lower_bound(d.dbls.begin(), d.dbls.end(), key,
                               [](double a, uint64_t k) { return ordered_double_key(a) < k; }) - d.dbls.begin();
        }
        require(g < n, PINOT_ERR_DEVICE, "group-by dictionary exchange: a local value is missing from the union");
        m[i] = (int32_t)g;
      }
    }
  }
  ks.fingerprint = fp;
  for (auto g : ks.gcard) {
    if (g == 0) { ks.G = 0; break; }
    if (ks.G > kDenseKeyLimit / g) {
      ks.hashed = true;
      break;
    }
    ks.G *= g;
  }
  return ks;
}

std::vector<int> group_acc_kind_list(const SegmentData &s, const pinot_query &q) { return group_acc_kinds(s, q).acc_kind; }

bool admission_cap_can_bind(const std::vector<SegmentData *> &segs, const pinot_query &q, const Engine &e, int64_t G) {
  return plan_admission(segs, q, e, G).cap_active;
}

void exec_group_by_partial_ks(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q,
                              const std::vector<int64_t> &gcard, const std::vector<std::vector<std::string>> &gvalues,
                              const std::vector<std::vector<std::vector<int32_t>>> &remap, int64_t *counts_dev,
                              void *const *accs_dev, pinot_exec_stats *stats, AdmissionIO *aio) {
  require(e.use_fused, PINOT_ERR_UNSUPPORTED, "multi-GPU group-by runs on the fused path (exec.fused=1)");
  KeySpace ks;
  ks.gcard = gcard;
  ks.gvalues = gvalues;
  ks.remap = remap;
  ks.G = 1;
  for (auto g : gcard) ks.G *= g;
  GroupAccs ga = group_acc_kinds(*segs[0], q);
  std::vector<void *> no_accs(q.num_aggregations, nullptr);  // export: the partial arrays are never touched
  const PartialOut po{counts_dev, accs_dev ? accs_dev : no_accs.data()};
  exec_group_by_fused(e, segs, q, ks, ga, stats, 0, &po, nullptr, true, aio);
}

void inter_segment_cap(std::vector<uint32_t> &bm, size_t S, int64_t words, int64_t cap) {
  apply_inter_segment_cap(bm, S, words, cap);
}

DenseOut slice_outputs(Engine &e, const pinot_query &q, const std::vector<int> &acc_kind, unsigned long long *counts,
                       const std::vector<void *> &accs, int64_t G, int64_t key_base) {
  long long *keys_dev = nullptr;
  const unsigned long long n = slice_compact(e, counts, G, keys_dev);
  std::vector<uint32_t> flags;
  return slice_outputs_keys(e, q, acc_kind, counts, accs, G, key_base, keys_dev, n, 0, flags);
}

unsigned long long slice_compact(Engine &e, const unsigned long long *counts, int64_t G, long long *&keys_dev) {
  keys_dev = nullptr;
  return G > 0 ? compact_dense(e, counts, G, keys_dev, {}) : 0;
}

DenseOut slice_outputs_keys(Engine &e, const pinot_query &q, const std::vector<int> &acc_kind, unsigned long long *counts,
                            const std::vector<void *> &accs, int64_t G, int64_t key_base, const long long *keys_dev,
                            unsigned long long n, int32_t top_n, std::vector<uint32_t> &flags) {
  KeySpace ks;
  ks.G = G;
  GroupAccs ga;
  ga.acc_kind = acc_kind;
  ga.acc_bytes_per_key.assign(acc_kind.size(), 0);
  const std::vector<int> alias(acc_kind.size(), -1);
  DenseGroups dg{&q, &ks, &ga, &ga, &alias, counts, accs, key_base, nullptr};
  flags.clear();
  if (top_n > 0 && n > 0) {  // this range's trimSize best groups per function (every group when it holds no more)
    const int64_t T = std::max<int64_t>(5 * (int64_t)top_n, 5000);
    std::vector<std::vector<int64_t>> kept;
    const long long *ukeys = device_trim(e, dg, keys_dev, n, top_n, kept, T, &flags);
    if (ukeys != keys_dev) return dense_outputs(e, dg, ukeys, n, true, false);
    flags.assign((size_t)n, (uint32_t)((1ull << q.num_aggregations) - 1));
  }
  return dense_outputs(e, dg, keys_dev, n);
}

void server_trim_select(GroupByResult &r, int32_t top_n, const std::vector<uint32_t> &flags, int64_t merged_groups) {
  const int64_t n = (int64_t)r.raw_keys.size();
  require((int64_t)flags.size() == n, PINOT_ERR_DEVICE, "server trim: candidate flags of another size");
  const int64_t T = std::max<int64_t>(5 * (int64_t)top_n, 5000);
  const int na = (int)r.functions.size();
  r.fn_kept.assign(na, {});
  for (int fn = 0; fn < na; fn++) {
    std::vector<int64_t> idx;
    for (int64_t g = 0; g < n; g++)
      if ((flags[g] >> fn) & 1u) idx.push_back(g);
    if ((int64_t)idx.size() > T) {  // GroupByResult::trim's order: the function's value, ties by raw key (group order)
      const int f = sv_function(r.functions[fn]);
      const HostVec<int64_t> &cnt = r.counts[r.counts_shared ? 0 : fn];
      auto val = [&](int64_t g) -> double {
        switch (f) {
          case PINOT_AGG_COUNT: return (double)cnt[g];
          case PINOT_AGG_AVG: return cnt[g] ? r.values[fn][g] / (double)cnt[g] : -INFINITY;
          case PINOT_AGG_DISTINCTCOUNTHLL: return (double)r.hll_card[fn][g];
          default: return r.values[fn][g];
        }
      };
      const bool asc = f == PINOT_AGG_MIN;
      auto better = [&](int64_t a, int64_t b) {
        const double va = val(a), vb = val(b);
        if (va != vb) return asc ? va < vb : va > vb;
        return a < b;
      };
      std::nth_element(idx.begin(), idx.begin() + T, idx.end(), better);
      idx.resize(T);
      std::sort(idx.begin(), idx.end());
    }
    r.fn_kept[fn] = std::move(idx);
  }
  r.trimmed_top_n = top_n;
  r.merged_groups = merged_groups;
}

DenseOut slice_alloc(Engine &e, const pinot_query &q, const std::vector<int> &acc_kind, unsigned long long n) {
  const int na = q.num_aggregations;
  DenseOut o;
  o.n = n;
  o.kind = acc_kind;
  o.derive.assign(na, -1);
  o.hll_off.assign(na, 0);
  o.values.assign(na, nullptr);
  o.cards.assign(na, nullptr);
  int n_card = 0;
  for (int i = 0; i < na; i++) {
    n_card += acc_kind[i] == 4;
    if (acc_kind[i] == 4) o.derive[i] = -2;
  }
  const size_t n8 = n * 8;
  e.group_gather.reserve(n8 * (2 + na + n_card) + 256);
  o.keys = e.group_gather.get<long long>();
  o.counts = o.keys + n;
  double *v = reinterpret_cast<double *>(o.counts + n);
  long long *c = reinterpret_cast<long long *>(v + n * na);
  for (int i = 0; i < na; i++) {
    o.values[i] = v + n * i;
    if (acc_kind[i] == 4) {
      o.cards[i] = c;
      c += n;
    }
  }
  if (n_card && n) {
    const size_t need = (size_t)n_card * n * 256 + 16;
    for (auto &b : e.hll_pool)
      if (b.use_count() == 1 && b->size() >= need) { o.hll = b; break; }
    if (!o.hll) {
      o.hll = std::make_shared<DeviceBuffer>(need + need / 4);
      if (e.hll_pool.size() < 4) e.hll_pool.push_back(o.hll);
    }
    int h = 0;
    for (int i = 0; i < na; i++)
      if (acc_kind[i] == 4) o.hll_off[i] = (size_t)(h++) * n * 256;
  }
  return o;
}

std::vector<std::pair<void *, size_t>> slice_arrays(const DenseOut &o) {
  std::vector<std::pair<void *, size_t>> a;
  a.push_back({o.keys, 8});
  a.push_back({o.counts, 8});
  for (size_t i = 0; i < o.kind.size(); i++) {
    if (o.derive[i] == -1) a.push_back({o.values[i], 8});
    if (o.kind[i] == 4) {
      a.push_back({o.cards[i], 8});
      a.push_back({o.hll ? o.hll->get<uint8_t>() + o.hll_off[i] : nullptr, 256});
    }
  }
  return a;
}

std::unique_ptr<GroupByResult> slice_result(Engine &e, const pinot_query &q, const std::vector<int64_t> &gcard,
                                            const std::vector<std::vector<std::string>> &gvalues, const DenseOut &o) {
  return dense_fetch(e, q, gcard, gvalues, o, nullptr);
}

uint64_t dictionary_fingerprint(const ColumnData &c) {
  uint64_t h = 1469598103934665603ull;  // FNV-1a over (type, cardinality, the BE dictionary bytes)
  auto mix = [&](uint64_t v) {
    for (int i = 0; i < 8; i++) {
      h ^= (v >> (8 * i)) & 0xFF;
      h *= 1099511628211ull;
    }
  };
  mix((uint64_t)c.data_type);
  mix((uint64_t)c.card);
  for (uint8_t b : c.dict_be) {
    h ^= b;
    h *= 1099511628211ull;
  }
  return h;
}

std::vector<SegmentData *> prune_for_query(const std::vector<SegmentData *> &segs, const pinot_query &q) {
  if (!q.pruners || segs.empty()) return segs;
  std::unique_ptr<FilterTreeInput> tree;
  if (q.num_filter_nodes > 0) tree = std::make_unique<FilterTreeInput>(decode_filter(q.num_filter_nodes, q.filter));
  std::vector<SegmentData *> kept;
  for (SegmentData *s : segs)
    if (!prune_segment(*s, q, tree.get(), q.pruners)) kept.push_back(s);
  return kept;
}

std::unique_ptr<GroupByResult> empty_group_result(const pinot_query &q) {
  auto r = std::make_unique<GroupByResult>();
  const int na = q.num_aggregations;
  r->num_columns = q.num_group_by;
  r->counts_shared = true;
  for (int a = 0; a < na; a++) r->functions.push_back(q.aggregations[a].function);
  r->counts.assign(na, {});
  r->values.assign(na, {});
  r->hll.assign(na, {});
  r->hll_card.assign(na, {});
  r->gcard.assign(q.num_group_by, 0);
  r->gvalues.assign(q.num_group_by, {});
  return r;
}

void agg_identities(const pinot_query &q, pinot_agg_result *out) {
  for (int a = 0; a < q.num_aggregations; a++) {
    memset(&out[a], 0, sizeof(pinot_agg_result));
    out[a].has_exact_sum = 1;
    const int f = sv_function(q.aggregations[a].function);
    out[a].value = f == PINOT_AGG_MIN ? INFINITY : f == PINOT_AGG_MAX ? -INFINITY : 0.0;
  }
}

int64_t admission_possible(const std::vector<SegmentData *> &segs, const pinot_query &q, const Engine &e) {
  const AdmissionPlan ap = plan_admission(segs, q, e, INT64_MAX);
  const bool mv = touches_mv_group_by(segs, q);  // a multi-value doc yields several keys: no docs bound
  int64_t possible = 0;
  for (size_t i = 0; i < segs.size(); i++) {
    __int128 product = 1;
    for (int j = 0; j < q.num_group_by; j++) product *= segs[i]->column(q.group_by[j])->card;
    const int64_t reach = (int64_t)std::min<__int128>(product, mv ? (__int128)INT64_MAX : (__int128)segs[i]->num_docs);
    possible += std::min(ap.upper[i], reach);
  }
  return possible;
}

// CombineService.mergeTwoBlocks (:48-90) over per-engine results of the same query: counts add, exact integer
// sums add exactly (any non-exact part makes the sum a double sum), MIN / MAX compare, HLL registers max.
void merge_agg_parts(const pinot_query &q, const std::vector<const pinot_agg_result *> &parts, pinot_agg_result *out) {
  for (int a = 0; a < q.num_aggregations; a++) {
    pinot_agg_result &r = out[a];
    memset(&r, 0, sizeof(r));
    const int f = sv_function(q.aggregations[a].function);  // an MV function merges as its SV form
    __int128 isum = 0;
    double dsum = 0.0;
    bool exact = true;
    double v = f == PINOT_AGG_MIN ? INFINITY : -INFINITY;
    for (const pinot_agg_result *p : parts) {  // Math.min / Math.max: NaN wins, -0.0 < 0.0
      const pinot_agg_result &x = p[a];
      r.count += x.count;
      if (f == PINOT_AGG_SUM || f == PINOT_AGG_AVG) {
        if (x.has_exact_sum) isum += x.exact_sum;
        else { dsum += x.value; exact = false; }
      } else if (f == PINOT_AGG_MIN) {
        v = java_min(v, x.value);
      } else if (f == PINOT_AGG_MAX) {
        v = java_max(v, x.value);
      } else if (f == PINOT_AGG_DISTINCTCOUNTHLL) {
        for (int j = 0; j < 256; j++) r.hll_registers[j] = std::max(r.hll_registers[j], x.hll_registers[j]);
      }
    }
    if (f == PINOT_AGG_SUM || f == PINOT_AGG_AVG) {
      if (exact) {
        r.value = (double)isum;
        if (isum >= INT64_MIN && isum <= INT64_MAX) {
          r.exact_sum = (int64_t)isum;
          r.has_exact_sum = 1;
        }
      } else {
        r.value = dsum + (double)isum;
      }
    } else if (f == PINOT_AGG_MIN || f == PINOT_AGG_MAX) {
      r.value = v;
    } else if (f == PINOT_AGG_DISTINCTCOUNTHLL) {
      r.hll_cardinality = hll_cardinality(r.hll_registers);
    }
  }
}

}  // namespace pinot

namespace pinot {
void exec_group_by_mv_partial(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q,
                              const MvPartial &mp, pinot_exec_stats *stats) {
  exec_group_by_mv(e, segs, q, stats, &mp);
}

// The engine's host task pool for other translation units (datatable.cpp): fn(0) .. fn(n - 1), every task joined.
void host_parallel(size_t n, const std::function<void(size_t)> &fn) { parallel_tasks(n, fn); }
size_t host_parallelism() { return host_threads(); }
}  // namespace pinot
