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
#include "exec_internal.h"

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

// Device scratch of a query: arena capacity (arena + `extra` bytes the caller appends once device
// addresses are known) and bitset slots, one region for all segments (run one after the other) or one
// region per segment (fused path: every `pre` bitset must exist when the single kernel runs).
QueryScratch prepare_scratch(Engine &e, const std::vector<SegPlan> &plans, const Arena &ar, bool per_segment,
                             size_t extra) {
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

// Runs the filter steps of one segment. Returns the final bitset (slot 0), or nullptr for MATCH_ALL.
const uint64_t *run_filter(Engine &e, SegPlan &p, const QueryScratch &qs, Timer &t, int64_t region) {
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

// Per segment, as the reference plans each segment on its own (AggregationPlanNode / AggregationGroupByPlanNode:
// StarTreeUtils.isFitForStarTree over that segment's trees).
bool star_plan_fits(const Engine &e, const SegmentData &seg, const pinot_query &q) {
  if (!e.use_star_tree) return false;
  int slots = q.num_aggregations;  // each AVG adds its AvgPair count column
  for (int a = 0; a < q.num_aggregations; a++) slots += q.aggregations[a].function == PINOT_AGG_AVG;
  return slots <= kMaxAggs && star_tree_fits(seg, q);
}

bool star_plan(const Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q) {
  for (SegmentData *s : segs)
    if (!star_plan_fits(e, *s, q)) return false;
  return true;
}

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
}  // namespace pinot
