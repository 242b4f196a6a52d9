// Group-by beyond the fused single-value plans: multi-value group columns and functions, star-tree group-by, the
// bitset-path (legacy) plan, the group-by dispatch (exec_group_by) and the torch-level partial / finalize entry
// points. Split from executor.cpp (see exec_internal.h).
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


// Group-by with multi-value group columns or MV functions: per segment the filter's bitset and one k_group_by_mv
// (every doc's cartesian product of group keys, DictionaryBasedGroupKeyGenerator's MV branch) into dense
// accumulators over the global key space, then the bitset path's finalisation. AvgMV needs its entry count beside
// its sum: a hidden CountMV accumulator per AvgMV, folded into the function's counts after finalisation. num.groups.limit:
// first-appearance admission per segment, then the 2 x limit cap (here, or the server's across ranks: `mp`).
std::unique_ptr<GroupByResult> exec_group_by_mv(Engine &e, const std::vector<SegmentData *> &segs,
                                                const pinot_query &q, pinot_exec_stats *stats,
                                                const MvPartial *mp, int attempt) {
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
