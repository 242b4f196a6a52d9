// Group-by on one GPU: the key space, accumulator plans and holders (DictionaryBasedGroupKeyGenerator), the fused
// group-by plans (LDS-privatised, HBM atomics, partitioned, ring, hashed), the dense back half (compaction, per-group
// outputs, the device trim) and the host result pool / task pool. Split from executor.cpp (see exec_internal.h).
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

AdmissionPlan plan_admission(const std::vector<SegmentData *> &segs, const pinot_query &q, const Engine &e, int64_t G);
AdmissionBuffers admission_buffers(Engine &e, size_t S, int64_t G);
void build_admitted(Engine &e, const AdmissionPlan &ap, size_t S, int64_t G, const AdmissionBuffers &ab);

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
                                               const KeySpace &ks, GroupByProgram gp, const MvHash *mh) {
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

// Result-array pool: a 1 M-group result is ~48 MB of fresh host pages, and first-touching them cost more than
// filling them. Released results hand their arrays back; the next large result takes them (capacity kept).

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

void parallel_tasks(size_t n, const std::function<void(size_t)> &fn);

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

// Runs fn(0..n-1) on up to n threads (the calling thread takes task 0).

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

size_t host_threads() { return std::min<size_t>(16, TaskPool::get().threads()); }

void set_host_spin(int pauses) { g_pool_spin.store(std::max(0, pauses), std::memory_order_relaxed); }

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

// extra(pinned) issues the caller's own small D2H reads into pinned[0, 4096) (read back after the wait).
unsigned long long compact_dense(Engine &e, const unsigned long long *counts, int64_t G, long long *&keys_dev,
                                 const std::function<void(uint8_t *)> &extra, size_t extra_bytes) {
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
                       bool gather_hll, bool compact_ok, bool serialize_hll) {
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
                                                  unsigned long long n, bool subset) {
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
                             int32_t top_n, std::vector<std::vector<int64_t>> &kept, int64_t min_groups,
                             std::vector<uint32_t> *flags_out) {
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
                                                   int attempt, const PartialOut *po,
                                                   const PartialOut *pin, bool allow_admission,
                                                   AdmissionIO *aio) {
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
  // GB_LDS with <= 3 read columns: a filter of at most one scan leaf per segment (<= 12 bits) evaluated per quarter
  // from its own lane-owns-quarter loads (GroupArgs.qfilter): no LDS chunk staging
  if (gp.mode == GB_LDS && a.lw == 2 && a.pf_nc > 0 && a.pf_nc <= 3 && a.emit_block != 256 && e.group_lds_qfilter &&
      !pin) {
    bool qf = true;
    for (const GroupSegment &g : gsegs) {
      if (g.nwords == 0) continue;
      qf = qf && g.n_leaves <= 1;
      for (int i = 0; i < g.n_leaves && qf; i++) {
        const FusedStep &l = leaves[g.first_leaf + i];
        qf = l.join == JOIN_NEW && l.bits <= kGroupMaxFusedLeafBits &&
             (l.kind == FK_LEAF_RANGE || l.kind == FK_LEAF_LUT64 || l.kind == FK_LEAF_LUT);
      }
    }
    if (qf) {
      a.qfilter = 1;
      a.stage_bytes = 0;
    }
  }
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
    rr.hll_sums = po && !po->hll_sum_room ? 0 : 1;  // the engine's HLL arrays have room for the sums (a caller's if said)
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
    const bool sums = ring_status && po->hll_sum_room;
    for (int i = 0; i < na; i++)
      if (alias[i] >= 0 && ga.acc_kind[i] != 5 && po->accs[i] != po->accs[alias[i]])
        PINOT_HIP(hipMemcpyAsync(po->accs[i], po->accs[alias[i]], ks.G * (ga.acc_kind[i] == 4 ? (sums ? 264 : 256) : 8),
                                 hipMemcpyDeviceToDevice, e.stream));
    PINOT_HIP(hipGetLastError());
    std::vector<unsigned long long> hm(S);
    uint32_t rs[4] = {0, 0, 0, 0};
    e.d2h_small.reserve(S * 8 + 64);  // pinned: asynchronous copies, one wait
    uint8_t *pin = e.d2h_small.get<uint8_t>();
    PINOT_HIP(hipMemcpyAsync(pin, matched, S * 8, hipMemcpyDeviceToHost, e.stream));
    if (ring_status) PINOT_HIP(hipMemcpyAsync(pin + S * 8, ring_status, 16, hipMemcpyDeviceToHost, e.stream));
    PINOT_HIP(hipEventRecord(e.ev_stop, e.stream));
    wait_stream(e);
    memcpy(hm.data(), pin, S * 8);
    if (ring_status) memcpy(rs, pin + S * 8, 16);
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
    if (po->hll_sums_written) *po->hll_sums_written = sums;
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

}  // namespace pinot
