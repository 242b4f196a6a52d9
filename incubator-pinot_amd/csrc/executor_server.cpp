// The multi-GPU server's host pieces (server.cpp calls them): the group-by dictionary exchange and global key space,
// the per-rank partials over it, the owner ranks' key-range outputs and trim, the aggregation merge. Split from
// executor.cpp (see exec_internal.h).
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
                              void *const *accs_dev, pinot_exec_stats *stats, AdmissionIO *aio, bool hll_sum_room,
                              bool *hll_sums_written) {
  require(e.use_fused, PINOT_ERR_UNSUPPORTED, "multi-GPU group-by runs on the fused path (exec.fused=1)");
  KeySpace ks;
  ks.gcard = gcard;
  ks.gvalues = gvalues;
  ks.remap = remap;
  ks.G = 1;
  for (auto g : gcard) ks.G *= g;
  GroupAccs ga = group_acc_kinds(*segs[0], q);
  std::vector<void *> no_accs(q.num_aggregations, nullptr);  // export: the partial arrays are never touched
  if (hll_sums_written) *hll_sums_written = false;
  const PartialOut po{counts_dev, accs_dev ? accs_dev : no_accs.data(), hll_sum_room && accs_dev, hll_sums_written};
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
                            unsigned long long n, int32_t top_n, std::vector<uint32_t> &flags,
                            const std::vector<int64_t> *gcard, const std::vector<const void *> *hll_sum) {
  KeySpace ks;
  ks.G = G;
  if (gcard) ks.gcard = *gcard;
  GroupAccs ga;
  ga.acc_kind = acc_kind;
  ga.acc_bytes_per_key.assign(acc_kind.size(), 0);
  const std::vector<int> alias(acc_kind.size(), -1);
  DenseGroups dg{&q, &ks, &ga, &ga, &alias, counts, accs, key_base, nullptr};
  if (hll_sum) dg.hll_sum = *hll_sum;
  const bool serialize = gcard != nullptr;  // a trimmed subset only, as build_dense_result does
  flags.clear();
  if (top_n > 0 && n > 0) {  // this range's trimSize best groups per function (every group when it holds no more)
    const int64_t T = std::max<int64_t>(5 * (int64_t)top_n, 5000);
    std::vector<std::vector<int64_t>> kept;
    const long long *ukeys = device_trim(e, dg, keys_dev, n, top_n, kept, T, &flags);
    if (ukeys != keys_dev) return dense_outputs(e, dg, ukeys, n, true, false, serialize);
    flags.assign((size_t)n, (uint32_t)((1ull << q.num_aggregations) - 1));
  }
  return dense_outputs(e, dg, keys_dev, n);  // (every group: the host writes the DataTable, as the engine's does)
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
  // (+ room after the arrays for the key tuples of slice_serialize)
  e.group_gather.reserve(n8 * (2 + na + n_card) + 256 + n * (size_t)q.num_group_by * 4 + 16);
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

void launch_hll_getbytes(const uint8_t *regs, long long n, uint8_t *out, hipStream_t stream);  // hll_serde.hip

void slice_serialize(Engine &e, const pinot_query &q, const std::vector<int64_t> &gcard, DenseOut &o) {
  const unsigned long long n = o.n;
  const int na = q.num_aggregations, nc = q.num_group_by;
  if (!n) return;
  int n_card = 0;
  for (int i = 0; i < na; i++) n_card += o.kind[i] == 4;
  if (nc <= kDigitsMaxCols && (int)gcard.size() == nc) {  // the gathered keys are global raw keys (key base 0)
    KeyDigits kd{};
    kd.nc = nc;
    for (int j = 0; j < nc; j++) kd.card[j] = gcard[j];
    o.key_ids = reinterpret_cast<int32_t *>(reinterpret_cast<uint8_t *>(o.keys) + n * 8 * (size_t)(2 + na + n_card));
    launch_key_digits(o.keys, (long long)n, 0, kd, o.key_ids, e.stream);
  }
  if (o.hll && n_card) {
    const size_t need = (size_t)n_card * n * 180 + 16;
    if (!e.hll_ser || e.hll_ser.use_count() > 1 || e.hll_ser->size() < need)
      e.hll_ser = std::make_shared<DeviceBuffer>(need + need / 4);
    o.hll_ser = e.hll_ser;
    o.hll_ser_off.assign(na, 0);
    int s = 0;
    for (int i = 0; i < na; i++)
      if (o.kind[i] == 4) {
        o.hll_ser_off[i] = (size_t)(s++) * n * 180;
        launch_hll_getbytes(o.hll->get<uint8_t>() + o.hll_off[i], (long long)n, o.hll_ser->get<uint8_t>() + o.hll_ser_off[i],
                            e.stream);
      }
  }
  PINOT_HIP(hipGetLastError());
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
