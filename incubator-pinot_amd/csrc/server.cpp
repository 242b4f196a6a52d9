// Multi-GPU server: the intra-server combine across the GPUs of a node, inside the .so.
//
// Restates, across devices instead of worker threads (PC = pinot-core/src/main/java/org/apache/pinot/core):
//   CombineOperator / CombineService.mergeTwoBlocks   PC/operator/CombineOperator.java:75-196, PC/query/reduce/CombineService.java:48-90
//   CombineGroupByOperator                            PC/operator/CombineGroupByOperator.java:104-228
// Segments are dealt to GPUs by the caller (one engine per GPU holds them in HBM). A query runs every engine's
// share concurrently (one host thread per engine, each on its own stream), then merges on the device:
//   group-by     every engine writes dense partials over the query's GLOBAL key space (union dictionaries across
//                all segments, so per-segment dictionaries may differ), padded to Gp = ceil(G / ranks) * ranks;
//                ONE grouped ncclReduceScatter per array (sum: counts / int64 / double sums; min / max: the
//                order-preserving u64 encodings; max: u8 HLL registers) leaves rank r the merged keys
//                [r * Gp / ranks, (r + 1) * Gp / ranks); each rank compacts and finalizes its own key range, and
//                the host concatenates the ranges (ascending keys) into one result.
//   aggregation  a few scalars per function: merged on the host in a single process, one grouped all-reduce
//                across processes.
// Multi-process form (one process per GPU, e.g. torchrun): before any data collective every rank all-reduces a
// small header (ok flag, key-space size, accumulator kinds, group-by dictionary fingerprint) so a rank that failed
// or disagrees makes every rank fail instead of leaving its peers blocked in a collective.
#include <rccl/rccl.h>

#include <algorithm>
#include <climits>
#include <cstring>
#include <thread>

#include "engine.h"

namespace pinot {

#define PINOT_NCCL(expr)                                                                                 \
  do {                                                                                                   \
    ncclResult_t _r = (expr);                                                                            \
    if (_r != ncclSuccess) throw Error(PINOT_ERR_DEVICE, std::string(#expr) + ": " + ncclGetErrorString(_r)); \
  } while (0)

struct ServerImpl {
  std::vector<std::unique_ptr<pinot_engine>> engines;  // local GPUs
  std::vector<ncclComm_t> comms;                       // one per local engine
  int nranks = 1;                                      // ranks of the communicator
  int rank0 = 0;                                       // rank of local engine 0 (local engine i = rank0 + i)
  bool multi_process = false;
  std::mutex mu;                                       // one server call at a time (engines are locked too)
  std::vector<DeviceBuffer> partial;                   // per engine: dense group-by partials
  std::vector<DeviceBuffer> small;                     // per engine: headers / aggregation partials
  ~ServerImpl() {
    for (auto c : comms)
      if (c) (void)ncclCommDestroy(c);
  }
};

namespace {

// Runs fn(i) for every local engine on its own thread (the device is set for the thread); the first error
// (by engine index) is rethrown after every thread has finished.
void for_engines(ServerImpl &s, const std::function<void(size_t)> &fn) {
  const size_t n = s.engines.size();
  std::vector<std::exception_ptr> err(n);
  auto run = [&](size_t i) {
    try {
      PINOT_HIP(hipSetDevice(s.engines[i]->device));
      fn(i);
    } catch (...) {
      err[i] = std::current_exception();
    }
  };
  if (n == 1) {
    run(0);
  } else {
    std::vector<std::thread> th;
    for (size_t i = 1; i < n; i++) th.emplace_back(run, i);
    run(0);
    for (auto &t : th) t.join();
  }
  for (auto &e : err)
    if (e) std::rethrow_exception(e);
}

std::vector<std::vector<SegmentData *>> segments_by_engine(ServerImpl &s, const std::vector<SegmentRef> &refs,
                                                           std::vector<SegmentData *> &all) {
  std::vector<std::vector<SegmentData *>> per(s.engines.size());
  for (const SegmentRef &r : refs) {
    require(r.engine >= 0 && r.engine < (int)s.engines.size(), PINOT_ERR_BAD_ARG, "segment ref: no such engine");
    SegmentData *sd = &s.engines[r.engine]->seg(r.handle);
    per[r.engine].push_back(sd);
    all.push_back(sd);
  }
  return per;
}

ncclDataType_t acc_type(int kind) {
  switch (kind) {
    case 0: return ncclInt64;
    case 1: return ncclFloat64;
    case 4: return ncclUint8;
    default: return ncclUint64;
  }
}

ncclRedOp_t acc_op(int kind) { return kind == 2 ? ncclMin : (kind == 3 || kind == 4) ? ncclMax : ncclSum; }

size_t acc_unit(int kind) { return kind == 4 ? 256 : kind == 5 ? 0 : 8; }  // bytes per key

// Header agreement across processes: MIN and MAX all-reduce of int64 fields; ranks that do not know a field
// send the identity of the reduction. Throws on every rank when any rank failed or any known field differs.
void agree(ServerImpl &s, std::vector<int64_t> fields, const std::vector<bool> &known, const char *what) {
  const size_t n = fields.size();
  Engine &e = *s.engines[0];
  s.small[0].reserve(n * 16 + 64);
  auto *dmin = s.small[0].get<int64_t>();
  auto *dmax = dmin + n;
  std::vector<int64_t> hmin(n), hmax(n);
  for (size_t i = 0; i < n; i++) {
    hmin[i] = known[i] ? fields[i] : INT64_MAX;
    hmax[i] = known[i] ? fields[i] : INT64_MIN;
  }
  PINOT_HIP(hipMemcpyAsync(dmin, hmin.data(), n * 8, hipMemcpyHostToDevice, e.stream));
  PINOT_HIP(hipMemcpyAsync(dmax, hmax.data(), n * 8, hipMemcpyHostToDevice, e.stream));
  PINOT_NCCL(ncclGroupStart());
  PINOT_NCCL(ncclAllReduce(dmin, dmin, n, ncclInt64, ncclMin, s.comms[0], e.stream));
  PINOT_NCCL(ncclAllReduce(dmax, dmax, n, ncclInt64, ncclMax, s.comms[0], e.stream));
  PINOT_NCCL(ncclGroupEnd());
  PINOT_HIP(hipMemcpyAsync(hmin.data(), dmin, n * 8, hipMemcpyDeviceToHost, e.stream));
  PINOT_HIP(hipMemcpyAsync(hmax.data(), dmax, n * 8, hipMemcpyDeviceToHost, e.stream));
  PINOT_HIP(hipStreamSynchronize(e.stream));
  require(hmin[0] == 1, PINOT_ERR_UNSUPPORTED, std::string(what) + ": a peer rank failed before the merge");
  for (size_t i = 1; i < n; i++)
    require(hmin[i] == hmax[i] || hmin[i] == INT64_MAX, PINOT_ERR_UNSUPPORTED,
            std::string(what) + ": ranks disagree on the query layout (field " + std::to_string(i) + ")");
}

// agree(), surfacing this rank's own failure (if any) rather than the agreement's.
void agree_or_rethrow(ServerImpl &s, const std::vector<int64_t> &fields, const std::vector<bool> &known, const char *what,
                      const std::exception_ptr &local_err) {
  try {
    agree(s, fields, known, what);
  } catch (...) {
    if (local_err) std::rethrow_exception(local_err);
    throw;
  }
}

}  // namespace

ServerImpl *server_create(const int32_t *devices, int32_t n, const char *config) {
  require(devices && n >= 1, PINOT_ERR_BAD_ARG, "at least one device");
  auto s = std::make_unique<ServerImpl>();
  std::vector<int> devs(devices, devices + n);
  for (int d : devs) s->engines.push_back(create_engine(d, config));
  s->comms.assign(n, nullptr);
  PINOT_NCCL(ncclCommInitAll(s->comms.data(), n, devs.data()));
  s->nranks = n;
  s->partial.resize(n);
  s->small.resize(n);
  return s.release();
}

void server_unique_id(uint8_t *id) {
  ncclUniqueId u;
  PINOT_NCCL(ncclGetUniqueId(&u));
  static_assert(sizeof(u) == 128, "ncclUniqueId is 128 bytes");
  memcpy(id, &u, sizeof(u));
}

ServerImpl *server_create_rank(int32_t device, int32_t nranks, int32_t rank, const uint8_t *id,
                                               const char *config) {
  require(id && nranks >= 1 && rank >= 0 && rank < nranks, PINOT_ERR_BAD_ARG, "rank / nranks / unique id");
  auto s = std::make_unique<ServerImpl>();
  s->engines.push_back(create_engine(device, config));
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  s->comms.assign(1, nullptr);
  PINOT_HIP(hipSetDevice(device));
  PINOT_NCCL(ncclCommInitRank(&s->comms[0], nranks, u, rank));
  s->nranks = nranks;
  s->rank0 = rank;
  s->multi_process = nranks > 1;
  s->partial.resize(1);
  s->small.resize(1);
  return s.release();
}

void server_destroy(ServerImpl *s) { delete s; }
int server_num_engines(const ServerImpl &s) { return (int)s.engines.size(); }
Engine *server_engine(ServerImpl &s, int i) {
  require(i >= 0 && i < (int)s.engines.size(), PINOT_ERR_BAD_ARG, "engine index");
  return s.engines[i].get();
}

// ------------------------------------------------------------------ aggregation-only
void server_aggregate(ServerImpl &s, const std::vector<SegmentRef> &refs, const pinot_query &q, pinot_agg_result *out,
                      pinot_exec_stats *stats) {
  std::lock_guard<std::mutex> lk(s.mu);
  std::vector<SegmentData *> all;
  auto per = segments_by_engine(s, refs, all);
  const size_t E = s.engines.size();
  const int na = q.num_aggregations;
  std::vector<std::vector<pinot_agg_result>> parts(E, std::vector<pinot_agg_result>(na));
  std::vector<pinot_exec_stats> st(E);
  std::exception_ptr local_err;
  try {
    for_engines(s, [&](size_t i) {
      memset(&st[i], 0, sizeof(st[i]));
      Engine &e = *s.engines[i];
      std::lock_guard<std::mutex> el(e.mu);
      if (per[i].empty()) {  // identities (MIN +inf, MAX -inf, exact zero sums)
        for (int a = 0; a < na; a++) {
          memset(&parts[i][a], 0, sizeof(pinot_agg_result));
          parts[i][a].has_exact_sum = 1;
          parts[i][a].value = q.aggregations[a].function == PINOT_AGG_MIN   ? INFINITY
                              : q.aggregations[a].function == PINOT_AGG_MAX ? -INFINITY
                                                                            : 0.0;
        }
        return;
      }
      DeadlineScope ds(e, q.timeout_ms);
      exec_aggregate(e, per[i], q, parts[i].data(), &st[i]);
    });
  } catch (...) {
    if (!s.multi_process) throw;
    local_err = std::current_exception();
  }
  std::vector<const pinot_agg_result *> ptrs;
  for (auto &p : parts) ptrs.push_back(p.data());
  merge_agg_parts(q, ptrs, out);
  pinot_exec_stats tot{};
  for (auto &x : st) {
    tot.num_docs_scanned += x.num_docs_scanned;
    tot.num_entries_scanned_in_filter += x.num_entries_scanned_in_filter;
    tot.num_entries_scanned_post_filter += x.num_entries_scanned_post_filter;
    tot.num_total_raw_docs += x.num_total_raw_docs;
    tot.num_segments_processed += x.num_segments_processed;
    tot.num_segments_matched += x.num_segments_matched;
    tot.device_ms = std::max(tot.device_ms, x.device_ms);
  }
  if (s.multi_process) {
    // every rank all-reduces: {ok} agreement first, then per function
    //   int64 SUM [count, exact_sum, non-exact flag] ... + the 6 stats counters, f64 SUM non-exact sums, f64 MIN of
    //   MIN values, f64 MAX of MAX values, u8 MAX HLL registers
    agree_or_rethrow(s, {local_err ? 0 : 1, (int64_t)na}, {true, true}, "aggregation", local_err);
    Engine &e = *s.engines[0];
    const size_t ni = 3 * na + 6, nd = na;
    s.small[0].reserve(8 * (ni + 3 * nd) + 256 * na + 64);
    auto *di = s.small[0].get<int64_t>();
    auto *dsum = reinterpret_cast<double *>(di + ni);
    auto *dmin = dsum + nd;
    auto *dmax = dmin + nd;
    auto *dreg = reinterpret_cast<uint8_t *>(dmax + nd);
    std::vector<int64_t> hi(ni, 0);
    std::vector<double> hs(nd, 0.0), hmn(nd, INFINITY), hmx(nd, -INFINITY);
    std::vector<uint8_t> hr(256 * na, 0);
    for (int a = 0; a < na; a++) {
      hi[3 * a] = out[a].count;
      if (out[a].has_exact_sum) hi[3 * a + 1] = out[a].exact_sum;
      else { hi[3 * a + 2] = 1; hs[a] = out[a].value; }
      if (q.aggregations[a].function == PINOT_AGG_MIN) hmn[a] = out[a].value;
      if (q.aggregations[a].function == PINOT_AGG_MAX) hmx[a] = out[a].value;
      memcpy(&hr[256 * a], out[a].hll_registers, 256);
    }
    const int64_t sv[6] = {tot.num_docs_scanned, tot.num_entries_scanned_in_filter, tot.num_entries_scanned_post_filter,
                           tot.num_total_raw_docs, tot.num_segments_processed, tot.num_segments_matched};
    for (int k = 0; k < 6; k++) hi[3 * na + k] = sv[k];
    PINOT_HIP(hipMemcpyAsync(di, hi.data(), ni * 8, hipMemcpyHostToDevice, e.stream));
    PINOT_HIP(hipMemcpyAsync(dsum, hs.data(), nd * 8, hipMemcpyHostToDevice, e.stream));
    PINOT_HIP(hipMemcpyAsync(dmin, hmn.data(), nd * 8, hipMemcpyHostToDevice, e.stream));
    PINOT_HIP(hipMemcpyAsync(dmax, hmx.data(), nd * 8, hipMemcpyHostToDevice, e.stream));
    PINOT_HIP(hipMemcpyAsync(dreg, hr.data(), hr.size(), hipMemcpyHostToDevice, e.stream));
    PINOT_NCCL(ncclGroupStart());
    PINOT_NCCL(ncclAllReduce(di, di, ni, ncclInt64, ncclSum, s.comms[0], e.stream));
    PINOT_NCCL(ncclAllReduce(dsum, dsum, nd, ncclFloat64, ncclSum, s.comms[0], e.stream));
    PINOT_NCCL(ncclAllReduce(dmin, dmin, nd, ncclFloat64, ncclMin, s.comms[0], e.stream));
    PINOT_NCCL(ncclAllReduce(dmax, dmax, nd, ncclFloat64, ncclMax, s.comms[0], e.stream));
    PINOT_NCCL(ncclAllReduce(dreg, dreg, hr.size(), ncclUint8, ncclMax, s.comms[0], e.stream));
    PINOT_NCCL(ncclGroupEnd());
    PINOT_HIP(hipMemcpyAsync(hi.data(), di, ni * 8, hipMemcpyDeviceToHost, e.stream));
    PINOT_HIP(hipMemcpyAsync(hs.data(), dsum, nd * 8, hipMemcpyDeviceToHost, e.stream));
    PINOT_HIP(hipMemcpyAsync(hmn.data(), dmin, nd * 8, hipMemcpyDeviceToHost, e.stream));
    PINOT_HIP(hipMemcpyAsync(hmx.data(), dmax, nd * 8, hipMemcpyDeviceToHost, e.stream));
    PINOT_HIP(hipMemcpyAsync(hr.data(), dreg, hr.size(), hipMemcpyDeviceToHost, e.stream));
    PINOT_HIP(hipStreamSynchronize(e.stream));
    for (int a = 0; a < na; a++) {
      const int f = q.aggregations[a].function;
      pinot_agg_result &r = out[a];
      r.count = hi[3 * a];
      if (f == PINOT_AGG_SUM || f == PINOT_AGG_AVG) {
        const bool exact = hi[3 * a + 2] == 0;
        r.has_exact_sum = exact ? 1 : 0;
        r.exact_sum = exact ? hi[3 * a + 1] : 0;
        r.value = exact ? (double)hi[3 * a + 1] : hs[a] + (double)hi[3 * a + 1];
      } else if (f == PINOT_AGG_MIN) {
        r.value = hmn[a];
      } else if (f == PINOT_AGG_MAX) {
        r.value = hmx[a];
      } else if (f == PINOT_AGG_DISTINCTCOUNTHLL) {
        memcpy(r.hll_registers, &hr[256 * a], 256);
        r.hll_cardinality = hll_cardinality(r.hll_registers);
      }
    }
    tot.num_docs_scanned = hi[3 * na];
    tot.num_entries_scanned_in_filter = hi[3 * na + 1];
    tot.num_entries_scanned_post_filter = hi[3 * na + 2];
    tot.num_total_raw_docs = hi[3 * na + 3];
    tot.num_segments_processed = hi[3 * na + 4];
    tot.num_segments_matched = hi[3 * na + 5];
  }
  if (stats) *stats = tot;
}

// ------------------------------------------------------------------ group-by
std::unique_ptr<GroupByResult> server_group_by(ServerImpl &s, const std::vector<SegmentRef> &refs, const pinot_query &q,
                                               pinot_exec_stats *stats) {
  std::lock_guard<std::mutex> lk(s.mu);
  std::vector<SegmentData *> all;
  auto per = segments_by_engine(s, refs, all);
  const size_t E = s.engines.size();
  const int na = q.num_aggregations;
  require(na >= 1 && na <= kMaxAggs, PINOT_ERR_UNSUPPORTED, "1..8 aggregation functions per query");
  require(q.num_group_by >= 1 && q.num_group_by <= kMaxGroupCols, PINOT_ERR_UNSUPPORTED, "1..16 group-by columns");
  // global key space and layout (multi process: local, then agreed with the peers)
  std::vector<int64_t> gcard;
  std::vector<std::vector<std::string>> gvalues;
  std::vector<std::vector<std::vector<int32_t>>> remap;
  int64_t G = 0;
  bool hashed = false;
  std::vector<int> kinds;
  uint64_t fp = 0;
  std::exception_ptr local_err;
  try {
    require(!all.empty(), PINOT_ERR_UNSUPPORTED, "multi-GPU group-by: every rank must hold at least one segment");
    build_global_key_space(all, q, gcard, gvalues, remap, G, hashed);
    require(!hashed, PINOT_ERR_UNSUPPORTED, "multi-GPU group-by needs a dense key space (LONG_MAP / ARRAY_MAP shapes: one GPU)");
    require(!admission_cap_can_bind(all, q, *s.engines[0], G), PINOT_ERR_UNSUPPORTED,
            "multi-GPU group-by where the 2 x num.groups.limit inter-segment cap can bind: one GPU");
    kinds = group_acc_kind_list(*all[0], q);
    if (s.multi_process)  // the union dictionary is local to this process: the peers must hold the same one
      for (int j = 0; j < q.num_group_by; j++) {
        const ColumnData &c = *all[0]->column(q.group_by[j]);
        fp = fp * 1099511628211ull + dictionary_fingerprint(c);
        for (auto *sd : all)
          require(dictionary_fingerprint(*sd->column(q.group_by[j])) == dictionary_fingerprint(c), PINOT_ERR_UNSUPPORTED,
                  "multi-process group-by needs identical group-by dictionaries on every segment");
      }
  } catch (...) {
    if (!s.multi_process) throw;
    local_err = std::current_exception();
  }
  if (s.multi_process) {
    std::vector<int64_t> h = {local_err ? 0 : 1, G, (int64_t)na, (int64_t)(fp & 0x7FFFFFFFFFFFFFFFull)};
    for (int a = 0; a < na; a++) h.push_back(local_err ? 0 : kinds[a]);
    std::vector<bool> known(h.size(), !local_err);
    known[0] = true;
    agree_or_rethrow(s, h, known, "group-by layout", local_err);
  }
  const int64_t slice = (G + s.nranks - 1) / s.nranks, Gp = slice * s.nranks;
  // per engine: dense partials over [0, G), identities on the padding [G, Gp)
  std::vector<std::vector<void *>> accs(E, std::vector<void *>(na, nullptr));
  std::vector<unsigned long long *> counts(E, nullptr);
  std::vector<pinot_exec_stats> st(E);
  try {
    for_engines(s, [&](size_t i) {
      memset(&st[i], 0, sizeof(st[i]));
      Engine &e = *s.engines[i];
      std::lock_guard<std::mutex> el(e.mu);
      DeadlineScope ds(e, q.timeout_ms);
      size_t bytes = (size_t)Gp * 8 + 256;
      for (int a = 0; a < na; a++) bytes += ((size_t)Gp * acc_unit(kinds[a]) + 255) / 256 * 256;
      s.partial[i].reserve(bytes);
      uint8_t *p = s.partial[i].get<uint8_t>();
      counts[i] = reinterpret_cast<unsigned long long *>(p);
      p += ((size_t)Gp * 8 + 255) / 256 * 256;
      for (int a = 0; a < na; a++) {
        if (kinds[a] == 5) continue;
        accs[i][a] = p;
        p += ((size_t)Gp * acc_unit(kinds[a]) + 255) / 256 * 256;
      }
      const int64_t from = per[i].empty() ? 0 : G;  // identities: everything, or the padding only
      PINOT_HIP(hipMemsetAsync(counts[i] + from, 0, (size_t)(Gp - from) * 8, e.stream));
      for (int a = 0; a < na; a++)
        if (accs[i][a])
          PINOT_HIP(hipMemsetAsync(static_cast<uint8_t *>(accs[i][a]) + (size_t)from * acc_unit(kinds[a]),
                                   kinds[a] == 2 ? 0xFF : 0, (size_t)(Gp - from) * acc_unit(kinds[a]), e.stream));
      if (!per[i].empty()) {
        std::vector<std::vector<std::vector<int32_t>>> rm;  // this engine's segments' remap rows
        for (auto *sd : per[i]) rm.push_back(remap[std::find(all.begin(), all.end(), sd) - all.begin()]);
        exec_group_by_partial_ks(e, per[i], q, gcard, gvalues, rm, reinterpret_cast<int64_t *>(counts[i]), accs[i].data(),
                                 &st[i]);
      }
      PINOT_HIP(hipStreamSynchronize(e.stream));
    });
  } catch (...) {
    if (!s.multi_process) throw;
    local_err = std::current_exception();
  }
  if (s.multi_process) agree_or_rethrow(s, {local_err ? 0 : 1}, {true}, "group-by partials", local_err);
  // merge: in-place reduce-scatter of every array; rank r keeps [r * slice, (r + 1) * slice)
  PINOT_NCCL(ncclGroupStart());
  for (size_t i = 0; i < E; i++) {
    Engine &e = *s.engines[i];
    const int64_t r = s.rank0 + (int64_t)i;
    PINOT_NCCL(ncclReduceScatter(counts[i], counts[i] + r * slice, slice, ncclUint64, ncclSum, s.comms[i], e.stream));
    for (int a = 0; a < na; a++) {
      if (!accs[i][a]) continue;
      const size_t unit = acc_unit(kinds[a]);
      const size_t cnt = (size_t)slice * (kinds[a] == 4 ? 256 : 1);
      uint8_t *base = static_cast<uint8_t *>(accs[i][a]);
      PINOT_NCCL(ncclReduceScatter(base, base + (size_t)r * slice * unit, cnt, acc_type(kinds[a]), acc_op(kinds[a]),
                                   s.comms[i], e.stream));
    }
  }
  PINOT_NCCL(ncclGroupEnd());
  // owner finalize of each local key range, concurrently
  std::vector<std::unique_ptr<GroupByResult>> res(E);
  for_engines(s, [&](size_t i) {
    Engine &e = *s.engines[i];
    std::lock_guard<std::mutex> el(e.mu);
    PINOT_HIP(hipStreamSynchronize(e.stream));
    const int64_t r = s.rank0 + (int64_t)i, base = r * slice;
    const int64_t g = std::max<int64_t>(0, std::min<int64_t>(slice, G - base));
    std::vector<void *> sl(na, nullptr);
    for (int a = 0; a < na; a++)
      if (accs[i][a]) sl[a] = static_cast<uint8_t *>(accs[i][a]) + (size_t)base * acc_unit(kinds[a]);
    res[i] = exec_group_by_slice(e, q, kinds, gcard, gvalues, counts[i] + base, sl, g, base);
  });
  // one result: the key ranges in rank order are ascending
  auto out = std::move(res[0]);
  for (size_t i = 1; i < E; i++) {
    GroupByResult &x = *res[i];
    const int64_t off = (int64_t)out->raw_keys.size();
    out->raw_keys.insert(out->raw_keys.end(), x.raw_keys.begin(), x.raw_keys.end());
    if (!out->counts.empty() && !x.counts.empty())
      out->counts[0].insert(out->counts[0].end(), x.counts[0].begin(), x.counts[0].end());
    for (int a = 0; a < na; a++) {
      out->values[a].insert(out->values[a].end(), x.values[a].begin(), x.values[a].end());
      out->hll_card[a].insert(out->hll_card[a].end(), x.hll_card[a].begin(), x.hll_card[a].end());
    }
    for (HllPart &p : x.hll_parts) {
      p.group_begin += off;
      out->hll_parts.push_back(std::move(p));
    }
  }
  out->counts_shared = true;
  pinot_exec_stats tot{};
  for (auto &x : st) {
    tot.num_docs_scanned += x.num_docs_scanned;
    tot.num_entries_scanned_in_filter += x.num_entries_scanned_in_filter;
    tot.num_entries_scanned_post_filter += x.num_entries_scanned_post_filter;
    tot.num_total_raw_docs += x.num_total_raw_docs;
    tot.num_segments_processed += x.num_segments_processed;
    tot.num_segments_matched += x.num_segments_matched;
    tot.device_ms = std::max(tot.device_ms, x.device_ms);
  }
  if (stats) *stats = tot;
  return out;
}

}  // namespace pinot
