// Multi-GPU server: the intra-server combine across the GPUs of a node, inside the .so.
//
// Restates, across devices instead of worker threads (PC = pinot-core/src/main/java/org/apache/pinot/core):
//   ServerQueryExecutorV1Impl.processQuery  PC/query/executor/ServerQueryExecutorV1Impl.java:100-267 (prune -> plan ->
//                                           run -> statistics, totalDocs over every segment, :183-216)
//   CombineOperator / CombineService        PC/operator/CombineOperator.java:75-196, PC/query/reduce/CombineService.java:48-90
//   CombineGroupByOperator                  PC/operator/CombineGroupByOperator.java:104-228
// Every GPU is a rank of one communicator (collective.h): RCCL over xGMI (ncclCommInitAll for the GPUs of one
// process, ncclCommInitRank for one process per GPU), or the one-device loopback. Each rank serves the segments it
// holds (segments are dealt to GPUs by the caller) and every rank — with or without segments — runs the same
// protocol, so no rank is ever left waiting in a collective:
//   aggregation  prune + run locally, then ONE all-gather of every rank's status, statistics and partial results;
//                every rank merges them in rank order (identities for a rank whose segments were all pruned).
//   group-by     A  prune, this rank's group-by dictionaries (union over its segments), accumulator kinds, the
//                   docs the num.groups.limit admission can reach -> all-gather: any failure fails every rank with the
//                   failing rank's status; the union of every rank's dictionaries is the global key space (each
//                   local segment gets a dictId -> global id remap) and Gp = ceil(G / ranks) * ranks
//                B  dense partials over [0, G) (identities on the padding, or everywhere for a rank without segments)
//                   -> all-gather of the status and statistics
//                C  ONE grouped reduce-scatter per array (sum: counts / sums; min / max: order-preserving u64
//                   encodings; max: u8 HLL registers): rank r keeps the merged keys [r * Gp / ranks, (r + 1) * Gp / ranks)
//                D  each rank compacts and finalizes its key range on its GPU (the one-GPU back half), then the key
//                   ranges are gathered to rank 0 (server.gather=1, the default), which returns the whole result —
//                   ranges ascend with the rank, so the concatenation is in raw-key order — while the other ranks
//                   return an empty one; server.gather=0: every rank returns its own range.
#include "collective.h"

#include <algorithm>
#include <atomic>
#include <climits>
#include <cmath>
#include <cstring>
#include <sstream>
#include <thread>
#include <unordered_map>

#include "engine.h"

namespace pinot {

// The last group-by's global key space of one local engine (phase A's union dictionaries, global values and local
// remaps), reused while its inputs are the same: this rank's segments (process-unique ids: their dictionaries never
// change), the group columns and every rank's exchanged dictionaries, byte for byte.
struct KeySpaceCache {
  std::vector<uint64_t> uids;
  std::vector<std::string> cols;
  std::vector<std::vector<uint8_t>> dicts;
  std::shared_ptr<const GlobalKeySpace> ks;
};

struct ServerImpl {
  std::vector<std::unique_ptr<pinot_engine>> engines;  // local GPUs (local engine i is rank rank0 + i)
  std::vector<std::unique_ptr<Collective>> comms;      // one per local engine (destroyed before the engines)
  int nranks = 1;
  int rank0 = 0;
  bool gather = true;                                  // group-by: the whole result on rank 0
  std::mutex mu;                                       // one server call at a time (engines are locked too)
  std::vector<DeviceBuffer> partial;                   // per engine: dense group-by partials
  std::vector<KeySpaceCache> ks_cache;                 // per engine
  double phase_ms[kServerPhases] = {};                 // last query, local engine 0's rank (server_last_phases)
};

namespace {

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t) { return std::chrono::duration<double, std::milli>(Clock::now() - t).count(); }

std::shared_ptr<const GlobalKeySpace> key_space_cached(KeySpaceCache &c, const std::vector<SegmentData *> &segs,
                                                       const pinot_query &q,
                                                       const std::vector<std::vector<uint8_t>> &dicts) {
  std::vector<uint64_t> uids;
  for (const SegmentData *sg : segs) uids.push_back(sg->uid);
  std::vector<std::string> cols;
  for (int j = 0; j < q.num_group_by; j++) cols.emplace_back(q.group_by[j]);
  if (c.ks && c.uids == uids && c.cols == cols && c.dicts == dicts) return c.ks;
  auto ks = std::make_shared<const GlobalKeySpace>(global_key_space(segs, q, dicts));
  c.uids = std::move(uids);
  c.cols = std::move(cols);
  c.dicts = dicts;
  c.ks = ks;
  return ks;
}

// phase timer of local engine 0 (the other engines' threads pass nullptr)
struct Phases {
  double *ms;
  Clock::time_point t0 = Clock::now(), last = t0;
  explicit Phases(double *m) : ms(m) {
    if (ms) std::fill(ms, ms + kServerPhases, 0.0);
  }
  void mark(int i) {
    const auto now = Clock::now();
    if (ms) ms[i] += std::chrono::duration<double, std::milli>(now - last).count();
    last = now;
  }
  ~Phases() {
    if (ms) ms[kServerPhases - 1] = ms_since(t0);
  }
};

struct ServerConfig {
  bool loopback = false;
  bool gather = true;
  int timeout_ms = 300000;  // in-process rendezvous: a rank that does not arrive fails the call
  std::string engine;       // the remaining keys, for the engines
};

ServerConfig parse_server_config(const char *config) {
  ServerConfig c;
  if (!config) return c;
  std::stringstream ss(config);
  std::string kv, rest;
  while (std::getline(ss, kv, ';')) {
    const auto p = kv.find('=');
    const std::string k = p == std::string::npos ? kv : kv.substr(0, p), v = p == std::string::npos ? "" : kv.substr(p + 1);
    if (k == "server.loopback") c.loopback = v == "1" || v == "true";
    else if (k == "server.gather") c.gather = v == "1" || v == "true";
    else if (k == "server.timeout_ms") c.timeout_ms = std::stoi(v);
    else if (!kv.empty()) rest += (rest.empty() ? "" : ";") + kv;
  }
  require(c.timeout_ms > 0, PINOT_ERR_BAD_ARG, "server.timeout_ms must be positive");
  c.engine = rest;
  return c;
}

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

CType acc_ctype(int kind) { return kind == 0 ? CType::I64 : kind == 1 ? CType::F64 : kind == 4 ? CType::U8 : CType::U64; }
COp acc_op(int kind) { return kind == 2 ? COp::MIN : (kind == 3 || kind == 4) ? COp::MAX : COp::SUM; }
size_t acc_unit(int kind) { return kind == 4 ? 256 : kind == 5 ? 0 : 8; }  // bytes per key

// ---- the control payloads every rank all-gathers (plain bytes: same build on every rank)
struct Status {
  int32_t status = PINOT_OK;
  std::string msg;
};

Status capture(const std::function<void()> &fn) {
  Status s;
  try {
    fn();
  } catch (const Error &e) {
    s.status = e.status;
    s.msg = e.what();
  } catch (const std::bad_alloc &) {
    s.status = PINOT_ERR_OOM;
    s.msg = "host out of memory";
  } catch (const std::exception &e) {
    s.status = PINOT_ERR_DEVICE;
    s.msg = e.what();
  }
  if (s.status == PINOT_OK) s.msg.clear();
  return s;
}

struct Writer {
  std::vector<uint8_t> b;
  void raw(const void *p, size_t n) { b.insert(b.end(), static_cast<const uint8_t *>(p), static_cast<const uint8_t *>(p) + n); }
  void i64(int64_t v) { raw(&v, 8); }
  void f64(double v) { raw(&v, 8); }
  void str(const std::string &s) {
    i64((int64_t)s.size());
    raw(s.data(), s.size());
  }
  void bytes(const std::vector<uint8_t> &v) {
    i64((int64_t)v.size());
    raw(v.data(), v.size());
  }
};

struct Reader {
  const std::vector<uint8_t> &b;
  size_t p = 0;
  void raw(void *out, size_t n) {
    require(p + n <= b.size(), PINOT_ERR_DEVICE, "server communicator: truncated control payload");
    memcpy(out, b.data() + p, n);
    p += n;
  }
  int64_t i64() {
    int64_t v;
    raw(&v, 8);
    return v;
  }
  double f64() {
    double v;
    raw(&v, 8);
    return v;
  }
  std::string str() {
    const int64_t n = i64();
    require(n >= 0 && p + (size_t)n <= b.size(), PINOT_ERR_DEVICE, "server communicator: bad control payload");
    std::string s(reinterpret_cast<const char *>(b.data() + p), (size_t)n);
    p += (size_t)n;
    return s;
  }
  std::vector<uint8_t> bytes() {
    const int64_t n = i64();
    require(n >= 0 && p + (size_t)n <= b.size(), PINOT_ERR_DEVICE, "server communicator: bad control payload");
    std::vector<uint8_t> v(b.begin() + p, b.begin() + p + n);
    p += (size_t)n;
    return v;
  }
};

void put_status(Writer &w, const Status &s) {
  w.i64(s.status);
  w.str(s.msg);
}
Status get_status(Reader &r) {
  Status s;
  s.status = (int32_t)r.i64();
  s.msg = r.str();
  return s;
}

void put_stats(Writer &w, const pinot_exec_stats &s) {
  w.i64(s.num_docs_scanned);
  w.i64(s.num_entries_scanned_in_filter);
  w.i64(s.num_entries_scanned_post_filter);
  w.i64(s.num_total_raw_docs);
  w.i64(s.num_segments_processed);
  w.i64(s.num_segments_matched);
  w.f64(s.device_ms);
}
void add_stats(Reader &r, pinot_exec_stats &t) {
  t.num_docs_scanned += r.i64();
  t.num_entries_scanned_in_filter += r.i64();
  t.num_entries_scanned_post_filter += r.i64();
  t.num_total_raw_docs += r.i64();
  t.num_segments_processed += r.i64();
  t.num_segments_matched += r.i64();
  t.device_ms = std::max(t.device_ms, r.f64());
}

// Every rank's status (rank order) -> the same failure on every rank: this rank's own error first, else the first
// failing rank's status with its message.
void fail_together(const std::vector<Status> &all, int my_rank, const char *what) {
  if (all[my_rank].status != PINOT_OK) throw Error((pinot_status)all[my_rank].status, all[my_rank].msg);
  for (size_t r = 0; r < all.size(); r++)
    if (all[r].status != PINOT_OK)
      throw Error((pinot_status)all[r].status, std::string(what) + ": rank " + std::to_string(r) + " failed: " + all[r].msg);
}

// ---- hashed key spaces across ranks (LONG_MAP / ARRAY_MAP holders, SV or MV group columns)
// One segment's groups as they travel to rank 0: key string, then per function its count (docs, or entries for the
// MV functions), value and, for DISTINCTCOUNTHLL / DISTINCTCOUNTHLLMV, the 256 registers.
bool is_hll_fn(int f) { return f == PINOT_AGG_DISTINCTCOUNTHLL || f == PINOT_AGG_DISTINCTCOUNTHLLMV; }

void put_groups(Writer &w, const GroupByResult &r) {
  const int64_t n = (int64_t)r.raw_keys.size();
  const int na = (int)r.functions.size();
  std::vector<std::vector<uint8_t>> regs(na);
  for (int f = 0; f < na; f++)
    if (is_hll_fn(r.functions[f]) && n) {
      regs[f].resize((size_t)n * 256);
      group_by_hll_registers(r, f, regs[f].data());
    }
  w.i64(n);
  for (int64_t g = 0; g < n; g++) {
    w.str(r.key(g));
    for (int f = 0; f < na; f++) {
      w.i64(r.counts[r.counts_shared ? 0 : f][g]);
      w.f64(r.values[f].empty() ? 0.0 : r.values[f][g]);
      if (!regs[f].empty()) w.raw(regs[f].data() + (size_t)g * 256, 256);
    }
  }
}

// CombineGroupByOperator's merge (CombineGroupByOperator.java:142-161) of every rank's segments' groups, in rank then
// segment order, by group-key string: a key new to the merged map enters only while the map holds fewer than `cap`
// keys (2 x num.groups.limit, :80,147); each function merges as its AggregationFunction.merge does (counts and sums
// add, AvgPair adds both, MIN / MAX, HyperLogLog register max). The result's keys are its one "column" of strings.
std::unique_ptr<GroupByResult> merge_rank_groups(const pinot_query &q, const std::vector<std::vector<uint8_t>> &blobs,
                                                 const std::vector<size_t> &offsets, int64_t cap) {
  const int na = q.num_aggregations;
  std::vector<int> fn(na);
  for (int a = 0; a < na; a++) fn[a] = q.aggregations[a].function;
  std::unordered_map<std::string, int64_t> at;
  std::vector<std::string> keys;
  std::vector<std::vector<int64_t>> cnt(na);
  std::vector<std::vector<double>> val(na);
  std::vector<std::vector<uint8_t>> reg(na);
  for (size_t r = 0; r < blobs.size(); r++) {
    Reader rd{blobs[r]};
    rd.p = offsets[r];
    const int64_t nseg = rd.i64();
    for (int64_t s = 0; s < nseg; s++) {
      const int64_t n = rd.i64();
      for (int64_t g = 0; g < n; g++) {
        const std::string k = rd.str();
        auto it = at.find(k);
        int64_t i = -1;
        if (it != at.end()) {
          i = it->second;
        } else if ((int64_t)keys.size() < cap) {
          i = (int64_t)keys.size();
          at.emplace(k, i);
          keys.push_back(k);
          for (int a = 0; a < na; a++) {
            const int f = sv_function(fn[a]);
            cnt[a].push_back(0);
            val[a].push_back(f == PINOT_AGG_MIN ? INFINITY : f == PINOT_AGG_MAX ? -INFINITY : 0.0);
            if (is_hll_fn(fn[a])) reg[a].resize(reg[a].size() + 256, 0);
          }
        }
        for (int a = 0; a < na; a++) {
          const int64_t c = rd.i64();
          const double v = rd.f64();
          uint8_t x[256];
          if (is_hll_fn(fn[a])) rd.raw(x, 256);
          if (i < 0) continue;  // the merged map is full: the key is dropped
          cnt[a][i] += c;
          const int f = sv_function(fn[a]);
          if (f == PINOT_AGG_MIN) val[a][i] = std::min(val[a][i], v);
          else if (f == PINOT_AGG_MAX) val[a][i] = std::max(val[a][i], v);
          else if (f == PINOT_AGG_SUM || f == PINOT_AGG_AVG) val[a][i] += v;
          if (is_hll_fn(fn[a]))
            for (int j = 0; j < 256; j++) reg[a][(size_t)i * 256 + j] = std::max(reg[a][(size_t)i * 256 + j], x[j]);
        }
      }
    }
  }
  // ascending key strings (the reference's map order is a hash order; the DataTable writer keeps this one)
  const int64_t n = (int64_t)keys.size();
  std::vector<int64_t> ord(n);
  for (int64_t g = 0; g < n; g++) ord[g] = g;
  std::sort(ord.begin(), ord.end(), [&](int64_t x, int64_t y) { return keys[x] < keys[y]; });
  auto out = empty_group_result(q);
  out->counts_shared = false;
  out->gcard = {n};
  out->gvalues.assign(1, std::vector<std::string>((size_t)n));
  out->raw_keys.resize(n);
  for (int a = 0; a < na; a++) {
    out->counts[a].resize(n);
    out->values[a].resize(n);
    if (is_hll_fn(fn[a])) {
      out->hll[a].resize((size_t)n * 256);
      out->hll_card[a].resize(n);
    }
  }
  for (int64_t g = 0; g < n; g++) {
    const int64_t i = ord[g];
    out->raw_keys[g] = g;
    out->gvalues[0][g] = std::move(keys[i]);
    for (int a = 0; a < na; a++) {
      out->counts[a][g] = cnt[a][i];
      out->values[a][g] = val[a][i];
      if (is_hll_fn(fn[a])) {
        memcpy(out->hll[a].data() + (size_t)g * 256, reg[a].data() + (size_t)i * 256, 256);
        out->hll_card[a][g] = hll_cardinality(out->hll[a].data() + (size_t)g * 256);
        out->values[a][g] = (double)out->hll_card[a][g];
      }
    }
  }
  out->merged_groups = n;
  return out;
}

// This rank's segments for the query: its refs resolved on its engine, pruned (pinot_query.pruners, the server's
// SegmentPrunerService), and the docs of all of them (totalDocs counts pruned segments, :214-215).
std::vector<SegmentData *> rank_segments(Engine &e, size_t engine_index, const std::vector<SegmentRef> &refs,
                                         const pinot_query &q, int64_t &total_docs) {
  require(q.timeout_ms >= 0, PINOT_ERR_TIMEOUT, "query budget already spent before execution");
  std::vector<SegmentData *> segs;
  for (const SegmentRef &r : refs)
    if (r.engine == (int)engine_index) segs.push_back(&e.seg(r.handle));
  total_docs = 0;
  for (auto *sd : segs) total_docs += sd->num_docs;
  return prune_for_query(segs, q);
}

}  // namespace

ServerImpl *server_create(const int32_t *devices, int32_t n, const char *config) {
  require(devices && n >= 1, PINOT_ERR_BAD_ARG, "at least one device");
  const ServerConfig cfg = parse_server_config(config);
  auto s = std::make_unique<ServerImpl>();
  std::vector<int> devs(devices, devices + n);
  for (int d : devs) s->engines.push_back(create_engine(d, cfg.engine.empty() ? nullptr : cfg.engine.c_str()));
  auto hub = std::make_shared<Hub>(n, cfg.timeout_ms);  // every rank is in this process: control data on the host
  if (cfg.loopback) {
    for (int d : devs) require(d == devs[0], PINOT_ERR_BAD_ARG, "server.loopback: every engine on the same device");
    hub->device = devs[0];
    for (int i = 0; i < n; i++) s->comms.push_back(make_loopback_collective(hub, i, devs[0]));
  } else {
    std::vector<ncclComm_t> raw(n, nullptr);
    const ncclResult_t r = ncclCommInitAll(raw.data(), n, devs.data());
    require(r == ncclSuccess, PINOT_ERR_DEVICE, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
    for (int i = 0; i < n; i++) s->comms.push_back(make_rccl_collective(raw[i], i, n, hub));
  }
  s->nranks = n;
  s->gather = cfg.gather;
  s->partial.resize(n);
  return s.release();
}

void server_unique_id(uint8_t *id) {
  ncclUniqueId u;
  const ncclResult_t r = ncclGetUniqueId(&u);
  require(r == ncclSuccess, PINOT_ERR_DEVICE, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  static_assert(sizeof(u) == 128, "ncclUniqueId is 128 bytes");
  memcpy(id, &u, sizeof(u));
}

ServerImpl *server_create_rank(int32_t device, int32_t nranks, int32_t rank, const uint8_t *id, const char *config) {
  require(id && nranks >= 1 && rank >= 0 && rank < nranks, PINOT_ERR_BAD_ARG, "rank / nranks / unique id");
  const ServerConfig cfg = parse_server_config(config);
  auto s = std::make_unique<ServerImpl>();
  s->engines.push_back(create_engine(device, cfg.engine.empty() ? nullptr : cfg.engine.c_str()));
  PINOT_HIP(hipSetDevice(device));
  if (cfg.loopback) {
    s->comms.push_back(make_loopback_collective(loopback_hub(id, nranks, cfg.timeout_ms, device), rank, device));
  } else {
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    ncclComm_t c = nullptr;
    const ncclResult_t r = ncclCommInitRank(&c, nranks, u, rank);
    require(r == ncclSuccess, PINOT_ERR_DEVICE, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    s->comms.push_back(make_rccl_collective(c, rank, nranks, nullptr));
  }
  s->nranks = nranks;
  s->rank0 = rank;
  s->gather = cfg.gather;
  s->partial.resize(1);
  return s.release();
}

void server_destroy(ServerImpl *s) { delete s; }
int server_num_engines(const ServerImpl &s) { return (int)s.engines.size(); }
void server_last_phases(const ServerImpl &s, double *ms, int n) {
  for (int i = 0; i < n && i < kServerPhases; i++) ms[i] = s.phase_ms[i];
}

Engine *server_engine(ServerImpl &s, int i) {
  require(i >= 0 && i < (int)s.engines.size(), PINOT_ERR_BAD_ARG, "engine index");
  return s.engines[i].get();
}

// ------------------------------------------------------------------ aggregation-only
void server_aggregate(ServerImpl &s, const std::vector<SegmentRef> &refs, const pinot_query &q, pinot_agg_result *out,
                      pinot_exec_stats *stats) {
  std::lock_guard<std::mutex> lk(s.mu);
  for (const SegmentRef &r : refs)
    require(r.engine >= 0 && r.engine < (int)s.engines.size(), PINOT_ERR_BAD_ARG, "segment ref: no such engine");
  const size_t E = s.engines.size();
  const int na = q.num_aggregations;
  std::vector<std::vector<pinot_agg_result>> merged(E, std::vector<pinot_agg_result>(na));
  std::vector<pinot_exec_stats> tot(E);
  for_engines(s, [&](size_t i) {
    Engine &e = *s.engines[i];
    Collective &c = *s.comms[i];
    Phases ph(i == 0 ? s.phase_ms : nullptr);
    std::vector<pinot_agg_result> part(na);
    pinot_exec_stats st{};
    const Status my = capture([&] {
      std::lock_guard<std::mutex> el(e.mu);
      int64_t tdocs = 0;
      const auto segs = rank_segments(e, i, refs, q, tdocs);
      if (segs.empty()) {
        agg_identities(q, part.data());
      } else {
        DeadlineScope ds(e, q.timeout_ms);
        exec_aggregate(e, segs, q, part.data(), &st);
      }
      st.num_total_raw_docs = tdocs;
    });
    ph.mark(0);
    Writer w;
    put_status(w, my);
    put_stats(w, st);
    w.raw(part.data(), sizeof(pinot_agg_result) * na);
    const auto all = c.all_gather_host(w.b, e.stream);
    ph.mark(1);
    std::vector<Status> sts;
    std::vector<std::vector<pinot_agg_result>> parts(all.size(), std::vector<pinot_agg_result>(na));
    for (size_t r = 0; r < all.size(); r++) {
      Reader rd{all[r]};
      sts.push_back(get_status(rd));
      add_stats(rd, tot[i]);
      rd.raw(parts[r].data(), sizeof(pinot_agg_result) * na);
    }
    fail_together(sts, c.rank(), "aggregation");
    std::vector<const pinot_agg_result *> ptrs;
    for (auto &p : parts) ptrs.push_back(p.data());
    merge_agg_parts(q, ptrs, merged[i].data());  // CombineService.mergeTwoBlocks in rank order
  });
  memcpy(out, merged[0].data(), sizeof(pinot_agg_result) * na);
  if (stats) *stats = tot[0];
}

// ------------------------------------------------------------------ group-by
std::unique_ptr<GroupByResult> server_group_by(ServerImpl &s, const std::vector<SegmentRef> &refs, const pinot_query &q0,
                                               pinot_exec_stats *stats, int32_t top_n) {
  std::lock_guard<std::mutex> lk(s.mu);
  for (const SegmentRef &r : refs)
    require(r.engine >= 0 && r.engine < (int)s.engines.size(), PINOT_ERR_BAD_ARG, "segment ref: no such engine");
  require(q0.num_aggregations >= 1 && q0.num_aggregations <= kMaxAggs, PINOT_ERR_UNSUPPORTED,
          "1..8 aggregation functions per query");
  // the partials run on the extended function list (a hidden CountMV per AvgMV carries its entry count), folded
  // back into the query's functions at the end
  std::vector<int> hidden;
  const std::vector<pinot_agg_spec> xspecs = mv_extended_specs(q0, hidden);
  pinot_query qx = q0;
  qx.aggregations = xspecs.data();
  qx.num_aggregations = (int32_t)xspecs.size();
  const pinot_query &q = qx;
  const int na = q.num_aggregations;
  bool mv_counts = na != q0.num_aggregations;
  for (int a = 0; a < q0.num_aggregations; a++) mv_counts = mv_counts || q0.aggregations[a].function == PINOT_AGG_COUNTMV;
  require(q.num_group_by >= 1 && q.num_group_by <= kMaxGroupCols, PINOT_ERR_UNSUPPORTED, "1..16 group-by columns");
  const size_t E = s.engines.size();
  std::vector<std::unique_ptr<GroupByResult>> res(E);
  std::vector<pinot_exec_stats> tot(E);
  std::atomic<bool> hashed_result{false};  // rank 0 holds the merged hashed result (the others an empty one)
  if (s.ks_cache.size() < E) s.ks_cache.resize(E);
  for_engines(s, [&](size_t i) {
    Engine &e = *s.engines[i];
    Collective &c = *s.comms[i];
    Phases ph(i == 0 ? s.phase_ms : nullptr);
    const int R = c.nranks(), me = c.rank();
    // A: prune, local dictionaries and accumulator kinds -> every rank's
    std::vector<SegmentData *> segs;
    int64_t tdocs = 0, possible = 0;
    std::vector<int> kinds;
    std::vector<uint8_t> dicts;
    bool mv = false;  // this rank's segments take the multi-value partial (MV group columns or MV functions)
    Status my = capture([&] {
      std::lock_guard<std::mutex> el(e.mu);
      segs = rank_segments(e, i, refs, q, tdocs);
      dicts = local_group_dictionaries(segs, q);
      if (!segs.empty()) {
        kinds = group_acc_kind_list(*segs[0], q);
        possible = admission_possible(segs, q, e);
        mv = touches_mv_group_by(segs, q0);
      }
    });
    ph.mark(0);
    Writer wa;
    put_status(wa, my);
    wa.i64(tdocs);
    wa.i64(possible);
    wa.i64((int64_t)kinds.size());
    for (int k : kinds) wa.i64(k);
    wa.bytes(dicts);
    const auto all_a = c.all_gather_host(wa.b, e.stream);
    std::vector<Status> sts;
    std::vector<std::vector<uint8_t>> rank_dicts;
    std::vector<int> gkinds;
    int64_t total_docs = 0, total_possible = 0;
    bool kinds_agree = true;
    for (const auto &blob : all_a) {
      Reader rd{blob};
      sts.push_back(get_status(rd));
      total_docs += rd.i64();
      total_possible += rd.i64();
      std::vector<int> k((size_t)rd.i64());
      for (int &x : k) x = (int)rd.i64();
      rank_dicts.push_back(rd.bytes());
      if (!k.empty()) {
        if (gkinds.empty()) gkinds = k;
        else kinds_agree = kinds_agree && gkinds == k;
      }
    }
    fail_together(sts, me, "group-by");
    require(kinds_agree, PINOT_ERR_UNSUPPORTED, "multi-GPU group-by: ranks disagree on the aggregated columns' types");
    // identical on every rank (same inputs)
    const std::shared_ptr<const GlobalKeySpace> ksp =
        gkinds.empty() ? std::make_shared<const GlobalKeySpace>() : key_space_cached(s.ks_cache[i], segs, q, rank_dicts);
    const GlobalKeySpace &ks = *ksp;
    ph.mark(1);
    const int64_t limit = q.num_groups_limit > 0 ? q.num_groups_limit : e.num_groups_limit;
    if (ks.hashed) {
      // LONG_MAP / ARRAY_MAP key spaces (SV or MV): no dense partials to reduce-scatter. Each rank runs its segments'
      // group-bys one segment at a time (each segment's holder applies its own num.groups.limit admission,
      // DictionaryBasedGroupKeyGenerator.java:293-302, 459-470), the segments' groups travel to rank 0 by key string,
      // and rank 0 merges them as CombineGroupByOperator does (merge_rank_groups)
      pinot_exec_stats st{};
      Writer wh;
      std::vector<uint8_t> groups;
      my = capture([&] {
        std::lock_guard<std::mutex> el(e.mu);
        DeadlineScope ds(e, q.timeout_ms);
        Writer w;
        w.i64((int64_t)segs.size());
        for (SegmentData *sg : segs) {
          pinot_exec_stats s1{};
          auto r = exec_group_by(e, std::vector<SegmentData *>{sg}, q0, &s1);
          st.num_docs_scanned += s1.num_docs_scanned;
          st.num_entries_scanned_in_filter += s1.num_entries_scanned_in_filter;
          st.num_entries_scanned_post_filter += s1.num_entries_scanned_post_filter;
          st.num_segments_processed += s1.num_segments_processed;
          st.num_segments_matched += s1.num_segments_matched;
          st.device_ms += s1.device_ms;
          put_groups(w, *r);
        }
        groups = std::move(w.b);
      });
      put_status(wh, my);
      put_stats(wh, st);
      wh.raw(groups.data(), groups.size());
      const auto all_h = c.all_gather_host(wh.b, e.stream);
      sts.clear();
      std::vector<size_t> offs;
      for (const auto &blob : all_h) {
        Reader rd{blob};
        sts.push_back(get_status(rd));
        add_stats(rd, tot[i]);
        offs.push_back(rd.p);
      }
      tot[i].num_total_raw_docs = total_docs;
      fail_together(sts, me, "group-by");
      ph.mark(2);
      if (me == 0 || !s.gather) {
        const int64_t trim_size = std::max<int64_t>(5 * (int64_t)top_n, 5000);
        if (me == 0) {
          res[i] = merge_rank_groups(q0, all_h, offs, 2 * limit);
          const int64_t n = (int64_t)res[i]->raw_keys.size();
          if (top_n > 0 && n > 4 * trim_size)
            server_trim_select(*res[i], top_n, std::vector<uint32_t>((size_t)n, 0xFFFFFFFFu), n);
        } else {
          res[i] = empty_group_result(q0);
        }
      } else {
        res[i] = empty_group_result(q0);
      }
      ph.mark(6);
      hashed_result = true;
      return;
    }
    if (gkinds.empty() || ks.G == 0) {  // no rank holds a segment after pruning: no group
      res[i] = empty_group_result(q);
      tot[i].num_total_raw_docs = total_docs;
      return;
    }
    // A2: the 2 x num.groups.limit inter-segment cap (CombineGroupByOperator.java:80,147) when it can bind: every
    // rank's segments' first-appearance admitted keys (each segment's holder rule applied on its own rank,
    // DictionaryBasedGroupKeyGenerator.java:293-302) -> every rank; keys enter the merged map in rank order, then each
    // rank's own segment order (the reference's thread-pool order is nondeterministic; this one is fixed), until
    // 2 x limit keys are in; each rank then runs its partials with its segments' capped bitmaps
    AdmissionIO admit;
    if (std::min(total_possible, ks.G) > 2 * limit) {
      AdmissionIO ex;
      ex.mode = 1;
      my = capture([&] {
        std::lock_guard<std::mutex> el(e.mu);
        DeadlineScope ds(e, q.timeout_ms);
        if (segs.empty()) return;
        if (mv)
          exec_group_by_mv_partial(e, segs, q0, MvPartial{&ks.gcard, &ks.gvalues, &ks.remap, nullptr, nullptr, &ex},
                                   nullptr);
        else
          exec_group_by_partial_ks(e, segs, q, ks.gcard, ks.gvalues, ks.remap, nullptr, nullptr, nullptr, &ex);
      });
      Writer wc;
      put_status(wc, my);
      wc.i64((int64_t)(segs.empty() ? 0 : segs.size()));
      wc.i64(ex.words);
      std::vector<uint8_t> raw(ex.bitmaps.size() * 4);
      if (!raw.empty()) memcpy(raw.data(), ex.bitmaps.data(), raw.size());
      wc.bytes(raw);
      const auto all_c = c.all_gather_host(wc.b, e.stream);
      sts.clear();
      std::vector<int64_t> nseg(R, 0);
      std::vector<std::vector<uint8_t>> rank_bm(R);
      int64_t words = 0;
      for (int r = 0; r < R; r++) {
        Reader rd{all_c[r]};
        sts.push_back(get_status(rd));
        nseg[r] = rd.i64();
        const int64_t w = rd.i64();
        rank_bm[r] = rd.bytes();
        if (nseg[r] > 0) words = std::max(words, w);
      }
      fail_together(sts, me, "group-by admission");
      std::vector<uint32_t> bm;
      int64_t S_all = 0, mine = 0;
      for (int r = 0; r < R; r++) {
        if (nseg[r] <= 0) continue;
        require((int64_t)rank_bm[r].size() == nseg[r] * words * 4, PINOT_ERR_DEVICE, "admitted bitmaps of another shape");
        if (r == me) mine = S_all;
        const size_t at = bm.size();
        bm.resize(at + (size_t)nseg[r] * words);
        memcpy(bm.data() + at, rank_bm[r].data(), rank_bm[r].size());
        S_all += nseg[r];
      }
      inter_segment_cap(bm, (size_t)S_all, words, 2 * limit);
      if (!segs.empty()) {
        admit.mode = 2;
        admit.words = words;
        admit.bitmaps.assign(bm.begin() + mine * words, bm.begin() + (mine + (int64_t)segs.size()) * words);
      }
    }
    const int64_t G = ks.G, slice = (G + R - 1) / R, Gp = slice * R;
    // B: dense partials over [0, G), identities on the padding (everywhere without segments)
    unsigned long long *counts = nullptr;
    std::vector<void *> accs(na, nullptr);
    pinot_exec_stats st{};
    // one rank: its range is the whole merged map, so the ring plan's packed HLL register sums (u64 [G] after each
    // HLL's registers) stay valid through D — the finalize then reads cardinalities as the engine's does
    const bool sum_room = R == 1 && !mv;
    bool sums_written = false;
    auto acc_bytes = [&](int a) {
      return ((size_t)Gp * acc_unit(gkinds[a]) + (sum_room && gkinds[a] == 4 ? (size_t)Gp * 8 : 0) + 255) / 256 * 256;
    };
    my = capture([&] {
      std::lock_guard<std::mutex> el(e.mu);
      DeadlineScope ds(e, q.timeout_ms);
      size_t bytes = ((size_t)Gp * 8 + 255) / 256 * 256 + 256;
      for (int a = 0; a < na; a++) bytes += acc_bytes(a);
      s.partial[i].reserve(bytes);
      uint8_t *p = s.partial[i].get<uint8_t>();
      counts = reinterpret_cast<unsigned long long *>(p);
      p += ((size_t)Gp * 8 + 255) / 256 * 256;
      for (int a = 0; a < na; a++) {
        if (gkinds[a] == 5) continue;
        accs[a] = p;
        p += acc_bytes(a);
      }
      const int64_t from = segs.empty() ? 0 : G;
      PINOT_HIP(hipMemsetAsync(counts + from, 0, (size_t)(Gp - from) * 8, e.stream));
      for (int a = 0; a < na; a++)
        if (accs[a])
          PINOT_HIP(hipMemsetAsync(static_cast<uint8_t *>(accs[a]) + (size_t)from * acc_unit(gkinds[a]),
                                   gkinds[a] == 2 ? 0xFF : 0, (size_t)(Gp - from) * acc_unit(gkinds[a]), e.stream));
      if (!segs.empty() && mv)
        exec_group_by_mv_partial(e, segs, q0,
                                 MvPartial{&ks.gcard, &ks.gvalues, &ks.remap, reinterpret_cast<int64_t *>(counts),
                                           accs.data(), admit.mode ? &admit : nullptr},
                                 &st);
      else if (!segs.empty())
        exec_group_by_partial_ks(e, segs, q, ks.gcard, ks.gvalues, ks.remap, reinterpret_cast<int64_t *>(counts),
                                 accs.data(), &st, admit.mode ? &admit : nullptr, sum_room, &sums_written);
      PINOT_HIP(hipStreamSynchronize(e.stream));
    });
    ph.mark(2);
    Writer wb;
    put_status(wb, my);
    put_stats(wb, st);
    const auto all_b = c.all_gather_host(wb.b, e.stream);
    ph.mark(3);
    sts.clear();
    for (const auto &blob : all_b) {
      Reader rd{blob};
      sts.push_back(get_status(rd));
      add_stats(rd, tot[i]);
    }
    tot[i].num_total_raw_docs = total_docs;
    fail_together(sts, me, "group-by partials");
    std::lock_guard<std::mutex> el(e.mu);
    // C: in-place reduce-scatter of every array; this rank keeps [me * slice, (me + 1) * slice)
    c.group_start();
    c.reduce_scatter(counts, (size_t)slice, CType::U64, COp::SUM, e.stream);
    for (int a = 0; a < na; a++)
      if (accs[a])
        c.reduce_scatter(accs[a], (size_t)slice * (gkinds[a] == 4 ? 256 : 1), acc_ctype(gkinds[a]), acc_op(gkinds[a]),
                         e.stream);
    c.group_end();
    if (e.timing) PINOT_HIP(hipStreamSynchronize(e.stream));  // the merge's device time on its own
    ph.mark(4);
    // D: owner finalize of this rank's key range, then the gather to rank 0. A trimmed answer (top_n: the server's
    // AggregationGroupByTrimmingService, CombineGroupByOperator.java:184-187) first learns the merged map's size (every
    // range's non-empty keys); above 4 x trimSize each rank keeps its range's trimSize best groups per function — the
    // merged map's best are among them, the ranges being disjoint — so only those leave the owner ranks
    const int64_t base = (int64_t)me * slice;
    const int64_t g = std::max<int64_t>(0, std::min<int64_t>(slice, G - base));
    std::vector<void *> sl(na, nullptr);
    for (int a = 0; a < na; a++)
      if (accs[a]) sl[a] = static_cast<uint8_t *>(accs[a]) + (size_t)base * acc_unit(gkinds[a]);
    long long *keys_dev = nullptr;
    const unsigned long long nr = slice_compact(e, counts + base, g, keys_dev);
    // (not with hidden CountMV functions: those leave the function list after the merge; the caller's trim applies)
    const bool top = top_n > 0 && (s.gather || R == 1) && na == q0.num_aggregations;
    int64_t merged = (int64_t)nr;
    if (top && R > 1) {
      Writer wg;
      wg.i64((int64_t)nr);
      const auto all_g = c.all_gather_host(wg.b, e.stream);
      merged = 0;
      for (int r = 0; r < R; r++) {
        Reader rd{all_g[r]};
        merged += rd.i64();
      }
    }
    const int64_t trim_size = std::max<int64_t>(5 * (int64_t)top_n, 5000);
    const bool trim = top && merged > 4 * trim_size;
    std::vector<uint32_t> flags;
    std::vector<const void *> sums;
    if (sums_written)
      for (int a = 0; a < na; a++)
        sums.push_back(gkinds[a] == 4 && accs[a] ? static_cast<const uint8_t *>(accs[a]) + (size_t)G * 256 : nullptr);
    const bool one = !s.gather || R == 1;  // this rank's outputs are the answer's (nothing gathered after them)
    const DenseOut own = slice_outputs_keys(e, q, gkinds, counts + base, sl, g, base, keys_dev, nr, trim ? top_n : 0, flags,
                                            R == 1 && !mv ? &ks.gcard : nullptr, sums_written ? &sums : nullptr);
    ph.mark(5);
    if (one) {
      res[i] = slice_result(e, q, ks.gcard, ks.gvalues, own);
      if (trim) server_trim_select(*res[i], top_n, flags, merged);
      ph.mark(6);
      return;
    }
    Writer wn;
    wn.i64((int64_t)own.n);
    if (trim) {
      std::vector<uint8_t> fb(flags.size() * 4);
      if (!fb.empty()) memcpy(fb.data(), flags.data(), fb.size());
      wn.bytes(fb);
    }
    const auto all_n = c.all_gather_host(wn.b, e.stream);
    std::vector<size_t> prefix(R + 1, 0);
    std::vector<uint32_t> all_flags;
    for (int r = 0; r < R; r++) {
      Reader rd{all_n[r]};
      prefix[r + 1] = prefix[r] + (size_t)rd.i64();
      if (trim) {
        const std::vector<uint8_t> fb = rd.bytes();
        require(fb.size() == (prefix[r + 1] - prefix[r]) * 4, PINOT_ERR_DEVICE, "server trim: flags of another size");
        const size_t at = all_flags.size();
        all_flags.resize(at + fb.size() / 4);
        if (!fb.empty()) memcpy(all_flags.data() + at, fb.data(), fb.size());
      }
    }
    DenseOut root = me == 0 ? slice_alloc(e, q, gkinds, prefix[R]) : DenseOut{};
    const auto send = slice_arrays(own);
    const auto recv = me == 0 ? slice_arrays(root) : std::vector<std::pair<void *, size_t>>(send.size(), {nullptr, 0});
    c.group_start();
    for (size_t k = 0; k < send.size(); k++) {
      const size_t unit = send[k].second;
      std::vector<size_t> off(R + 1);
      for (int r = 0; r <= R; r++) off[r] = prefix[r] * unit;
      c.gather(send[k].first, (size_t)own.n * unit, recv[k].first, off, 0, e.stream);
    }
    c.group_end();
    if (me == 0) {
      if (trim && !mv) slice_serialize(e, q, ks.gcard, root);  // the trimmed answer's DataTable pieces, on the device
      res[i] = slice_result(e, q, ks.gcard, ks.gvalues, root);
      if (trim) server_trim_select(*res[i], top_n, all_flags, merged);
    } else {
      DenseOut none;
      none.kind = gkinds;
      res[i] = slice_result(e, q, ks.gcard, ks.gvalues, none);
      PINOT_HIP(hipStreamSynchronize(e.stream));  // the sends have left this rank's buffers
    }
    ph.mark(6);
  });
  std::unique_ptr<GroupByResult> out = std::move(res[0]);
  if (hashed_result) {  // merged on rank 0 with the query's own functions (no hidden CountMV)
    if (stats) *stats = tot[0];
    return out;
  }
  if (!s.gather && E > 1) {  // one process, several GPUs, key ranges kept apart: concatenate them (ascending)
    for (size_t i = 1; i < E; i++) {
      GroupByResult &x = *res[i];
      const int64_t off = (int64_t)out->raw_keys.size();
      out->raw_keys.insert(out->raw_keys.end(), x.raw_keys.begin(), x.raw_keys.end());
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
  }
  out->counts_shared = true;
  if (mv_counts) fold_mv_counts(*out, q0, hidden);  // CountMV / AvgMV counts: entries, not docs
  if (stats) *stats = tot[0];
  return out;
}

}  // namespace pinot
