// extern "C" entry points of libpinot_gpu.so (declared in include/pinot_gpu.h).
// Every call: validate -> take the engine lock -> run -> map exceptions to pinot_status.
#include <chrono>
#include <cstring>
#include <sstream>

#include "engine.h"

namespace pinot {

Engine::~Engine() {
  // drain every queue first: result copies (copy streams, async D2H of pooled results) still in flight at teardown
  // would complete after their buffers and streams are gone
  if (stream) (void)hipStreamSynchronize(stream);
  for (auto cs : copy_streams) (void)hipStreamSynchronize(cs);
  (void)hipDeviceSynchronize();
  segments.clear();
  for (auto ev : kev) (void)hipEventDestroy(ev);
  if (ev_start) (void)hipEventDestroy(ev_start);
  if (ev_stop) (void)hipEventDestroy(ev_stop);
  for (auto cs : copy_streams) (void)hipStreamDestroy(cs);
  if (ev_copy) (void)hipEventDestroy(ev_copy);
  if (stream) (void)hipStreamDestroy(stream);
}

SegmentData &Engine::seg(int64_t h) {
  auto it = segments.find(h);
  require(it != segments.end(), PINOT_ERR_BAD_ARG, "unknown segment handle " + std::to_string(h));
  return *it->second;
}

}  // namespace pinot

using namespace pinot;

struct pinot_server {
  ServerImpl *impl = nullptr;
  ~pinot_server() { server_destroy(impl); }
};


namespace {

double elapsed_ms(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}
thread_local std::string g_last_error;

template <typename F>
pinot_status guard(F f) {
  try {
    f();
    g_last_error.clear();
    return PINOT_OK;
  } catch (const Error &e) {
    g_last_error = e.what();
    return e.status;
  } catch (const std::bad_alloc &) {
    g_last_error = "host out of memory";
    return PINOT_ERR_OOM;
  } catch (const std::exception &e) {
    g_last_error = e.what();
    return PINOT_ERR_DEVICE;
  }
}

void set_device(Engine &e) { PINOT_HIP(hipSetDevice(e.device)); }
void parse_config(Engine &e, const char *cfg);
}  // namespace

namespace pinot {
std::unique_ptr<pinot_engine> create_engine(int32_t device, const char *config) {
  int n = 0;
  PINOT_HIP(hipGetDeviceCount(&n));
  require(device >= 0 && device < n, PINOT_ERR_BAD_ARG, "no such HIP device");
  auto e = std::make_unique<pinot_engine>();
  e->device = device;
  parse_config(*e, config);
  PINOT_HIP(hipSetDevice(device));
  PINOT_HIP(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
  hipDeviceProp_t prop;
  PINOT_HIP(hipGetDeviceProperties(&prop, device));
  e->num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) == hipSuccess && khz > 0)
    e->wall_clock_khz = khz;
  PINOT_HIP(hipEventCreate(&e->ev_start));
  PINOT_HIP(hipEventCreate(&e->ev_stop));
  return e;
}
}  // namespace pinot

namespace {

std::vector<SegmentData *> resolve(Engine &e, const pinot_segment_handle *segs, int32_t n) {
  require(n >= 1 && segs != nullptr, PINOT_ERR_BAD_ARG, "at least one segment required");
  std::vector<SegmentData *> out;
  for (int32_t i = 0; i < n; i++) out.push_back(&e.seg(segs[i]));
  return out;
}

int64_t total_docs(const std::vector<SegmentData *> &segs) {
  int64_t t = 0;
  for (auto *s : segs) t += s->num_docs;
  return t;
}

void check_query(const pinot_query *q) {
  require(q != nullptr, PINOT_ERR_BAD_ARG, "null query");
  require(q->num_filter_nodes == 0 || q->filter != nullptr, PINOT_ERR_BAD_ARG, "filter nodes");
  require(q->num_aggregations >= 1 && q->aggregations != nullptr, PINOT_ERR_BAD_ARG, "aggregations");
  require(q->num_group_by == 0 || q->group_by != nullptr, PINOT_ERR_BAD_ARG, "group_by");
}

// stats.exact=1: numEntriesScannedInFilter as a Java server counts it (filter_stats.cpp), summed over the processed
// segments; the shortcut plans (no filter) scan nothing either way
void exact_filter_stats(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q, pinot_exec_stats *st) {
  if (!e.stats_exact || !st || q.num_filter_nodes == 0) return;
  const FilterTreeInput tree = decode_filter(q.num_filter_nodes, q.filter);
  int64_t n = 0;
  for (SegmentData *s : segs)  // a segment on its star-tree counts its traversal's remaining-predicate entries
    n += std::count(e.star_answered.begin(), e.star_answered.end(), s) ? star_tree_match(*s, q, &tree).entries_in_filter
                                                                       : filter_entries_scanned(e, *s, &tree);
  st->num_entries_scanned_in_filter = n;
}

void parse_config(Engine &e, const char *cfg) {
  if (!cfg) return;
  e.config_epoch++;
  std::stringstream ss(cfg);
  std::string kv;
  while (std::getline(ss, kv, ';')) {
    auto p = kv.find('=');
    if (p == std::string::npos) continue;
    std::string k = kv.substr(0, p), v = kv.substr(p + 1);
    if (k == "num.groups.limit") e.num_groups_limit = std::stoi(v);
    else if (k == "filter.force") e.force_filter = v;
    else if (k == "timing") e.timing = v == "1" || v == "true";
    else if (k == "agg.affine") e.use_affine = v == "1" || v == "true";
    else if (k == "exec.fused") e.use_fused = v == "1" || v == "true";
    else if (k == "group.mode") {
      require(v.empty() || v == "auto" || v == "lds" || v == "global" || v == "partition", PINOT_ERR_BAD_ARG,
              "group.mode: auto | lds | global | partition");
      e.group_mode = v == "auto" ? "" : v;
    } else if (k == "sync.poll") e.sync_poll = v == "1" || v == "true";
    else if (k == "sync.flag") e.sync_flag = v == "1" || v == "true";
    else if (k == "group.pshift") e.group_pshift = std::stoi(v);
    else if (k == "group.nt_store") e.group_nt_store = std::stoi(v) != 0;
    else if (k == "group.prefetch") e.group_prefetch = v == "1" || v == "true";
    else if (k == "group.bucket") e.group_bucket = v == "1" || v == "true";
    else if (k == "group.ring") e.group_ring = v == "1" || v == "true";
    else if (k == "group.ring_qfilter") e.group_ring_qfilter = v == "1" || v == "true";
    else if (k == "group.ring_hll") e.group_ring_hll = v == "1" || v == "true";
    else if (k == "group.lds_qfilter") e.group_lds_qfilter = v == "1" || v == "true";
    else if (k == "group.ring_rec6") e.group_ring_rec6 = v == "1" || v == "true";
    else if (k == "raw.device") e.raw_device = v == "1" || v == "true";
    else if (k == "group.aligned") e.group_aligned = v == "1" || v == "true";
    else if (k == "group.lds_block") {
      e.group_lds_block = std::stoi(v);
      require(e.group_lds_block == 256 || e.group_lds_block == 512, PINOT_ERR_BAD_ARG, "group.lds_block: 256 | 512");
    } else if (k == "group.emit_block") {
      e.group_emit_block = std::stoi(v);
      require(e.group_emit_block == 512 || e.group_emit_block == 1024, PINOT_ERR_BAD_ARG, "group.emit_block: 512 | 1024");
    }
    else if (k == "group.lw") {
      e.group_lw = v == "true" ? 1 : std::stoi(v);
      require(e.group_lw >= 0 && e.group_lw <= 2, PINOT_ERR_BAD_ARG, "group.lw: 0 (per doc) | 1 (lane owns word) | 2 (contiguous quarters)");
    }
    else if (k == "plan.shortcut") e.use_shortcut_plans = v == "1" || v == "true";
    else if (k == "plan.cache") e.use_plan_cache = v == "1" || v == "true";
    else if (k == "group.split") {
      e.group_split = std::stoi(v);
      require(e.group_split >= -1 && e.group_split <= 8, PINOT_ERR_BAD_ARG, "group.split: -1 (auto) .. 8");
    }
    else if (k == "debug.host_phases") e.host_phases = v == "1" || v == "true";
    else if (k == "host.spin") set_host_spin(std::stoi(v));
    else if (k == "exec.nt") e.use_nt = v == "1" || v == "true";
    else if (k == "exec.pipe") e.use_pipe = v == "1" || v == "true";
    else if (k == "stats.exact") e.stats_exact = v == "1" || v == "true";
    else if (k == "startree.use") e.use_star_tree = v == "1" || v == "true";
    else if (k == "d2h.compact") e.compact_d2h = v == "1" || v == "true";
    else if (k == "d2h.streams") {
      e.d2h_streams = std::stoi(v);
      require(e.d2h_streams >= 1 && e.d2h_streams <= 8, PINOT_ERR_BAD_ARG, "d2h.streams: 1 .. 8");
    }
    else throw Error(PINOT_ERR_BAD_ARG, "unknown config key " + k);
  }
}
}  // namespace

extern "C" {

const char *pinot_gpu_last_error(void) { return g_last_error.c_str(); }
int32_t pinot_gpu_abi_version(void) { return PINOT_GPU_ABI_VERSION; }

int32_t pinot_gpu_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

pinot_status pinot_gpu_engine_create(int32_t device, const char *config, pinot_engine **out) {
  return guard([&] {
    require(out != nullptr, PINOT_ERR_BAD_ARG, "out");
    *out = create_engine(device, config).release();
  });
}

pinot_status pinot_gpu_engine_destroy(pinot_engine *engine) {
  return guard([&] {
    if (!engine) return;
    set_device(*engine);
    delete engine;
  });
}

pinot_status pinot_gpu_engine_set_config(pinot_engine *engine, const char *config) {
  return guard([&] {
    require(engine != nullptr, PINOT_ERR_BAD_ARG, "null engine");
    std::lock_guard<std::mutex> lk(engine->mu);
    parse_config(*engine, config);
  });
}

pinot_status pinot_gpu_segment_register(pinot_engine *engine, const pinot_segment_desc *desc,
                                        pinot_segment_handle *out) {
  return guard([&] {
    require(engine && desc && out, PINOT_ERR_BAD_ARG, "null argument");
    std::lock_guard<std::mutex> lk(engine->mu);
    set_device(*engine);
    auto seg = register_segment(*engine, *desc);
    const int64_t h = engine->next_handle++;
    engine->segments[h] = std::move(seg);
    *out = h;
  });
}

namespace {
// ImmutableSegmentLoader.load of a directory into a new handle (caller holds engine->mu)
int64_t load_segment_dir(Engine &engine, const char *index_dir) {
  SegmentDirData files;
  read_segment_dir(index_dir, files);
  const pinot_segment_desc desc = files.desc();
  set_device(engine);
  auto seg = register_segment(engine, desc);
  seg->unserved = files.skipped;
  // ColumnMinMaxValueGenerator in its default mode (TIME, CommonConstants.java:264): the time column's min / max
  // from its dictionary when the metadata lacks them (ColumnMinMaxValueGenerator.java:55-140)
  auto tc = seg->by_name.find(files.time_column);
  if (tc != seg->by_name.end()) {
    ColumnData &c = *seg->cols[tc->second];
    if (!c.has_minmax && c.card >= 1) {
      c.has_minmax = true;
      c.min_value = c.string_value(0);
      c.max_value = c.string_value(c.card - 1);
    }
  }
  if (files.has_star) {  // StarTreeLoaderUtils: the segment's star-tree, attached like pinot_gpu_segment_attach_star_tree
    const pinot_segment_desc docs = files.star_desc();
    pinot_star_tree_desc sd{files.star_tree, files.star_tree_len, &docs};
    attach_star_tree(engine, *seg, sd);
  }
  const int64_t h = engine.next_handle++;
  engine.segments[h] = std::move(seg);
  return h;
}
}  // namespace

pinot_status pinot_gpu_segment_load(pinot_engine *engine, const char *index_dir, pinot_segment_handle *out) {
  return guard([&] {
    require(engine && index_dir && out, PINOT_ERR_BAD_ARG, "null argument");
    std::lock_guard<std::mutex> lk(engine->mu);
    *out = load_segment_dir(*engine, index_dir);
  });
}

pinot_status pinot_gpu_segment_acquire(pinot_engine *engine, const char *index_dir, pinot_segment_handle *out,
                                       int32_t *cache_hit) {
  return guard([&] {
    require(engine && index_dir && out, PINOT_ERR_BAD_ARG, "null argument");
    std::string name;
    int64_t crc = 0;
    const bool has_crc = read_segment_identity(index_dir, name, crc);
    std::lock_guard<std::mutex> lk(engine->mu);
    auto it = has_crc ? engine->segment_cache.find(name) : engine->segment_cache.end();
    if (it != engine->segment_cache.end() && it->second.first == crc && engine->segments.count(it->second.second)) {
      *out = it->second.second;
      engine->acquire_refs[*out]++;
      if (cache_hit) *cache_hit = 1;
      return;
    }
    const int64_t h = load_segment_dir(*engine, index_dir);
    if (it != engine->segment_cache.end()) {  // replaced: out of the cache now, dropped once its holders release it
      const int64_t old = it->second.second;
      engine->segment_cache.erase(it);
      auto r = engine->acquire_refs.find(old);
      if (r == engine->acquire_refs.end() || r->second <= 0) {
        PINOT_HIP(hipStreamSynchronize(engine->stream));
        engine->segments.erase(old);
        if (r != engine->acquire_refs.end()) engine->acquire_refs.erase(r);
      }
    }
    if (has_crc) engine->segment_cache[name] = {crc, h};
    engine->acquire_refs[h] = 1;
    *out = h;
    if (cache_hit) *cache_hit = 0;
  });
}

pinot_status pinot_gpu_segment_attach_star_tree(pinot_engine *engine, pinot_segment_handle handle,
                                                const pinot_star_tree_desc *desc) {
  return guard([&] {
    require(engine && desc, PINOT_ERR_BAD_ARG, "null argument");
    std::lock_guard<std::mutex> lk(engine->mu);
    set_device(*engine);
    SegmentData &s = engine->seg(handle);
    require(!s.star, PINOT_ERR_BAD_ARG, s.name + ": star-tree already attached");
    attach_star_tree(*engine, s, *desc);
  });
}

pinot_status pinot_segment_read_raw_forward_index(const uint8_t *bytes, uint64_t len, int32_t data_type, int32_t num_docs,
                                          void *values) {
  return guard([&] {
    require(bytes && values && num_docs >= 0, PINOT_ERR_BAD_ARG, "null argument");
    require(data_type >= PINOT_INT && data_type <= PINOT_DOUBLE, PINOT_ERR_BAD_ARG, "fixed-width data type");
    const int w = (data_type == PINOT_INT || data_type == PINOT_FLOAT) ? 4 : 8;
    const std::vector<uint8_t> be = read_raw_chunks(bytes, len, num_docs, w, "raw forward index");
    uint8_t *out = static_cast<uint8_t *>(values);
    for (size_t i = 0; i < (size_t)num_docs; i++)
      for (int k = 0; k < w; k++) out[i * w + k] = be[i * w + (w - 1 - k)];  // big-endian -> host (little-endian)
  });
}

pinot_status pinot_gpu_segment_dir_info(const char *index_dir, int32_t *num_docs, int32_t *num_columns,
                                        int32_t *num_skipped) {
  return guard([&] {
    require(index_dir != nullptr, PINOT_ERR_BAD_ARG, "null argument");
    SegmentDirData files;
    read_segment_dir(index_dir, files);
    validate_segment(files.desc());
    if (num_docs) *num_docs = files.num_docs;
    if (num_columns) *num_columns = (int32_t)files.cols.size();
    if (num_skipped) *num_skipped = (int32_t)files.skipped.size();
  });
}

pinot_status pinot_gpu_segment_register_synthetic_ex(pinot_engine *engine, const char *name, int32_t num_docs,
                                                     int32_t num_columns, const char *const *column_names,
                                                     const int32_t *cardinalities, const int32_t *kinds, uint64_t seed,
                                                     pinot_segment_handle *out) {
  return guard([&] {
    require(engine && out, PINOT_ERR_BAD_ARG, "null argument");
    std::lock_guard<std::mutex> lk(engine->mu);
    set_device(*engine);
    auto seg = register_synthetic(*engine, name, num_docs, num_columns, column_names, cardinalities, seed, kinds);
    const int64_t h = engine->next_handle++;
    engine->segments[h] = std::move(seg);
    *out = h;
  });
}

pinot_status pinot_gpu_segment_register_synthetic(pinot_engine *engine, const char *name, int32_t num_docs,
                                                  int32_t num_columns, const char *const *column_names,
                                                  const int32_t *cardinalities, uint64_t seed,
                                                  pinot_segment_handle *out) {
  return pinot_gpu_segment_register_synthetic_ex(engine, name, num_docs, num_columns, column_names, cardinalities,
                                                 nullptr, seed, out);
}

pinot_status pinot_gpu_segment_release(pinot_engine *engine, pinot_segment_handle handle) {
  return guard([&] {
    require(engine != nullptr, PINOT_ERR_BAD_ARG, "null engine");
    std::lock_guard<std::mutex> lk(engine->mu);
    set_device(*engine);
    require(engine->segments.count(handle) == 1, PINOT_ERR_BAD_ARG, "unknown segment handle");
    auto r = engine->acquire_refs.find(handle);
    if (r != engine->acquire_refs.end()) {  // an acquired handle: the last reference drops the device copy
      if (--r->second > 0) return;
      engine->acquire_refs.erase(r);
    }
    PINOT_HIP(hipStreamSynchronize(engine->stream));
    engine->segments.erase(handle);
    for (auto it = engine->segment_cache.begin(); it != engine->segment_cache.end(); ++it)
      if (it->second.second == handle) {
        engine->segment_cache.erase(it);
        break;
      }
  });
}

pinot_status pinot_gpu_transcode_raw(pinot_engine *engine, const pinot_column_desc *column, int32_t num_docs,
                                     int32_t on_device, int32_t *cardinality, int32_t *bits_per_value,
                                     uint8_t *dictionary, uint64_t dictionary_cap, uint64_t *dictionary_len,
                                     uint8_t *forward_index, uint64_t forward_cap, uint64_t *forward_len) {
  return guard([&] {
    require(engine && column && cardinality && bits_per_value && dictionary_len && forward_len, PINOT_ERR_BAD_ARG,
            "null argument");
    std::lock_guard<std::mutex> lk(engine->mu);
    set_device(*engine);
    TranscodedColumn tc;
    const bool saved = engine->raw_device;
    engine->raw_device = on_device != 0;
    bool raw = false;
    try {
      raw = transcode_column(*engine, *column, num_docs, tc);
    } catch (...) {
      engine->raw_device = saved;
      throw;
    }
    engine->raw_device = saved;
    require(raw, PINOT_ERR_BAD_ARG, "not a raw column");
    *cardinality = tc.desc.cardinality;
    *bits_per_value = tc.desc.bits_per_value;
    *dictionary_len = tc.dictionary.size();
    *forward_len = tc.forward_index.size();
    if (dictionary) {
      require(dictionary_cap >= tc.dictionary.size(), PINOT_ERR_BAD_ARG, "dictionary buffer too small");
      memcpy(dictionary, tc.dictionary.data(), tc.dictionary.size());
    }
    if (forward_index) {
      require(forward_cap >= tc.forward_index.size(), PINOT_ERR_BAD_ARG, "forward index buffer too small");
      memcpy(forward_index, tc.forward_index.data(), tc.forward_index.size());
    }
  });
}

pinot_status pinot_gpu_segment_validate(const pinot_segment_desc *desc) {
  return guard([&] {
    require(desc != nullptr, PINOT_ERR_BAD_ARG, "null descriptor");
    validate_segment(*desc);
  });
}

pinot_status pinot_gpu_segment_device_bytes(pinot_engine *engine, pinot_segment_handle handle, uint64_t *out) {
  return guard([&] {
    require(engine && out, PINOT_ERR_BAD_ARG, "null argument");
    std::lock_guard<std::mutex> lk(engine->mu);
    *out = engine->seg(handle).device_bytes;
  });
}

pinot_status pinot_gpu_filter(pinot_engine *engine, pinot_segment_handle segment, int32_t num_filter_nodes,
                              const pinot_filter_node *filter, uint64_t *bitset_out, int64_t *count_out) {
  return guard([&] {
    require(engine != nullptr, PINOT_ERR_BAD_ARG, "null engine");
    require(num_filter_nodes == 0 || filter != nullptr, PINOT_ERR_BAD_ARG, "filter nodes");
    std::lock_guard<std::mutex> lk(engine->mu);
    set_device(*engine);
    SegmentData &s = engine->seg(segment);
    std::unique_ptr<FilterTreeInput> tree;
    if (num_filter_nodes > 0) tree = std::make_unique<FilterTreeInput>(decode_filter(num_filter_nodes, filter));
    exec_filter(*engine, s, tree.get(), bitset_out, count_out);
  });
}

pinot_status pinot_gpu_aggregate(pinot_engine *engine, const pinot_segment_handle *segments, int32_t num_segments,
                                 const pinot_query *query, pinot_agg_result *out, pinot_exec_stats *stats) {
  return guard([&] {
    require(engine && out, PINOT_ERR_BAD_ARG, "null argument");
    check_query(query);
    require(query->num_group_by == 0, PINOT_ERR_BAD_ARG, "group-by query passed to pinot_gpu_aggregate");
    const auto t0 = std::chrono::steady_clock::now();
    std::lock_guard<std::mutex> lk(engine->mu);
    set_device(*engine);
    DeadlineScope ds(*engine, query->timeout_ms);
    const std::vector<SegmentData *> segs = resolve(*engine, segments, num_segments);
    const std::vector<SegmentData *> kept = prune_for_query(segs, *query);
    const auto t1 = std::chrono::steady_clock::now();
    if (kept.empty()) {  // every segment pruned (ServerQueryExecutorV1Impl.java:187-196)
      agg_identities(*query, out);
      if (stats) memset(stats, 0, sizeof(*stats));
    } else {
      engine->star_answered.clear();
      exec_aggregate(*engine, kept, *query, out, stats);
      exact_filter_stats(*engine, kept, *query, stats);
    }
    if (engine->host_phases)
      fprintf(stderr, "[pinot_gpu] aggregate C-ABI phases (us): resolve+prune %.1f, execute %.1f\n",
              std::chrono::duration<double, std::micro>(t1 - t0).count(), elapsed_ms(t1) * 1e3);
    if (stats) {
      if (query->pruners) stats->num_total_raw_docs = total_docs(segs);
      stats->host_ms = elapsed_ms(t0);
    }
  });
}

namespace {
pinot_status group_by_call(pinot_engine *engine, const pinot_segment_handle *segments, int32_t num_segments,
                           const pinot_query *query, int32_t top_n, pinot_groupby_result **out, pinot_exec_stats *stats) {
  return guard([&] {
    require(engine && out, PINOT_ERR_BAD_ARG, "null argument");
    require(top_n >= 0, PINOT_ERR_BAD_ARG, "top_n must be positive (AggregationGroupByTrimmingService.java:52)");
    check_query(query);
    require(query->num_group_by >= 1, PINOT_ERR_BAD_ARG, "aggregation-only query passed to pinot_gpu_group_by");
    const auto t0 = std::chrono::steady_clock::now();
    std::lock_guard<std::mutex> lk(engine->mu);
    set_device(*engine);
    DeadlineScope ds(*engine, query->timeout_ms);
    const std::vector<SegmentData *> segs = resolve(*engine, segments, num_segments);
    const std::vector<SegmentData *> kept = prune_for_query(segs, *query);
    const auto t1 = std::chrono::steady_clock::now();
    std::unique_ptr<GroupByResult> r;
    if (kept.empty()) {
      r = empty_group_result(*query);
      if (stats) memset(stats, 0, sizeof(*stats));
    } else {
      engine->star_answered.clear();
      struct TrimScope {
        Engine &e;
        ~TrimScope() { e.trim_top_n = 0; }
      } ts{*engine};
      engine->trim_top_n = top_n;
      r = exec_group_by(*engine, kept, *query, stats);
      exact_filter_stats(*engine, kept, *query, stats);
    }
    if (stats) {
      if (query->pruners) stats->num_total_raw_docs = total_docs(segs);
      stats->host_ms = elapsed_ms(t0);
    }
    const auto t2 = std::chrono::steady_clock::now();
    auto *res = new pinot_groupby_result();
    static_cast<GroupByResult &>(*res) = std::move(*r);
    *out = res;
    if (engine->host_phases) {
      auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
      fprintf(stderr, "[pinot_gpu] group-by C-ABI phases (us): resolve+prune %.1f, execute %.1f, result %.1f\n",
              us(t0, t1), us(t1, t2), us(t2, std::chrono::steady_clock::now()));
    }
  });
}
}  // namespace

pinot_status pinot_gpu_group_by(pinot_engine *engine, const pinot_segment_handle *segments, int32_t num_segments,
                                const pinot_query *query, pinot_groupby_result **out, pinot_exec_stats *stats) {
  return group_by_call(engine, segments, num_segments, query, 0, out, stats);
}

pinot_status pinot_gpu_group_by_top(pinot_engine *engine, const pinot_segment_handle *segments, int32_t num_segments,
                                    const pinot_query *query, int32_t top_n, pinot_groupby_result **out,
                                    pinot_exec_stats *stats) {
  if (top_n <= 0)
    return guard([&] { require(false, PINOT_ERR_BAD_ARG, "top_n must be positive (AggregationGroupByTrimmingService.java:52)"); });
  return group_by_call(engine, segments, num_segments, query, top_n, out, stats);
}

int64_t pinot_groupby_num_groups(const pinot_groupby_result *r) { return r ? (int64_t)r->raw_keys.size() : 0; }
int32_t pinot_groupby_num_columns(const pinot_groupby_result *r) { return r ? r->num_columns : 0; }

const char *pinot_groupby_key(const pinot_groupby_result *r, int64_t group) {
  if (!r || group < 0 || group >= (int64_t)r->raw_keys.size()) return nullptr;
  return r->key(group).c_str();
}

pinot_status pinot_groupby_values(const pinot_groupby_result *r, int32_t fn, int64_t *counts, double *values) {
  return guard([&] {
    require(r && fn >= 0 && fn < (int32_t)r->functions.size(), PINOT_ERR_BAD_ARG, "function index");
    const size_t n = r->raw_keys.size();
    if (counts && n) memcpy(counts, r->counts[r->counts_shared ? 0 : fn].data(), n * 8);
    if (values && n) memcpy(values, r->values[fn].data(), n * 8);
  });
}

pinot_status pinot_groupby_hll(const pinot_groupby_result *r, int32_t fn, uint8_t *registers, int64_t *cardinalities) {
  return guard([&] {
    require(r && fn >= 0 && fn < (int32_t)r->functions.size(), PINOT_ERR_BAD_ARG, "function index");
    require(sv_function(r->functions[fn]) == PINOT_AGG_DISTINCTCOUNTHLL, PINOT_ERR_BAD_ARG, "not a DISTINCTCOUNTHLL function");
    const size_t n = r->raw_keys.size();
    if (registers && n) group_by_hll_registers(*r, fn, registers);
    if (cardinalities && n) memcpy(cardinalities, r->hll_card[fn].data(), n * 8);
  });
}

pinot_status pinot_datatable_aggregation(const pinot_query *query, const pinot_agg_result *results,
                                         const pinot_exec_stats *stats, const pinot_datatable_server *server,
                                         uint8_t *buf, uint64_t buf_len, uint64_t *out_len) {
  return guard([&] {
    require(results && stats && out_len, PINOT_ERR_BAD_ARG, "null argument");
    check_query(query);
    const std::vector<uint8_t> b = aggregation_datatable(*query, results, *stats, server);
    *out_len = b.size();
    if (!buf) return;
    require(buf_len >= b.size(), PINOT_ERR_BAD_ARG, "DataTable buffer too small");
    memcpy(buf, b.data(), b.size());
  });
}

pinot_status pinot_datatable_group_by(const pinot_query *query, const pinot_groupby_result *result,
                                      const int64_t *const *fn_groups, const int64_t *fn_num_groups,
                                      const pinot_exec_stats *stats, const pinot_datatable_server *server,
                                      const uint8_t **data, uint64_t *len) {
  return guard([&] {
    require(result && stats && data && len, PINOT_ERR_BAD_ARG, "null argument");
    check_query(query);
    require(query->num_aggregations == (int32_t)result->functions.size(), PINOT_ERR_BAD_ARG,
            "query and result disagree on the aggregations");
    require(!fn_groups || fn_num_groups, PINOT_ERR_BAD_ARG, "fn_groups without fn_num_groups");
    result->datatables.push_back(group_by_datatable(*query, *result, fn_groups, fn_num_groups, *stats, server));
    *data = result->datatables.back().data();
    *len = result->datatables.back().size();
  });
}

pinot_status pinot_datatable_empty(const pinot_query *query, int64_t total_docs, const pinot_datatable_server *server,
                                   uint8_t *buf, uint64_t buf_len, uint64_t *out_len) {
  return guard([&] {
    require(out_len != nullptr, PINOT_ERR_BAD_ARG, "null argument");
    check_query(query);
    const std::vector<uint8_t> b = empty_datatable(*query, total_docs, server);
    *out_len = b.size();
    if (!buf) return;
    require(buf_len >= b.size(), PINOT_ERR_BAD_ARG, "DataTable buffer too small");
    memcpy(buf, b.data(), b.size());
  });
}

pinot_status pinot_broker_reduce(const pinot_query *query, int32_t num_tables, const uint8_t *const *tables,
                                 const uint64_t *lens, int32_t top_n, char *buf, uint64_t buf_len, uint64_t *out_len) {
  return guard([&] {
    require(out_len != nullptr && num_tables >= 0 && (num_tables == 0 || (tables && lens)), PINOT_ERR_BAD_ARG,
            "null argument");
    check_query(query);
    const std::string j = broker_reduce(*query, num_tables, tables, lens, top_n);
    *out_len = j.size();
    if (!buf) return;
    require(buf_len >= j.size(), PINOT_ERR_BAD_ARG, "response buffer too small");
    memcpy(buf, j.data(), j.size());
  });
}

pinot_status pinot_gpu_prune_segments(pinot_engine *engine, const pinot_segment_handle *segments, int32_t num_segments,
                                      const pinot_query *query, int32_t pruners, uint8_t *pruned,
                                      int64_t *total_raw_docs) {
  return guard([&] {
    require(engine && pruned, PINOT_ERR_BAD_ARG, "null argument");
    require(num_segments >= 0 && (num_segments == 0 || segments), PINOT_ERR_BAD_ARG, "segments");
    check_query(query);
    // processQuery checks the scheduling wait against the budget before it prunes (:116-126)
    require(query->timeout_ms >= 0, PINOT_ERR_TIMEOUT, "query budget already spent before execution");
    std::unique_ptr<FilterTreeInput> tree;
    if (query->num_filter_nodes > 0)
      tree = std::make_unique<FilterTreeInput>(decode_filter(query->num_filter_nodes, query->filter));
    std::lock_guard<std::mutex> lk(engine->mu);
    int64_t total = 0;
    for (int32_t i = 0; i < num_segments; i++) {
      const SegmentData &s = engine->seg(segments[i]);
      total += s.num_docs;
      pruned[i] = prune_segment(s, *query, tree.get(), pruners) ? 1 : 0;
    }
    if (total_raw_docs) *total_raw_docs = total;
  });
}

pinot_status pinot_segment_prune(const pinot_segment_desc *desc, const pinot_query *query, int32_t pruners,
                                 int32_t *pruned) {
  return guard([&] {
    require(desc && pruned, PINOT_ERR_BAD_ARG, "null argument");
    check_query(query);
    std::unique_ptr<FilterTreeInput> tree;
    if (query->num_filter_nodes > 0)
      tree = std::make_unique<FilterTreeInput>(decode_filter(query->num_filter_nodes, query->filter));
    *pruned = prune_segment_desc(*desc, *query, tree.get(), pruners) ? 1 : 0;
  });
}

pinot_status pinot_groupby_raw_keys(const pinot_groupby_result *r, int64_t *keys) {
  return guard([&] {
    require(r && keys, PINOT_ERR_BAD_ARG, "null argument");
    if (!r->raw_keys.empty()) memcpy(keys, r->raw_keys.data(), r->raw_keys.size() * 8);
  });
}

pinot_status pinot_groupby_export_keys(const pinot_groupby_result *r, char *buf, uint64_t buf_len, int64_t *offsets,
                                       uint64_t *bytes_needed) {
  return guard([&] {
    require(r != nullptr, PINOT_ERR_BAD_ARG, "null result");
    const uint64_t need = r->export_keys(buf, buf_len, offsets);
    if (bytes_needed) *bytes_needed = need;
  });
}

pinot_status pinot_groupby_trim(const pinot_groupby_result *r, int32_t top_n, int32_t fn, int64_t *groups,
                                int64_t *num_out) {
  return guard([&] {
    require(r && num_out && fn >= 0 && fn < (int32_t)r->functions.size(), PINOT_ERR_BAD_ARG, "function index");
    require(top_n > 0, PINOT_ERR_BAD_ARG, "top_n must be positive (AggregationGroupByTrimmingService.java:52)");
    const std::vector<int64_t> kept = r->trim(top_n, fn);
    *num_out = (int64_t)kept.size();
    if (groups && !kept.empty()) memcpy(groups, kept.data(), kept.size() * 8);
  });
}

void pinot_groupby_free(pinot_groupby_result *r) { delete r; }

pinot_status pinot_gpu_group_by_layout(pinot_engine *engine, const pinot_segment_handle *segments,
                                       int32_t num_segments, const pinot_query *query, pinot_partial_layout *layout) {
  return guard([&] {
    require(engine && layout, PINOT_ERR_BAD_ARG, "null argument");
    check_query(query);
    require(query->num_aggregations <= 8, PINOT_ERR_UNSUPPORTED, "at most 8 aggregations");
    std::lock_guard<std::mutex> lk(engine->mu);
    set_device(*engine);
    exec_group_by_layout(*engine, resolve(*engine, segments, num_segments), *query, layout);
  });
}

pinot_status pinot_gpu_group_by_partial(pinot_engine *engine, const pinot_segment_handle *segments,
                                        int32_t num_segments, const pinot_query *query, int64_t *counts_dev,
                                        void *const *accs_dev, pinot_exec_stats *stats) {
  return guard([&] {
    require(engine && counts_dev, PINOT_ERR_BAD_ARG, "null argument");
    check_query(query);
    std::lock_guard<std::mutex> lk(engine->mu);
    set_device(*engine);
    exec_group_by_partial(*engine, resolve(*engine, segments, num_segments), *query, counts_dev, accs_dev, stats);
  });
}

pinot_status pinot_gpu_group_by_finalize(pinot_engine *engine, const pinot_segment_handle *segments,
                                         int32_t num_segments, const pinot_query *query, const int64_t *counts_dev,
                                         void *const *accs_dev, pinot_groupby_result **out) {
  return guard([&] {
    require(engine && counts_dev && out, PINOT_ERR_BAD_ARG, "null argument");
    check_query(query);
    std::lock_guard<std::mutex> lk(engine->mu);
    set_device(*engine);
    auto r = exec_group_by_finalize(*engine, resolve(*engine, segments, num_segments), *query, counts_dev, accs_dev);
    auto *res = new pinot_groupby_result();
    static_cast<GroupByResult &>(*res) = std::move(*r);
    *out = res;
  });
}

pinot_status pinot_gpu_server_create(const int32_t *devices, int32_t num_devices, const char *config, pinot_server **out) {
  return guard([&] {
    require(out != nullptr, PINOT_ERR_BAD_ARG, "out");
    auto s = std::make_unique<pinot_server>();
    s->impl = server_create(devices, num_devices, config);
    *out = s.release();
  });
}

pinot_status pinot_gpu_server_unique_id(uint8_t *unique_id) {
  return guard([&] {
    require(unique_id != nullptr, PINOT_ERR_BAD_ARG, "unique_id");
    server_unique_id(unique_id);
  });
}

pinot_status pinot_gpu_server_create_rank(int32_t device, int32_t nranks, int32_t rank, const uint8_t *unique_id,
                                          const char *config, pinot_server **out) {
  return guard([&] {
    require(out != nullptr, PINOT_ERR_BAD_ARG, "out");
    auto s = std::make_unique<pinot_server>();
    s->impl = server_create_rank(device, nranks, rank, unique_id, config);
    *out = s.release();
  });
}

pinot_status pinot_gpu_server_destroy(pinot_server *server) {
  return guard([&] { delete server; });
}

pinot_status pinot_gpu_server_last_phases(const pinot_server *server, double *ms, int32_t n) {
  return guard([&] {
    require(server && server->impl && ms && n >= 0, PINOT_ERR_BAD_ARG, "null argument");
    server_last_phases(*server->impl, ms, n);
  });
}

int32_t pinot_gpu_server_num_engines(const pinot_server *server) {
  return server && server->impl ? server_num_engines(*server->impl) : 0;
}

pinot_status pinot_gpu_server_engine(pinot_server *server, int32_t index, pinot_engine **out) {
  return guard([&] {
    require(server && server->impl && out, PINOT_ERR_BAD_ARG, "null argument");
    *out = static_cast<pinot_engine *>(server_engine(*server->impl, index));
  });
}

static std::vector<SegmentRef> server_refs(const pinot_segment_ref *segments, int32_t n) {
  require(n >= 0 && (n == 0 || segments != nullptr), PINOT_ERR_BAD_ARG, "segments");
  std::vector<SegmentRef> refs;
  for (int32_t i = 0; i < n; i++) refs.push_back(SegmentRef{segments[i].engine, segments[i].handle});
  return refs;
}

pinot_status pinot_gpu_server_aggregate(pinot_server *server, const pinot_segment_ref *segments, int32_t num_segments,
                                        const pinot_query *query, pinot_agg_result *out, pinot_exec_stats *stats) {
  return guard([&] {
    require(server && server->impl && out, PINOT_ERR_BAD_ARG, "null argument");
    check_query(query);
    require(query->num_group_by == 0, PINOT_ERR_BAD_ARG, "group-by query passed to pinot_gpu_server_aggregate");
    const auto t0 = std::chrono::steady_clock::now();
    server_aggregate(*server->impl, server_refs(segments, num_segments), *query, out, stats);
    if (stats) stats->host_ms = elapsed_ms(t0);
  });
}

static pinot_status server_group_by_call(pinot_server *server, const pinot_segment_ref *segments, int32_t num_segments,
                                         const pinot_query *query, int32_t top_n, pinot_groupby_result **out,
                                         pinot_exec_stats *stats) {
  return guard([&] {
    require(server && server->impl && out, PINOT_ERR_BAD_ARG, "null argument");
    check_query(query);
    require(query->num_group_by >= 1, PINOT_ERR_BAD_ARG, "aggregation-only query passed to pinot_gpu_server_group_by");
    require(top_n >= 0, PINOT_ERR_BAD_ARG, "top_n must be >= 0");
    const auto t0 = std::chrono::steady_clock::now();
    auto r = server_group_by(*server->impl, server_refs(segments, num_segments), *query, stats, top_n);
    if (stats) stats->host_ms = elapsed_ms(t0);
    auto *res = new pinot_groupby_result();
    static_cast<GroupByResult &>(*res) = std::move(*r);
    *out = res;
  });
}

pinot_status pinot_gpu_server_group_by(pinot_server *server, const pinot_segment_ref *segments, int32_t num_segments,
                                       const pinot_query *query, pinot_groupby_result **out, pinot_exec_stats *stats) {
  return server_group_by_call(server, segments, num_segments, query, 0, out, stats);
}

pinot_status pinot_gpu_server_group_by_top(pinot_server *server, const pinot_segment_ref *segments, int32_t num_segments,
                                           const pinot_query *query, int32_t top_n, pinot_groupby_result **out,
                                           pinot_exec_stats *stats) {
  return server_group_by_call(server, segments, num_segments, query, top_n, out, stats);
}

pinot_status pinot_gpu_server_prune_segments(pinot_server *server, const pinot_segment_ref *segments,
                                             int32_t num_segments, const pinot_query *query, int32_t pruners,
                                             uint8_t *pruned, int64_t *total_raw_docs) {
  return guard([&] {
    require(server && server->impl && pruned, PINOT_ERR_BAD_ARG, "null argument");
    check_query(query);
    require(query->timeout_ms >= 0, PINOT_ERR_TIMEOUT, "query budget already spent before execution");
    const std::vector<SegmentRef> refs = server_refs(segments, num_segments);
    std::unique_ptr<FilterTreeInput> tree;
    if (query->num_filter_nodes > 0)
      tree = std::make_unique<FilterTreeInput>(decode_filter(query->num_filter_nodes, query->filter));
    const int32_t ne = server_num_engines(*server->impl);
    int64_t total = 0;
    for (size_t i = 0; i < refs.size(); i++) {
      require(refs[i].engine >= 0 && refs[i].engine < ne, PINOT_ERR_BAD_ARG, "segment ref: no such engine");
      Engine &e = *static_cast<Engine *>(server_engine(*server->impl, refs[i].engine));
      std::lock_guard<std::mutex> lk(e.mu);
      const SegmentData &s = e.seg(refs[i].handle);
      total += s.num_docs;
      pruned[i] = prune_segment(s, *query, tree.get(), pruners) ? 1 : 0;
    }
    if (total_raw_docs) *total_raw_docs = total;
  });
}

pinot_status pinot_gpu_synchronize(pinot_engine *engine) {
  return guard([&] {
    require(engine != nullptr, PINOT_ERR_BAD_ARG, "null engine");
    set_device(*engine);
    PINOT_HIP(hipStreamSynchronize(engine->stream));
  });
}

pinot_status pinot_gpu_last_kernel_ms(pinot_engine *engine, int32_t kind, double *ms, int64_t *launches) {
  return guard([&] {
    require(engine && kind >= 0 && kind < 2, PINOT_ERR_BAD_ARG, "kind");
    if (ms) *ms = engine->last_ms[kind];
    if (launches) *launches = engine->last_launches[kind];
  });
}

pinot_status pinot_gpu_engine_stat(pinot_engine *engine, const char *name, int64_t *value) {
  return guard([&] {
    require(engine && name && value, PINOT_ERR_BAD_ARG, "engine, name, value");
    const std::string n = name;
    if (n == "group.ring_queries") *value = engine->ring_queries;
    else if (n == "group.ring_fallbacks") *value = engine->ring_fallbacks;
    else if (n == "group.ring_qfilter_queries") *value = engine->ring_qfilter_queries;
    else if (n == "group.ring_rec_bytes") *value = engine->ring_last_rec_bytes;
    else if (n == "group.ring_hll_slot") *value = engine->ring_last_hll_slot;
    else if (n == "group.ring_last_status") *value = engine->ring_last_status;
    else if (n == "raw.device_columns") *value = engine->raw_device_columns;
    else if (n == "raw.host_fallbacks") *value = engine->raw_host_fallbacks;
    else if (n == "group.last_instance") *value = engine->last_group_instance;
    else if (n == "exec.last_pre_segments") *value = engine->last_pre_segments;
    else require(false, PINOT_ERR_BAD_ARG, "unknown engine stat");
  });
}

}  // extern "C"
