// Server → broker wire format of a query's combined result: IntermediateResultsBlock.getDataTable
// (PC/operator/blocks/IntermediateResultsBlock.java:206-317) built with DataTableBuilder
// (PC/common/datatable/DataTableBuilder.java:72-160) and written by DataTableImplV2.toBytes
// (PC/common/datatable/DataTableImplV2.java:233-347); object cells per ObjectSerDeUtils
// (PC/common/ObjectSerDeUtils.java:47-98 type ids, :144-330 serializers). PC = pinot-core/src/main/java/org/apache/pinot/core.
//
// Layout (all integers big-endian, DataOutputStream):
//   int VERSION (2), int numRows, int numColumns,
//   (int start, int length) x 5 for: dictionary map, metadata, data schema, fixed-size rows, variable-size data
//   (HEADER_SIZE = 13 ints; starts are absolute offsets), then the five sections back to back.
// Maps the reference builds as java.util.HashMap are written in HashMap iteration order (bucket (h ^ h >>> 16) &
// (capacity - 1) of String.hashCode / Integer.hashCode, insertion order within a bucket), so the metadata and
// dictionary sections are byte-identical to the reference's. The group-by result maps are written in ascending raw
// key order: the reference's map is a ConcurrentHashMap filled by concurrent segment threads, whose order is not
// deterministic either; the broker reads it back into a HashMap (order-free).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "engine.h"

namespace pinot {
void host_parallel(size_t n, const std::function<void(size_t)> &fn);  // executor.cpp: the engine's task pool
size_t host_parallelism();

namespace {


class Out {
 public:
  std::vector<uint8_t> b;
  uint8_t *grow(size_t n) {  // n more bytes at the end (amortised doubling)
    const size_t at = b.size();
    if (at + n > b.capacity()) b.reserve(std::max<size_t>(2 * b.capacity(), at + n + 4096));
    b.resize(at + n);
    return b.data() + at;
  }
  void i32(int32_t v) {
    const uint32_t u = (uint32_t)v;
    uint8_t *x = grow(4);
    x[0] = (uint8_t)(u >> 24);
    x[1] = (uint8_t)(u >> 16);
    x[2] = (uint8_t)(u >> 8);
    x[3] = (uint8_t)u;
  }
  void i64(int64_t v) {
    const uint64_t u = (uint64_t)v;
    uint8_t *x = grow(8);
    for (int i = 0; i < 8; i++) x[i] = (uint8_t)(u >> (56 - 8 * i));
  }
  void f64(double d) {  // Double.doubleToRawLongBits
    int64_t v;
    memcpy(&v, &d, 8);
    i64(v);
  }
  void bytes(const void *p, size_t n) {
    if (n) memcpy(grow(n), p, n);
  }
  void str(const std::string &s) {  // int length + UTF-8 bytes (StringUtil.encodeUtf8)
    i32((int32_t)s.size());
    bytes(s.data(), s.size());
  }
  void put_i32_at(size_t off, int32_t v) {
    const uint32_t u = (uint32_t)v;
    b[off] = (uint8_t)(u >> 24);
    b[off + 1] = (uint8_t)(u >> 16);
    b[off + 2] = (uint8_t)(u >> 8);
    b[off + 3] = (uint8_t)u;
  }
};

inline uint8_t *put_be32(uint8_t *x, uint32_t u) {
  x[0] = (uint8_t)(u >> 24);
  x[1] = (uint8_t)(u >> 16);
  x[2] = (uint8_t)(u >> 8);
  x[3] = (uint8_t)u;
  return x + 4;
}
inline uint8_t *put_be64(uint8_t *x, uint64_t u) {
  for (int i = 0; i < 8; i++) x[i] = (uint8_t)(u >> (56 - 8 * i));
  return x + 8;
}

// java.lang.String.hashCode over the UTF-16 code units of a UTF-8 string.
int32_t java_string_hash(const std::string &s) {
  uint32_t h = 0;
  for (size_t i = 0; i < s.size();) {
    const uint8_t c = (uint8_t)s[i];
    uint32_t cp;
    int len;
    if (c < 0x80) { cp = c; len = 1; }
    else if ((c >> 5) == 6 && i + 1 < s.size()) { cp = ((c & 0x1Fu) << 6) | (s[i + 1] & 0x3Fu); len = 2; }
    else if ((c >> 4) == 14 && i + 2 < s.size()) { cp = ((c & 0x0Fu) << 12) | ((s[i + 1] & 0x3Fu) << 6) | (s[i + 2] & 0x3Fu); len = 3; }
    else if (i + 3 < s.size()) {
      cp = ((c & 0x07u) << 18) | ((s[i + 1] & 0x3Fu) << 12) | ((s[i + 2] & 0x3Fu) << 6) | (s[i + 3] & 0x3Fu);
      len = 4;
    } else { cp = c; len = 1; }
    i += len;
    if (cp >= 0x10000) {  // surrogate pair
      cp -= 0x10000;
      h = 31u * h + (0xD800u + (cp >> 10));
      h = 31u * h + (0xDC00u + (cp & 0x3FFu));
    } else {
      h = 31u * h + cp;
    }
  }
  return (int32_t)h;
}

// Iteration order of a java.util.HashMap filled with keys of these hashes in this order (default capacity 16,
// load factor 0.75, doubling; resizes keep the relative order of a bucket's entries; small maps never treeify).
std::vector<size_t> java_hashmap_order(const std::vector<int32_t> &hashes) {
  size_t cap = 16;
  while ((double)hashes.size() > 0.75 * (double)cap) cap <<= 1;
  std::vector<std::vector<size_t>> buckets(cap);
  for (size_t i = 0; i < hashes.size(); i++) {
    const uint32_t h = (uint32_t)hashes[i];
    buckets[(h ^ (h >> 16)) & (cap - 1)].push_back(i);
  }
  std::vector<size_t> order;
  for (auto &bk : buckets) order.insert(order.end(), bk.begin(), bk.end());
  return order;
}

// AggregationFunction.getColumnName (CountAggregationFunction.java:43-45 "count_star"; others
// AggregationFunctionType.getName() + "_" + column, e.g. SumAggregationFunction.java:42-44).
std::string aggregation_column_name(const pinot_agg_spec &a) {
  const std::string col = (a.column && *a.column) ? a.column : "*";
  switch (a.function) {
    case PINOT_AGG_COUNT: return "count_star";
    case PINOT_AGG_SUM: return "sum_" + col;
    case PINOT_AGG_MIN: return "min_" + col;
    case PINOT_AGG_MAX: return "max_" + col;
    case PINOT_AGG_AVG: return "avg_" + col;
    case PINOT_AGG_DISTINCTCOUNTHLL: return "distinctCountHLL_" + col;
    // the *MVAggregationFunction overrides (e.g. CountMVAggregationFunction.java:37-40): COUNTMV.getName() + "_" + column
    case PINOT_AGG_COUNTMV: return "countMV_" + col;
    case PINOT_AGG_SUMMV: return "sumMV_" + col;
    case PINOT_AGG_MINMV: return "minMV_" + col;
    case PINOT_AGG_MAXMV: return "maxMV_" + col;
    case PINOT_AGG_AVGMV: return "avgMV_" + col;
    case PINOT_AGG_DISTINCTCOUNTHLLMV: return "distinctCountHLLMV_" + col;
    default: throw Error(PINOT_ERR_BAD_ARG, "aggregation function");
  }
}

enum ObjType : int32_t { OBJ_STRING = 0, OBJ_LONG = 1, OBJ_DOUBLE = 2, OBJ_AVG_PAIR = 4, OBJ_HLL = 6, OBJ_MAP = 8 };

// stream-lib 2.7.0 HyperLogLog.getBytes (log2m 8): int log2m, int registerSet.size * 4, then the RegisterSet's 43
// int words, register p in word p / 6 at bit 5 * (p % 6) (RegisterSet.set; LOG2_BITS_PER_WORD 6, REGISTER_SIZE 5).
// HyperLogLog.getBytes into x (8 + 43 * 4 bytes): log2m, register-set size, the 43 words of six 5-bit registers.
void hll_bytes_at(uint8_t *x, const uint8_t *regs) {
  x = put_be32(put_be32(x, 8u), 43u * 4u);
  for (int w = 0; w < 42; w++) {
    const uint8_t *r = regs + 6 * w;
    x = put_be32(x, (uint32_t)(r[0] & 0x1F) | (uint32_t)(r[1] & 0x1F) << 5 | (uint32_t)(r[2] & 0x1F) << 10 |
                        (uint32_t)(r[3] & 0x1F) << 15 | (uint32_t)(r[4] & 0x1F) << 20 | (uint32_t)(r[5] & 0x1F) << 25);
  }
  put_be32(x, (uint32_t)(regs[252] & 0x1F) | (uint32_t)(regs[253] & 0x1F) << 5 | (uint32_t)(regs[254] & 0x1F) << 10 |
                  (uint32_t)(regs[255] & 0x1F) << 15);
}

void hll_bytes(Out &o, const uint8_t *regs) { hll_bytes_at(o.grow(8 + 43 * 4), regs); }

// Uninitialised pinned staging bytes (PinnedCache-backed): the device registers' copy target.
struct PinnedBytes {
  void *p = nullptr;
  size_t bytes = 0;
  bool pinned = false;
  explicit PinnedBytes(size_t n) {
    bytes = size_t(1) << PinnedCache::size_class(n < 4096 ? 4096 : n);
    p = PinnedCache::get().take(bytes);
    pinned = p != nullptr || hipHostMalloc(&p, bytes, hipHostMallocDefault) == hipSuccess;
    if (!pinned) {
      (void)hipGetLastError();
      p = std::malloc(bytes);
      if (!p) throw std::bad_alloc();
    }
  }
  ~PinnedBytes() {
    if (!pinned) std::free(p);
    else if (!PinnedCache::get().give(p, bytes)) (void)hipHostFree(p);
  }
  PinnedBytes(const PinnedBytes &) = delete;
  PinnedBytes &operator=(const PinnedBytes &) = delete;
  uint8_t *data() { return static_cast<uint8_t *>(p); }
};

// A group key's value strings (GroupByResult::key's '\t'-joined parts); returns the joined length.
size_t group_key_parts(const GroupByResult &r, int64_t g, const std::string **part) {
  const size_t nc = r.gcard.size();
  size_t len = nc ? nc - 1 : 0;
  int64_t k = r.raw_keys[g];
  for (size_t j = 0; j < nc; j++) {
    if (!r.key_ids.empty()) {
      part[j] = &r.gvalues[j][r.key_ids[g * nc + j]];
    } else {
      part[j] = &r.gvalues[j][k % r.gcard[j]];
      k /= r.gcard[j];
    }
    len += part[j]->size();
  }
  return len;
}

// DataSchema.toBytes (pinot-common/.../utils/DataSchema.java:114-139): names, then type names.
void schema_bytes(Out &o, const std::vector<std::string> &names, const std::vector<std::string> &types) {
  o.i32((int32_t)names.size());
  for (auto &n : names) o.str(n);
  for (auto &t : types) o.str(t);
}

struct Table {
  int32_t rows = 0, cols = 0;
  bool has_schema = true;
  std::vector<std::pair<std::string, std::vector<std::string>>> dictionaries;  // column -> values by dictId
  std::vector<std::pair<std::string, std::string>> metadata;                  // insertion order
  Out schema, fixed, var;
};

// toBytes (DataTableImplV2.java:233-303) with the variable section written in place by write_var(dst) (var_size bytes):
// the header, dictionary map, metadata, schema and fixed section first, then the variable section, in one buffer.
template <typename W>
std::vector<uint8_t> table_bytes_var(const Table &t, size_t var_size, W &&write_var) {
  Out dict;  // serializeDictionaryMap (DataTableImplV2.java:305-328): HashMap<String, HashMap<Integer, String>>
  {
    std::vector<int32_t> h;
    for (auto &d : t.dictionaries) h.push_back(java_string_hash(d.first));
    dict.i32((int32_t)t.dictionaries.size());
    for (size_t i : java_hashmap_order(h)) {
      const auto &d = t.dictionaries[i];
      dict.str(d.first);
      dict.i32((int32_t)d.second.size());
      std::vector<int32_t> ih(d.second.size());
      for (size_t k = 0; k < ih.size(); k++) ih[k] = (int32_t)k;  // Integer.hashCode
      for (size_t k : java_hashmap_order(ih)) {
        dict.i32((int32_t)k);
        dict.str(d.second[k]);
      }
    }
  }
  Out meta;  // serializeMetadata (:330-347)
  {
    std::vector<int32_t> h;
    for (auto &kv : t.metadata) h.push_back(java_string_hash(kv.first));
    meta.i32((int32_t)t.metadata.size());
    for (size_t i : java_hashmap_order(h)) {
      meta.str(t.metadata[i].first);
      meta.str(t.metadata[i].second);
    }
  }
  const size_t schema_size = t.has_schema ? t.schema.b.size() : 0;
  const int32_t header = 13 * 4;
  const size_t total = header + dict.b.size() + meta.b.size() + schema_size + t.fixed.b.size() + var_size;
  require(total < (size_t)INT32_MAX, PINOT_ERR_UNSUPPORTED, "DataTable over 2 GB (int offsets)");
  std::vector<uint8_t> o(total);
  uint8_t *x = o.data();
  int32_t off = header;
  const int32_t head[13] = {2, t.rows, t.cols,
                            off, (int32_t)dict.b.size(),
                            off + (int32_t)dict.b.size(), (int32_t)meta.b.size(),
                            off + (int32_t)(dict.b.size() + meta.b.size()), (int32_t)schema_size,
                            off + (int32_t)(dict.b.size() + meta.b.size() + schema_size), (int32_t)t.fixed.b.size(),
                            off + (int32_t)(dict.b.size() + meta.b.size() + schema_size + t.fixed.b.size()),
                            (int32_t)var_size};
  for (int i = 0; i < 13; i++) x = put_be32(x, (uint32_t)head[i]);
  memcpy(x, dict.b.data(), dict.b.size());
  x += dict.b.size();
  memcpy(x, meta.b.data(), meta.b.size());
  x += meta.b.size();
  if (schema_size) memcpy(x, t.schema.b.data(), schema_size);
  x += schema_size;
  memcpy(x, t.fixed.b.data(), t.fixed.b.size());
  x += t.fixed.b.size();
  write_var(x);
  return o;
}

std::vector<uint8_t> table_bytes(const Table &t) {
  return table_bytes_var(t, t.var.b.size(), [&](uint8_t *x) { memcpy(x, t.var.b.data(), t.var.b.size()); });
}

// attachMetadataToDataTable (IntermediateResultsBlock.java:298-317) + the server's own keys
// (ServerQueryExecutorV1Impl.java:244-245) when the caller passes them.
void attach_metadata(Table &t, const pinot_exec_stats &s, bool groups_limit_reached, const pinot_datatable_server *srv) {
  t.metadata.emplace_back("numDocsScanned", std::to_string(s.num_docs_scanned));
  t.metadata.emplace_back("numEntriesScannedInFilter", std::to_string(s.num_entries_scanned_in_filter));
  t.metadata.emplace_back("numEntriesScannedPostFilter", std::to_string(s.num_entries_scanned_post_filter));
  t.metadata.emplace_back("numSegmentsProcessed", std::to_string(s.num_segments_processed));
  t.metadata.emplace_back("numSegmentsMatched", std::to_string(s.num_segments_matched));
  t.metadata.emplace_back("totalDocs", std::to_string(s.num_total_raw_docs));
  if (groups_limit_reached) t.metadata.emplace_back("numGroupsLimitReached", "true");
  if (srv) {
    t.metadata.emplace_back("numSegmentsQueried", std::to_string(srv->num_segments_queried));
    t.metadata.emplace_back("timeUsedMs", std::to_string(srv->time_used_ms));
    if (srv->request_id >= 0) t.metadata.emplace_back("requestId", std::to_string(srv->request_id));
  }
}

// DataTableBuilder.setColumn(int, Object) (:141-152): fixed cell = (variable offset, serialized length); variable
// data = int object type + serialized bytes.
template <typename F>
void object_cell(Table &t, int32_t type, F &&serialize) {
  Out v;
  serialize(v);
  t.fixed.i32((int32_t)t.var.b.size());
  t.fixed.i32((int32_t)v.b.size());
  t.var.i32(type);
  t.var.bytes(v.b.data(), v.b.size());
}

}  // namespace

std::vector<uint8_t> aggregation_datatable(const pinot_query &q, const pinot_agg_result *r, const pinot_exec_stats &s,
                                           const pinot_datatable_server *srv) {
  // getAggregationResultDataTable (:234-270): one row, one column per function (intermediate result types)
  Table t;
  t.rows = 1;
  t.cols = q.num_aggregations;
  std::vector<std::string> names, types;
  for (int i = 0; i < q.num_aggregations; i++) {
    names.push_back(aggregation_column_name(q.aggregations[i]));
    const int f = sv_function(q.aggregations[i].function);
    types.push_back(f == PINOT_AGG_COUNT ? "LONG" : (f == PINOT_AGG_AVG || f == PINOT_AGG_DISTINCTCOUNTHLL) ? "OBJECT" : "DOUBLE");
  }
  schema_bytes(t.schema, names, types);
  for (int i = 0; i < q.num_aggregations; i++) {
    const pinot_agg_result &a = r[i];
    switch (sv_function(q.aggregations[i].function)) {
      case PINOT_AGG_COUNT: t.fixed.i64(a.count); break;
      case PINOT_AGG_SUM:
      case PINOT_AGG_MIN:
      case PINOT_AGG_MAX: t.fixed.f64(a.value); break;
      case PINOT_AGG_AVG:  // AvgPair.toBytes (customobject/AvgPair.java:53-58): double sum, long count
        object_cell(t, OBJ_AVG_PAIR, [&](Out &v) { v.f64(a.value); v.i64(a.count); });
        break;
      default:
        object_cell(t, OBJ_HLL, [&](Out &v) { hll_bytes(v, a.hll_registers); });
        break;
    }
  }
  attach_metadata(t, s, false, srv);
  return table_bytes(t);
}

std::vector<uint8_t> group_by_datatable(const pinot_query &q, const GroupByResult &r, const int64_t *const *fn_groups,
                                        const int64_t *fn_num_groups, const pinot_exec_stats &s,
                                        const pinot_datatable_server *srv) {
  // getAggregationGroupByResultDataTable (:272-292): per function a row (functionName STRING via the column's
  // dictionary, GroupByResultMap OBJECT = Map<String group key, intermediate result>). The final buffer is laid out
  // once (every map entry's size from its key's length), then the entries are written in place by the host's task
  // pool in chunks of the concatenated entry lists.
  const int na = (int)r.functions.size();
  const int64_t n = (int64_t)r.raw_keys.size();
  static const bool phases = getenv("PINOT_DATATABLE_PHASES") != nullptr;  // diagnostic timing on stderr
  const auto t0 = std::chrono::steady_clock::now();
  Table t;
  t.rows = na;
  t.cols = 2;
  schema_bytes(t.schema, {"functionName", "GroupByResultMap"}, {"STRING", "OBJECT"});
  struct Fn {
    int64_t m = 0;           // entries of the map
    const int64_t *sel = nullptr;  // its groups (null: 0 .. m - 1)
    int f = 0;
    int32_t vtype = 0, vbytes = 0;
    const uint8_t *ser = nullptr, *regs = nullptr;  // HLL: getBytes rows / u8 register rows
    std::unique_ptr<PinnedBytes> stage;
    int64_t first = 0;       // index of its first entry in the concatenated list
  };
  std::vector<Fn> fns(na);
  int64_t total_entries = 0;
  for (int i = 0; i < na; i++) {
    Fn &F = fns[i];
    F.m = fn_groups && fn_groups[i] ? fn_num_groups[i] : n;
    F.sel = fn_groups && fn_groups[i] ? fn_groups[i] : nullptr;
    bool in_range = true;
    for (int64_t j = 0; F.sel && j < F.m; j++) in_range = in_range && F.sel[j] >= 0 && F.sel[j] < n;
    require(in_range, PINOT_ERR_BAD_ARG, "group index out of range");
    F.f = sv_function(r.functions[i]);
    F.vtype = F.f == PINOT_AGG_COUNT ? OBJ_LONG : F.f == PINOT_AGG_AVG ? OBJ_AVG_PAIR
              : F.f == PINOT_AGG_DISTINCTCOUNTHLL ? OBJ_HLL : OBJ_DOUBLE;
    F.vbytes = F.f == PINOT_AGG_AVG ? 16 : F.f == PINOT_AGG_DISTINCTCOUNTHLL ? 8 + 43 * 4 : 8;
    if (F.f == PINOT_AGG_DISTINCTCOUNTHLL && F.m) {
      // a device-trimmed result carries the getBytes rows (hll_serde.hip); else the registers: the host copy, or the
      // device parts through pinned staging (a large pageable copy target is pinned in place by the runtime, and its
      // later unmap stalls the GPU's queues)
      if ((size_t)i < r.hll_bytes.size() && r.hll_bytes[i].size() == (size_t)n * 180) {
        F.ser = r.hll_bytes[i].data();
      } else if (r.hll_parts.empty()) {
        F.regs = r.hll[i].data();
      } else {
        F.stage.reset(new PinnedBytes((size_t)n * 256));
        group_by_hll_registers(r, i, F.stage->data(), true);
        F.regs = F.stage->data();
      }
    }
    F.first = total_entries;
    total_entries += F.m;
  }
  const auto t1 = std::chrono::steady_clock::now();
  // entry sizes (MAP_SER_DE, ObjectSerDeUtils.java:262-300: key String = int length + bytes, value = int length +
  // bytes), in chunks over the pool
  const size_t nt = total_entries >= 4096 ? std::max<size_t>(1, std::min<size_t>(host_parallelism(), 16)) : 1;
  std::vector<uint32_t> esize((size_t)total_entries);
  auto fn_of = [&](int64_t e) {
    int i = 0;
    while (i + 1 < na && fns[i + 1].first <= e) i++;
    return i;
  };
  auto for_chunks = [&](const std::function<void(int64_t, int64_t)> &body) {
    if (nt == 1) {
      body(0, total_entries);
      return;
    }
    std::vector<std::exception_ptr> errs(nt);
    host_parallel(nt, [&](size_t c) {
      try {
        body(total_entries * (int64_t)c / (int64_t)nt, total_entries * (int64_t)(c + 1) / (int64_t)nt);
      } catch (...) {
        errs[c] = std::current_exception();
      }
    });
    for (auto &e : errs)
      if (e) std::rethrow_exception(e);
  };
  for_chunks([&](int64_t lo, int64_t hi) {
    const std::string *part[kMaxGroupCols];
    for (int64_t e = lo; e < hi;) {
      const int i = fn_of(e);
      const Fn &F = fns[i];
      const int64_t end = std::min(hi, F.first + F.m);
      for (; e < end; e++) {
        const int64_t j = e - F.first, g = F.sel ? F.sel[j] : j;
        esize[e] = (uint32_t)(8 + group_key_parts(r, g, part) + F.vbytes);
      }
    }
  });
  const auto t2 = std::chrono::steady_clock::now();
  // cell sizes and the variable section's layout: per row the object type, then the map (size, key and value types,
  // entries); the entries' offsets as one exclusive prefix sum
  std::vector<uint64_t> eoff((size_t)total_entries + 1);
  std::vector<int64_t> cell(na);
  size_t var = 0;
  for (int i = 0; i < na; i++) {
    const Fn &F = fns[i];
    var += 4;  // object type
    const size_t start = var;
    var += 4 + (F.m ? 8 : 0);
    for (int64_t j = 0; j < F.m; j++) {
      eoff[F.first + j] = var;
      var += esize[F.first + j];
    }
    cell[i] = (int64_t)(var - start);
  }
  std::vector<std::string> fn_names;
  size_t vpos = 0;
  for (int i = 0; i < na; i++) {
    const std::string name = aggregation_column_name(q.aggregations[i]);
    int32_t id = (int32_t)fn_names.size();
    for (size_t k = 0; k < fn_names.size(); k++)
      if (fn_names[k] == name) id = (int32_t)k;
    if (id == (int32_t)fn_names.size()) fn_names.push_back(name);
    t.fixed.i32(id);
    t.fixed.i32((int32_t)vpos);  // DataTableBuilder.setColumn(int, Object): (variable offset, serialized length)
    t.fixed.i32((int32_t)cell[i]);
    vpos += 4 + (size_t)cell[i];
  }
  t.dictionaries.emplace_back("functionName", fn_names);
  // CombineGroupByOperator.java:212-214: the merged map reached the inner-segment groups limit
  const int64_t merged = r.merged_groups >= 0 ? r.merged_groups : n;  // the device trim keeps fewer than it merged
  attach_metadata(t, s, merged >= (int64_t)q.num_groups_limit && q.num_groups_limit > 0, srv);
  auto bits = [](double d) {
    uint64_t u;
    memcpy(&u, &d, 8);
    return u;
  };
  const auto t3 = std::chrono::steady_clock::now();
  auto t4 = t3;
  std::vector<uint8_t> out = table_bytes_var(t, var, [&](uint8_t *v) {
    t4 = std::chrono::steady_clock::now();
    size_t at = 0;
    for (int i = 0; i < na; i++) {  // the rows' heads
      uint8_t *x = put_be32(v + at, (uint32_t)OBJ_MAP);
      x = put_be32(x, (uint32_t)fns[i].m);
      if (fns[i].m) put_be32(put_be32(x, (uint32_t)OBJ_STRING), (uint32_t)fns[i].vtype);
      at += 4 + (size_t)cell[i];
    }
    for_chunks([&](int64_t lo, int64_t hi) {
      const std::string *part[kMaxGroupCols];
      const size_t nc = r.gcard.size();
      for (int64_t e = lo; e < hi;) {
        const int i = fn_of(e);
        const Fn &F = fns[i];
        const HostVec<int64_t> &cnt = r.counts[r.counts_shared ? 0 : i];
        const HostVec<double> &val = r.values[i];
        const int64_t end = std::min(hi, F.first + F.m);
        for (; e < end; e++) {
          const int64_t j = e - F.first, g = F.sel ? F.sel[j] : j;
          // the key written straight from the columns' value strings (DictionaryBasedGroupKeyGenerator.java:421-437)
          const size_t klen = group_key_parts(r, g, part);
          uint8_t *x = put_be32(v + eoff[e], (uint32_t)klen);
          for (size_t c = 0; c < nc; c++) {
            if (c) *x++ = '\t';
            memcpy(x, part[c]->data(), part[c]->size());
            x += part[c]->size();
          }
          x = put_be32(x, (uint32_t)F.vbytes);
          switch (F.f) {
            case PINOT_AGG_COUNT: put_be64(x, (uint64_t)cnt[g]); break;
            case PINOT_AGG_AVG: put_be64(put_be64(x, bits(val[g])), (uint64_t)cnt[g]); break;
            case PINOT_AGG_DISTINCTCOUNTHLL:
              if (F.ser) memcpy(x, F.ser + (size_t)g * 180, 180);
              else hll_bytes_at(x, F.regs + (size_t)g * 256);
              break;
            default: put_be64(x, bits(val[g])); break;
          }
        }
      }
    });
  });
  if (phases) {
    const auto t5 = std::chrono::steady_clock::now();
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    fprintf(stderr, "[pinot_gpu] datatable phases (us): stage %.1f, sizes %.1f, layout+metadata %.1f, header+alloc %.1f, "
            "entries %.1f (%lld entries, %zu bytes)\n", us(t0, t1), us(t1, t2), us(t2, t3), us(t3, t4), us(t4, t5),
            (long long)total_entries, out.size());
  }
  return out;
}

std::vector<uint8_t> empty_datatable(const pinot_query &q, int64_t total_docs, const pinot_datatable_server *srv) {
  // processQuery with every segment pruned (ServerQueryExecutorV1Impl.java:187-196): buildEmptyDataTable then
  // totalDocs and zero statistics. The keys go in as totalDocs, numDocsScanned, ... there; none of them shares a
  // 16-slot HashMap bucket with another except numSegmentsProcessed / numSegmentsMatched, which keep their relative
  // order, so attach_metadata's order writes the same bytes.
  pinot_exec_stats s{};
  s.num_total_raw_docs = total_docs;
  if (q.num_group_by == 0) {
    // aggregation-only (:331-369): extractAggregationResult(createAggregationResultHolder()) per function
    std::vector<pinot_agg_result> r((size_t)q.num_aggregations);
    for (int i = 0; i < q.num_aggregations; i++) {
      memset(&r[i], 0, sizeof(r[i]));
      const int f = sv_function(q.aggregations[i].function);
      if (f == PINOT_AGG_MIN) r[i].value = INFINITY;    // MinAggregationFunction.java:32
      if (f == PINOT_AGG_MAX) r[i].value = -INFINITY;   // MaxAggregationFunction.java:32
    }
    return aggregation_datatable(q, r.data(), s, srv);
  }
  // group-by (:314-329): per function its column name and an empty HashMap
  Table t;
  t.rows = q.num_aggregations;
  t.cols = 2;
  schema_bytes(t.schema, {"functionName", "GroupByResultMap"}, {"STRING", "OBJECT"});
  std::vector<std::string> fn_names;
  for (int i = 0; i < q.num_aggregations; i++) {
    const std::string name = aggregation_column_name(q.aggregations[i]);
    int32_t id = (int32_t)fn_names.size();
    for (size_t k = 0; k < fn_names.size(); k++)
      if (fn_names[k] == name) id = (int32_t)k;
    if (id == (int32_t)fn_names.size()) fn_names.push_back(name);
    t.fixed.i32(id);
    object_cell(t, OBJ_MAP, [](Out &v) { v.i32(0); });
  }
  t.dictionaries.emplace_back("functionName", fn_names);
  attach_metadata(t, s, false, srv);
  return table_bytes(t);
}

}  // namespace pinot
