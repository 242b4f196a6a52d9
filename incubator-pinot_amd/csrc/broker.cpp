// Broker-side reduce of the servers' DataTables: BrokerReduceService.reduceOnDataTable
// (PC/query/reduce/BrokerReduceService.java:69-270) for aggregation-only (setAggregationResults :347-393) and
// group-by queries (setGroupByHavingResults :405-530 without HAVING), with the final top-N of
// AggregationGroupByTrimmingService.trimFinalResults (PC/query/aggregation/groupby/AggregationGroupByTrimmingService
// .java:123-149, ComparableSorter :190-250) and AggregationFunctionUtils.formatValue (PC/query/aggregation/function/
// AggregationFunctionUtils.java:113-128). PC = pinot-core/src/main/java/org/apache/pinot/core.
//
// Input: DataTableImplV2 bytes (PC/common/datatable/DataTableImplV2.java:104-171) as any server writes them;
// object cells per ObjectSerDeUtils (PC/common/ObjectSerDeUtils.java:144-330). Output: the BrokerResponseNative JSON
// (pinot-common/.../response/broker/BrokerResponseNative.java:42 property order).
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "engine.h"

namespace pinot {
namespace {

class In {
 public:
  In(const uint8_t *p, uint64_t n) : p_(p), n_(n) {}
  void seek(uint64_t off) {
    require(off <= n_, PINOT_ERR_BAD_ARG, "DataTable: offset out of range");
    i_ = off;
  }
  uint64_t pos() const { return i_; }
  const uint8_t *take(uint64_t k) {
    require(k <= n_ - i_, PINOT_ERR_BAD_ARG, "DataTable: truncated");
    const uint8_t *r = p_ + i_;
    i_ += k;
    return r;
  }
  int32_t i32() {
    const uint8_t *b = take(4);
    return (int32_t)(((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3]);
  }
  int64_t i64() {
    const uint64_t hi = (uint32_t)i32();
    return (int64_t)((hi << 32) | (uint32_t)i32());
  }
  double f64() {
    const int64_t v = i64();
    double d;
    memcpy(&d, &v, 8);
    return d;
  }
  std::string str() {
    const int32_t len = i32();
    require(len >= 0, PINOT_ERR_BAD_ARG, "DataTable: negative string length");
    const uint8_t *b = take((uint64_t)len);
    return std::string(reinterpret_cast<const char *>(b), (size_t)len);
  }

 private:
  const uint8_t *p_;
  uint64_t n_, i_ = 0;
};

enum ObjType : int32_t { OBJ_STRING = 0, OBJ_LONG = 1, OBJ_DOUBLE = 2, OBJ_AVG_PAIR = 4, OBJ_HLL = 6, OBJ_MAP = 8 };

// An intermediate result as the broker holds it (Long, Double, AvgPair, HyperLogLog).
struct Value {
  int type = OBJ_LONG;
  int64_t l = 0;
  double d = 0;
  uint8_t regs[256] = {};
};

Value read_object(int32_t type, In &in, uint64_t end) {
  Value v;
  v.type = type;
  switch (type) {
    case OBJ_LONG: v.l = in.i64(); break;
    case OBJ_DOUBLE: v.d = in.f64(); break;
    case OBJ_AVG_PAIR: v.d = in.f64(); v.l = in.i64(); break;  // AvgPair.fromBytes: double sum, long count
    case OBJ_HLL: {  // HyperLogLog.Builder.build(bytes): int log2m, int byte size, RegisterSet words
      const int32_t log2m = in.i32(), size = in.i32();
      require(log2m == 8 && size == 43 * 4, PINOT_ERR_UNSUPPORTED, "DataTable: HyperLogLog other than log2m 8");
      uint32_t w[43];
      for (int k = 0; k < 43; k++) w[k] = (uint32_t)in.i32();
      for (int p = 0; p < 256; p++) v.regs[p] = (uint8_t)((w[p / 6] >> (5 * (p % 6))) & 0x1F);
      break;
    }
    default: throw Error(PINOT_ERR_UNSUPPORTED, "DataTable: object type " + std::to_string(type));
  }
  require(in.pos() <= end, PINOT_ERR_BAD_ARG, "DataTable: object overruns its cell");
  return v;
}

struct Table {
  int32_t rows = 0, cols = 0;
  bool has_schema = false;
  std::vector<std::pair<std::string, std::string>> metadata;
  std::vector<std::string> names, types;
  std::unordered_map<std::string, std::unordered_map<int32_t, std::string>> dictionaries;
  const uint8_t *base = nullptr;
  uint64_t len = 0, fixed = 0, var = 0, var_len = 0;
  std::vector<int32_t> col_off;
  int32_t row_size = 0;
};

int32_t column_size(const std::string &t) {  // DataTableBuilder column sizes (DataTableBuilder.java:90-120)
  if (t == "INT" || t == "FLOAT" || t == "STRING") return 4;
  return 8;  // LONG, DOUBLE, OBJECT (int offset + int length)
}

Table parse_table(const uint8_t *b, uint64_t n) {
  Table t;
  t.base = b;
  t.len = n;
  In in(b, n);
  require(in.i32() == 2, PINOT_ERR_UNSUPPORTED, "DataTable: version other than 2");
  t.rows = in.i32();
  t.cols = in.i32();
  require(t.rows >= 0 && t.cols >= 0, PINOT_ERR_BAD_ARG, "DataTable: negative shape");
  int32_t start[5], length[5];
  for (int s = 0; s < 5; s++) {
    start[s] = in.i32();
    length[s] = in.i32();
    require(start[s] >= 0 && length[s] >= 0 && (uint64_t)start[s] + (uint64_t)length[s] <= n, PINOT_ERR_BAD_ARG,
            "DataTable: section out of range");
  }
  if (length[0] > 0) {  // dictionary map
    In d(b, (uint64_t)start[0] + length[0]);
    d.seek(start[0]);
    const int32_t nd = d.i32();
    for (int32_t i = 0; i < nd; i++) {
      const std::string col = d.str();
      const int32_t ne = d.i32();
      auto &m = t.dictionaries[col];
      for (int32_t k = 0; k < ne; k++) {
        const int32_t id = d.i32();
        m[id] = d.str();
      }
    }
  }
  {  // metadata
    In m(b, (uint64_t)start[1] + length[1]);
    m.seek(start[1]);
    if (length[1] > 0) {
      const int32_t nm = m.i32();
      for (int32_t i = 0; i < nm; i++) {
        std::string k = m.str();
        t.metadata.emplace_back(std::move(k), m.str());
      }
    }
  }
  if (length[2] > 0) {  // DataSchema.fromBytes
    In s(b, (uint64_t)start[2] + length[2]);
    s.seek(start[2]);
    const int32_t nc = s.i32();
    for (int32_t i = 0; i < nc; i++) t.names.push_back(s.str());
    for (int32_t i = 0; i < nc; i++) t.types.push_back(s.str());
    t.has_schema = true;
    require(nc == t.cols, PINOT_ERR_BAD_ARG, "DataTable: schema / column count mismatch");
    for (auto &ty : t.types) {
      t.col_off.push_back(t.row_size);
      t.row_size += column_size(ty);
    }
    require((uint64_t)t.rows * (uint64_t)t.row_size <= (uint64_t)length[3], PINOT_ERR_BAD_ARG,
            "DataTable: fixed-size section too short");
  }
  t.fixed = (uint64_t)start[3];
  t.var = (uint64_t)start[4];
  t.var_len = (uint64_t)length[4];
  return t;
}

In cell(const Table &t, int32_t row, int32_t col) {
  require(t.has_schema && row >= 0 && row < t.rows && col >= 0 && col < t.cols, PINOT_ERR_BAD_ARG, "DataTable: cell");
  In in(t.base, t.len);
  in.seek(t.fixed + (uint64_t)row * t.row_size + t.col_off[col]);
  return in;
}

Value get_object(const Table &t, int32_t row, int32_t col, std::vector<std::pair<std::string, Value>> *map_out) {
  In c = cell(t, row, col);
  const int32_t off = c.i32(), size = c.i32();
  // variable section: int object type, then `size` serialized bytes (DataTableBuilder.setColumn(Object))
  require(off >= 0 && size >= 0 && (uint64_t)off + 4 + (uint64_t)size <= t.var_len, PINOT_ERR_BAD_ARG,
          "DataTable: object cell out of range");
  const uint64_t end = t.var + (uint64_t)off + 4 + (uint64_t)size;
  In in(t.base, end);
  in.seek(t.var + off);
  const int32_t type = in.i32();
  if (type != OBJ_MAP) return read_object(type, in, end);
  require(map_out != nullptr, PINOT_ERR_BAD_ARG, "DataTable: unexpected map cell");
  const int32_t n = in.i32();  // MAP_SER_DE (ObjectSerDeUtils.java:262-300)
  if (n == 0) return Value{};
  const int32_t kt = in.i32(), vt = in.i32();
  require(kt == OBJ_STRING, PINOT_ERR_UNSUPPORTED, "DataTable: group map keys other than String");
  for (int32_t i = 0; i < n; i++) {
    const std::string key = in.str();
    const int32_t vl = in.i32();
    require(vl >= 0, PINOT_ERR_BAD_ARG, "DataTable: negative value length");
    const uint64_t vend = in.pos() + (uint64_t)vl;
    map_out->emplace_back(key, read_object(vt, in, vend));
    in.seek(vend);
  }
  return Value{};
}

int fn_of(const pinot_query &q, int i) { return sv_function(q.aggregations[i].function); }

// AggregationFunction.merge for each function (CountAggregationFunction.merge :…, Math.min / Math.max on doubles,
// AvgPair.apply, HyperLogLog.addAll).
void merge_into(int f, Value &a, const Value &b) {
  switch (f) {
    case PINOT_AGG_COUNT: a.l = (int64_t)((uint64_t)a.l + (uint64_t)b.l); break;  // Java long arithmetic wraps
    case PINOT_AGG_SUM: a.d += b.d; break;
    case PINOT_AGG_MIN: a.d = (std::isnan(a.d) || std::isnan(b.d)) ? NAN : (a.d < b.d || (a.d == b.d && std::signbit(a.d))) ? a.d : b.d; break;
    case PINOT_AGG_MAX: a.d = (std::isnan(a.d) || std::isnan(b.d)) ? NAN : (a.d > b.d || (a.d == b.d && !std::signbit(a.d))) ? a.d : b.d; break;
    case PINOT_AGG_AVG: a.d += b.d; a.l = (int64_t)((uint64_t)a.l + (uint64_t)b.l); break;
    default:
      for (int p = 0; p < 256; p++) a.regs[p] = std::max(a.regs[p], b.regs[p]);
      break;
  }
}

// A final result (extractFinalResult): Long for COUNT / DISTINCTCOUNTHLL, Double otherwise.
struct Final {
  bool is_long = false;
  int64_t l = 0;
  double d = 0;
};

Final final_result(int f, const Value &v) {
  Final r;
  switch (f) {
    case PINOT_AGG_COUNT: r.is_long = true; r.l = v.l; break;
    case PINOT_AGG_AVG: r.d = v.l == 0 ? -INFINITY : v.d / (double)v.l; break;  // AvgAggregationFunction.java:222-230
    case PINOT_AGG_DISTINCTCOUNTHLL: r.is_long = true; r.l = hll_cardinality(v.regs); break;
    default: r.d = v.d; break;
  }
  return r;
}

int java_compare_final(const Final &a, const Final &b) {  // Long.compareTo / Double.compareTo
  if (a.is_long) return a.l < b.l ? -1 : a.l > b.l ? 1 : 0;
  if (a.d < b.d) return -1;
  if (a.d > b.d) return 1;
  const bool an = std::isnan(a.d), bn = std::isnan(b.d);
  if (an || bn) return an == bn ? 0 : (an ? 1 : -1);
  const bool as = std::signbit(a.d), bs = std::signbit(b.d);
  return as == bs ? 0 : (as ? -1 : 1);
}

// The shortest decimal digits that read back as v (what FloatingDecimal feeds Formatter), as digits + exponent:
// v = 0.d1d2d3... x 10^exp.
void shortest_digits(double v, std::string &digits, int &exp10) {
  char buf[64];
  for (int prec = 1; prec <= 17; prec++) {
    snprintf(buf, sizeof buf, "%.*e", prec - 1, v);
    if (strtod(buf, nullptr) == v) break;
  }
  digits.clear();
  const char *p = buf;
  for (; *p && *p != 'e'; p++)
    if (*p >= '0' && *p <= '9') digits.push_back(*p);
  const int e = atoi(p + 1);
  exp10 = e + 1;
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
}

// String.format(Locale.US, "%1.5f", v): FormattedFloatingDecimal's digits rounded half-up at 5 decimals.
std::string java_format_5f(double v) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) return v > 0 ? "Infinity" : "-Infinity";
  const bool neg = std::signbit(v);
  std::string digits;
  int e;
  if (v == 0) {
    digits = "0";
    e = 1;
  } else {
    shortest_digits(std::fabs(v), digits, e);
  }
  // integer part: digits[0, e); fraction: digits[e, ...) (zero-padded)
  std::string intpart, frac;
  for (int i = 0; i < e; i++) intpart.push_back(i < (int)digits.size() ? digits[i] : '0');
  if (intpart.empty()) intpart = "0";
  for (int i = e; i < e + 6; i++) frac.push_back(i >= 0 && i < (int)digits.size() ? digits[i] : '0');
  bool round_up = frac[5] >= '5';
  frac.resize(5);
  if (round_up) {
    std::string all = intpart + frac;
    int i = (int)all.size() - 1;
    while (i >= 0 && all[i] == '9') all[i--] = '0';
    if (i < 0) all.insert(all.begin(), '1');
    else all[i]++;
    intpart = all.substr(0, all.size() - 5);
    frac = all.substr(all.size() - 5);
  }
  size_t nz = intpart.find_first_not_of('0');
  intpart = nz == std::string::npos ? "0" : intpart.substr(nz);
  return (neg ? "-" : "") + intpart + "." + frac;  // the sign stays on a value that rounds to zero ("-0.00000")
}

// AggregationFunctionUtils.formatValue (:113-128).
std::string format_value(const Final &r) {
  if (r.is_long) return std::to_string(r.l);
  const double d = r.d;
  // DoubleMath.isMathematicalInteger and d <= Long.MAX_VALUE (a double compare: 2^63 passes): Long.toString((long) d)
  if (std::isfinite(d) && d == std::floor(d) && d <= 9223372036854775807.0) {
    const int64_t l = d >= 9223372036854775807.0 ? INT64_MAX : d < -9223372036854775808.0 ? INT64_MIN : (int64_t)d;
    return std::to_string(l) + ".00000";
  }
  return java_format_5f(d);
}

void json_str(std::string &o, const std::string &s) {
  o.push_back('"');
  for (unsigned char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      case '\b': o += "\\b"; break;
      case '\f': o += "\\f"; break;
      default:
        if (c < 0x20) {
          char u[8];
          snprintf(u, sizeof u, "\\u%04x", c);
          o += u;
        } else {
          o.push_back((char)c);
        }
    }
  }
  o.push_back('"');
}

const std::string *meta(const Table &t, const char *key) {
  for (auto &kv : t.metadata)
    if (kv.first == key) return &kv.second;
  return nullptr;
}

}  // namespace

std::string broker_reduce(const pinot_query &q, int32_t n, const uint8_t *const *tables, const uint64_t *lens,
                          int32_t top_n) {
  const int na = q.num_aggregations;
  std::vector<Table> ts;
  for (int32_t i = 0; i < n; i++) {
    require(tables[i] != nullptr, PINOT_ERR_BAD_ARG, "null DataTable");
    ts.push_back(parse_table(tables[i], lens[i]));
  }
  // execution statistics and exceptions from every table's metadata (:94-176)
  int64_t docs = 0, in_filter = 0, post_filter = 0, queried = 0, processed = 0, matched = 0, total = 0;
  bool limit = false;
  std::string exceptions;
  auto parse_long = [](const std::string &s) -> int64_t {  // Long.parseLong
    try {
      // Long.parseLong takes an optional sign then digits only (std::stoll would skip leading whitespace)
      require(!s.empty() && (s[0] == '-' || s[0] == '+' || (s[0] >= '0' && s[0] <= '9')), PINOT_ERR_BAD_ARG,
              "DataTable: metadata value is not a long: " + s);
      size_t used = 0;
      const long long v = std::stoll(s, &used);
      require(used == s.size(), PINOT_ERR_BAD_ARG, "DataTable: metadata value is not a long: " + s);
      return (int64_t)v;
    } catch (const std::logic_error &) {
      throw Error(PINOT_ERR_BAD_ARG, "DataTable: metadata value is not a long: " + s);
    }
  };
  auto add = [&](int64_t &acc, const std::string *s) {
    if (s) acc = (int64_t)((uint64_t)acc + (uint64_t)parse_long(*s));
  };
  std::vector<const Table *> with_rows;
  for (const Table &t : ts) {
    for (auto &kv : t.metadata) {
      if (kv.first.rfind("Exception", 0) == 0) {  // DataTable.EXCEPTION_METADATA_KEY + error code
        if (!exceptions.empty()) exceptions += ",";
        exceptions += "{\"errorCode\":" + std::to_string((int32_t)parse_long(kv.first.substr(9))) + ",\"message\":";
        json_str(exceptions, kv.second);
        exceptions += "}";
      }
    }
    add(docs, meta(t, "numDocsScanned"));
    add(in_filter, meta(t, "numEntriesScannedInFilter"));
    add(post_filter, meta(t, "numEntriesScannedPostFilter"));
    add(queried, meta(t, "numSegmentsQueried"));
    add(processed, meta(t, "numSegmentsProcessed"));
    add(matched, meta(t, "numSegmentsMatched"));
    add(total, meta(t, "totalDocs"));
    const std::string *gl = meta(t, "numGroupsLimitReached");
    limit |= gl && gl->size() == 4 && std::equal(gl->begin(), gl->end(), "true", [](char a, char b) {
               return std::tolower((unsigned char)a) == b;
             });  // Boolean.valueOf: "true", ignoring case
    if (t.has_schema && t.rows > 0) with_rows.push_back(&t);
  }
  std::string results;
  if (!with_rows.empty() && q.num_group_by == 0) {
    // setAggregationResults (:347-393): merge row 0 of every table, extract, format
    std::vector<Value> acc(na);
    std::vector<bool> have(na, false);
    const Table &schema = *with_rows.back();
    for (const Table *t : with_rows) {
      require(t->cols == na, PINOT_ERR_BAD_ARG, "DataTable: column count differs from the query's aggregations");
      for (int i = 0; i < na; i++) {
        Value v;
        const std::string &ty = t->types[i];
        if (ty == "LONG") { In c = cell(*t, 0, i); v.type = OBJ_LONG; v.l = c.i64(); }
        else if (ty == "DOUBLE") { In c = cell(*t, 0, i); v.type = OBJ_DOUBLE; v.d = c.f64(); }
        else if (ty == "OBJECT") v = get_object(*t, 0, i, nullptr);
        else throw Error(PINOT_ERR_BAD_ARG, "Illegal column data type in aggregation results: " + ty);
        if (!have[i]) acc[i] = v, have[i] = true;
        else merge_into(fn_of(q, i), acc[i], v);
      }
    }
    for (int i = 0; i < na; i++) {
      if (i) results += ",";
      results += "{\"function\":";
      json_str(results, schema.names[i]);
      results += ",\"value\":";
      json_str(results, format_value(final_result(fn_of(q, i), acc[i])));
      results += "}";
    }
  } else if (!with_rows.empty()) {
    // setGroupByHavingResults (:405-530): per function, merge the maps by key, extract, keep the top N
    std::vector<std::string> names(na);
    std::string gcols = "[";
    for (int g = 0; g < q.num_group_by; g++) {
      if (g) gcols += ",";
      json_str(gcols, q.group_by[g]);
    }
    gcols += "]";
    for (int i = 0; i < na; i++) {
      std::map<std::string, Value> merged;  // ordered: ties below broken by key (the reference's heap order is
                                            // the arbitrary HashMap order)
      for (const Table *t : with_rows) {
        require(t->rows == na && t->cols == 2, PINOT_ERR_BAD_ARG, "DataTable: group-by table shape");
        if (names[i].empty()) {
          In c = cell(*t, i, 0);
          const int32_t id = c.i32();
          auto dit = t->dictionaries.find(t->names[0]);
          require(dit != t->dictionaries.end() && dit->second.count(id), PINOT_ERR_BAD_ARG,
                  "DataTable: functionName not in the dictionary");
          names[i] = dit->second.at(id);
        }
        std::vector<std::pair<std::string, Value>> entries;
        get_object(*t, i, 1, &entries);
        for (auto &kv : entries) {
          auto it = merged.find(kv.first);
          if (it == merged.end()) merged.emplace(kv.first, kv.second);
          else merge_into(fn_of(q, i), it->second, kv.second);
        }
      }
      // trimFinalResults: MIN ascending, every other function descending; top_n of them
      std::vector<std::pair<const std::string *, Final>> fin;
      fin.reserve(merged.size());
      for (auto &kv : merged) fin.emplace_back(&kv.first, final_result(fn_of(q, i), kv.second));
      const bool asc = fn_of(q, i) == PINOT_AGG_MIN;
      auto better = [&](const std::pair<const std::string *, Final> &a, const std::pair<const std::string *, Final> &b) {
        const int c = java_compare_final(a.second, b.second);
        if (c != 0) return asc ? c < 0 : c > 0;
        return *a.first < *b.first;
      };
      const size_t keep = std::min(fin.size(), (size_t)std::max(top_n, 0));
      std::partial_sort(fin.begin(), fin.begin() + keep, fin.end(), better);
      if (i) results += ",";
      results += "{\"groupByResult\":[";
      for (size_t k = 0; k < keep; k++) {
        if (k) results += ",";
        results += "{\"value\":";
        json_str(results, format_value(fin[k].second));
        results += ",\"group\":[";
        const std::string &key = *fin[k].first;  // split("\t", -1): trailing empty keys kept
        size_t s = 0;
        for (bool first = true;; first = false) {
          const size_t p = key.find('\t', s);
          if (!first) results += ",";
          json_str(results, key.substr(s, p == std::string::npos ? std::string::npos : p - s));
          if (p == std::string::npos) break;
          s = p + 1;
        }
        results += "]}";
      }
      results += "],\"function\":";
      json_str(results, names[i]);
      results += ",\"groupByColumns\":" + gcols + "}";
    }
  }
  std::string o = "{\"aggregationResults\":[" + results + "],\"exceptions\":[" + exceptions + "]";
  o += ",\"numServersQueried\":" + std::to_string(n) + ",\"numServersResponded\":" + std::to_string(n);
  o += ",\"numSegmentsQueried\":" + std::to_string(queried) + ",\"numSegmentsProcessed\":" + std::to_string(processed);
  o += ",\"numSegmentsMatched\":" + std::to_string(matched) + ",\"numConsumingSegmentsQueried\":0";
  o += ",\"numDocsScanned\":" + std::to_string(docs) + ",\"numEntriesScannedInFilter\":" + std::to_string(in_filter);
  o += ",\"numEntriesScannedPostFilter\":" + std::to_string(post_filter);
  o += std::string(",\"numGroupsLimitReached\":") + (limit ? "true" : "false");
  o += ",\"totalDocs\":" + std::to_string(total) + ",\"timeUsedMs\":0,\"segmentStatistics\":[],\"traceInfo\":{}}";
  return o;
}

std::string java_format_value_double(double d) { return format_value(Final{false, 0, d}); }

}  // namespace pinot
