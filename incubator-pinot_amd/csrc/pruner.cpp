// Segment pruning, the step ServerQueryExecutorV1Impl.processQuery runs before planning
// (PC/query/executor/ServerQueryExecutorV1Impl.java:183-216 and pruneSegments :270-294). PC = pinot-core/src/main/
// java/org/apache/pinot/core. SegmentPrunerService.prune (PC/query/pruner/SegmentPrunerService.java:52-60) asks each
// configured pruner in turn and drops the segment at the first "true"; the server's default list
// (pinot-server/.../DefaultHelixStarterServerConfig.java:60-65) is restated here in that order:
//   DataSchemaSegmentPruner   (PC/query/pruner/DataSchemaSegmentPruner.java:38-41): a query column the segment lacks
//   ColumnValueSegmentPruner  (PC/query/pruner/ColumnValueSegmentPruner.java:49-200, AbstractSegmentPruner.java:56-105):
//                             EQUALITY / RANGE leaves against the column's min / max value, and an EQUALITY value the
//                             column's bloom filter rules out (:140-144); AND prunes when any child does, OR when every
//                             child does; other leaves never prune
//   ValidSegmentPruner        (PC/query/pruner/ValidSegmentPruner.java:47-58): an empty segment
//   PartitionSegmentPruner    (PC/query/pruner/PartitionSegmentPruner.java:73-111): an EQUALITY value whose partition
//                             (the column's partition function) the segment does not hold
//
// Min / max: the column metadata's minValue / maxValue strings (ColumnMetadata.java:155-156), parsed with the
// column's type; absent (the creator does not write them; the loader's ColumnMinMaxValueGenerator adds them only
// for the time column in its default TIME mode) means the column never prunes by range.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>

#include "engine.h"

namespace pinot {
namespace {

// A column's type, value range, bloom filter and partition metadata, as ColumnMetadata / the data source expose them
// to the pruners.
struct ColumnRange {
  int data_type = PINOT_INT;
  bool has_range = false;  // minValue / maxValue present (a non-empty dictionary)
  int64_t imin = 0, imax = 0;
  double dmin = 0, dmax = 0;
  std::string smin, smax;
  const BloomFilter *bloom = nullptr;           // null / empty: no bloom filter
  int partition_fn = PF_NONE;
  int32_t num_partitions = 0;
  const std::vector<int32_t> *partitions = nullptr;
};

// A literal of the column's type (AbstractSegmentPruner.getValue -> FieldSpec.DataType.convert; a bad literal is a
// BadQueryRequestException).
struct Literal {
  int64_t i = 0;
  double d = 0;
  std::string s;
};

Literal convert(const ColumnRange &c, const std::string &raw) {
  Literal v;
  switch (c.data_type) {
    case PINOT_INT: v.i = java_parse_integer(raw, INT32_MIN, INT32_MAX); break;
    case PINOT_LONG: v.i = java_parse_integer(raw, INT64_MIN, INT64_MAX); break;
    case PINOT_FLOAT: v.d = java_parse_double(raw, true); break;  // Float.valueOf
    case PINOT_DOUBLE: v.d = java_parse_double(raw); break;
    default: v.s = raw; break;
  }
  return v;
}

// Double.compare / Float.compare: NaN above everything (and equal to itself), -0.0 below 0.0.
int java_double_compare(double a, double b) {
  if (a < b) return -1;
  if (a > b) return 1;
  const bool an = std::isnan(a), bn = std::isnan(b);
  if (an || bn) return an == bn ? 0 : (an ? 1 : -1);
  const bool as = std::signbit(a), bs = std::signbit(b);
  return as == bs ? 0 : (as ? -1 : 1);
}

// Comparable.compareTo on the column's type. STRING: byte order of the UTF-8 values, which is String.compareTo's
// order except between supplementary characters and U+E000..U+FFFF (the planner's dictionary search has the same
// convention).
int compare(const ColumnRange &c, const Literal &a, const Literal &b) {
  switch (c.data_type) {
    case PINOT_INT:
    case PINOT_LONG: return a.i < b.i ? -1 : a.i > b.i ? 1 : 0;
    case PINOT_FLOAT:
    case PINOT_DOUBLE: return java_double_compare(a.d, b.d);
    default: {
      const int r = a.s.compare(b.s);
      return r < 0 ? -1 : r > 0 ? 1 : 0;
    }
  }
}

// ColumnMetadata's typed minValue / maxValue (Integer / Long / Float / Double.valueOf, or the string).
void set_range(ColumnRange &c, const std::string &name, const std::string &mn, const std::string &mx) {
  try {
    const Literal a = convert(c, mn), b = convert(c, mx);
    c.imin = a.i, c.imax = b.i, c.dmin = a.d, c.dmax = b.d, c.smin = a.s, c.smax = b.s;
  } catch (const Error &) {
    throw Error(PINOT_ERR_BAD_ARG, name + ": minValue / maxValue do not parse as the column's type");
  }
  c.has_range = true;
}

Literal range_min(const ColumnRange &c) { return Literal{c.imin, c.dmin, c.smin}; }
Literal range_max(const ColumnRange &c) { return Literal{c.imax, c.dmax, c.smax}; }

// The typed value's toString (Integer / Long / Float / Double.toString, or the string): what mightContain hashes
// (BloomFilterReader.mightContain -> key.toString()) and the Murmur / ByteArray partition functions read.
std::string java_to_string(const ColumnRange &c, const Literal &v) {
  switch (c.data_type) {
    case PINOT_INT:
    case PINOT_LONG: return std::to_string(v.i);
    case PINOT_FLOAT: return java_float_to_string((float)v.d);
    case PINOT_DOUBLE: return java_double_to_string(v.d);
    default: return v.s;
  }
}

// pruneNonLeaf (AbstractSegmentPruner.java:56-90): AND prunes when any child does, OR when every child does.
template <typename Leaf>
bool prune_nonleaf(const FilterTreeInput &t, const Leaf &leaf) {
  if (t.op == PINOT_FILTER_AND || t.op == PINOT_FILTER_OR) {
    if (t.children.empty()) return false;
    if (t.op == PINOT_FILTER_AND) {
      for (const auto &c : t.children)
        if (prune_nonleaf(c, leaf)) return true;
      return false;
    }
    for (const auto &c : t.children)
      if (!prune_nonleaf(c, leaf)) return false;
    return true;
  }
  return leaf(t);
}

// PartitionSegmentPruner.pruneSegment's leaf (:85-110): EQUALITY only; a column without partition metadata never prunes.
template <typename Lookup>
bool prune_partition_leaf(const FilterTreeInput &t, const Lookup &lookup) {
  if (t.op != PINOT_FILTER_EQUALITY) return false;
  ColumnRange c;
  if (!lookup(t.column, c)) return true;  // "should have already been pruned in DataSchemaSegmentPruner"
  if (c.partition_fn == PF_NONE) return false;
  require(!t.values.empty(), PINOT_ERR_BAD_QUERY, "predicate on " + t.column + " has no value");
  const Literal v = convert(c, t.values[0]);
  TypedValue tv;
  tv.data_type = c.data_type;
  tv.i = v.i;
  tv.d = c.data_type == PINOT_FLOAT ? (double)(float)v.d : v.d;
  tv.s = java_to_string(c, v);
  const int32_t p = partition_of((PartitionFunctionKind)c.partition_fn, c.num_partitions, tv);
  return !std::binary_search(c.partitions->begin(), c.partitions->end(), p);
}

// ColumnValueSegmentPruner.pruneSegment's leaf (:108-200).
template <typename Lookup>
bool prune_column_value_leaf(const FilterTreeInput &t, const Lookup &lookup) {
  if (t.op != PINOT_FILTER_EQUALITY && t.op != PINOT_FILTER_RANGE) return false;
  ColumnRange c;
  if (!lookup(t.column, c)) return true;  // "Should not reach here after DataSchemaSegmentPruner"
  require(!t.values.empty(), PINOT_ERR_BAD_QUERY, "predicate on " + t.column + " has no value");
  if (t.op == PINOT_FILTER_EQUALITY) {
    const Literal v = convert(c, t.values[0]);
    bool prune = c.has_range && (compare(c, v, range_min(c)) < 0 || compare(c, v, range_max(c)) > 0);
    if (!prune && c.bloom && !c.bloom->empty()) prune = !c.bloom->might_contain(java_to_string(c, v));
    return prune;
  }
  const RangeBounds rb = parse_range(t.values[0]);
  const bool has_lo = rb.lower != "*", has_hi = rb.upper != "*";
  Literal lo, hi;
  if (has_lo) lo = convert(c, rb.lower);
  if (has_hi) hi = convert(c, rb.upper);
  if (has_lo && has_hi) {  // an empty range prunes whatever the segment holds
    const int r = compare(c, lo, hi);
    if (rb.inc_lower && rb.inc_upper ? r > 0 : r >= 0) return true;
  }
  if (!c.has_range) return false;
  if (has_lo) {
    const int r = compare(c, lo, range_max(c));
    if (rb.inc_lower ? r > 0 : r >= 0) return true;
  }
  if (has_hi) {
    const int r = compare(c, hi, range_min(c));
    if (rb.inc_upper ? r < 0 : r <= 0) return true;
  }
  return false;
}

void filter_columns(const FilterTreeInput &t, std::vector<std::string> &out) {
  if (t.op == PINOT_FILTER_AND || t.op == PINOT_FILTER_OR) {
    for (const auto &c : t.children) filter_columns(c, out);
  } else {
    out.push_back(t.column);
  }
}

// ServerQueryRequest.getAllColumns (PC/query/request/ServerQueryRequest.java:81-133): filter columns, the columns
// of every aggregation except COUNT, group-by columns.
std::vector<std::string> query_columns(const pinot_query &q, const FilterTreeInput *tree) {
  std::vector<std::string> cols;
  if (tree) filter_columns(*tree, cols);
  for (int i = 0; i < q.num_aggregations; i++)
    if (q.aggregations[i].function != PINOT_AGG_COUNT && q.aggregations[i].column)
      cols.emplace_back(q.aggregations[i].column);
  for (int i = 0; i < q.num_group_by; i++)
    if (q.group_by[i]) cols.emplace_back(q.group_by[i]);
  return cols;
}

template <typename Has, typename Lookup>
bool prune_with(int32_t num_docs, const pinot_query &q, const FilterTreeInput *tree, int32_t mask, const Has &has,
                const Lookup &lookup) {
  if (mask & PINOT_PRUNER_DATA_SCHEMA)
    for (const auto &c : query_columns(q, tree))
      if (!has(c)) return true;
  if ((mask & PINOT_PRUNER_COLUMN_VALUE) && tree &&
      prune_nonleaf(*tree, [&](const FilterTreeInput &t) { return prune_column_value_leaf(t, lookup); }))
    return true;
  if ((mask & PINOT_PRUNER_VALID) && num_docs == 0) return true;
  if ((mask & PINOT_PRUNER_PARTITION) && tree &&
      prune_nonleaf(*tree, [&](const FilterTreeInput &t) { return prune_partition_leaf(t, lookup); }))
    return true;
  return false;
}

}  // namespace

bool prune_segment(const SegmentData &s, const pinot_query &q, const FilterTreeInput *tree, int32_t mask) {
  auto has = [&](const std::string &name) {
    if (s.by_name.count(name)) return true;
    for (const auto &u : s.unserved)
      require(u != name, PINOT_ERR_UNSUPPORTED, "column " + name + " is multi-value / raw / BYTES: not served");
    return false;
  };
  auto lookup = [&](const std::string &name, ColumnRange &c) {
    auto it = s.by_name.find(name);
    if (it == s.by_name.end()) return false;
    const ColumnData &cd = *s.cols[it->second];
    c.data_type = cd.data_type;
    if (cd.has_minmax) set_range(c, name, cd.min_value, cd.max_value);
    c.bloom = &cd.bloom;
    c.partition_fn = cd.partition_fn;
    c.num_partitions = cd.num_partitions;
    c.partitions = &cd.partitions;
    return true;
  };
  return prune_with(s.num_docs, q, tree, mask, has, lookup);
}

bool prune_segment_desc(const pinot_segment_desc &d, const pinot_query &q, const FilterTreeInput *tree, int32_t mask) {
  require(d.num_columns >= 0 && (d.num_columns == 0 || d.columns != nullptr), PINOT_ERR_BAD_ARG, "segment columns");
  auto find = [&](const std::string &name) -> const pinot_column_desc * {
    for (int32_t i = 0; i < d.num_columns; i++)
      if (d.columns[i].name && name == d.columns[i].name) return &d.columns[i];
    return nullptr;
  };
  auto has = [&](const std::string &name) { return find(name) != nullptr; };
  // bloom filters (parsed, or built from the decoded dictionary) and partition metadata of the descriptor's columns
  std::map<std::string, ColumnData> meta;
  auto lookup = [&](const std::string &name, ColumnRange &c) {
    const pinot_column_desc *cd = find(name);
    if (!cd) return false;
    require(cd->data_type >= PINOT_INT && cd->data_type <= PINOT_STRING, PINOT_ERR_BAD_ARG, name + ": data type");
    c.data_type = cd->data_type;
    require((cd->min_value == nullptr) == (cd->max_value == nullptr), PINOT_ERR_BAD_ARG,
            name + ": minValue without maxValue (or the reverse)");
    if (cd->min_value) set_range(c, name, cd->min_value, cd->max_value);
    if (cd->bloom_filter || cd->create_bloom_filter || cd->partition_function) {
      auto it = meta.find(name);
      if (it == meta.end()) {
        ColumnData &m = meta[name];
        if (cd->create_bloom_filter || cd->num_partition_values == -1) {  // built from the decoded dictionary
          // a dictionary column decodes its dictionary only; a raw column needs its values sorted into one (the
          // transcode registration does: O(N log N) per call, not cached — register the segment to pay it once)
          TranscodedColumn tc;
          if (transcode_raw(*cd, d.num_docs, tc)) parse_dictionary_only(m, tc.desc);
          else parse_dictionary_only(m, *cd);
        } else {
          m.name = name;
          m.data_type = cd->data_type;
          parse_pruning_metadata(m, *cd);
        }
        it = meta.find(name);
      }
      c.bloom = &it->second.bloom;
      c.partition_fn = it->second.partition_fn;
      c.num_partitions = it->second.num_partitions;
      c.partitions = &it->second.partitions;
    }
    return true;
  };
  return prune_with(d.num_docs, q, tree, mask, has, lookup);
}

}  // namespace pinot
