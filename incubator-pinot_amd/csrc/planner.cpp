// Host-side query planning for one segment: predicate evaluation on the dictionary and the physical
// filter plan. Restates (PC = pinot-core/src/main/java/org/apache/pinot/core):
//   PredicateEvaluatorProvider.getPredicateEvaluator      PC/operator/filter/predicate/PredicateEvaluatorProvider.java:37-80
//   EqualsPredicateEvaluatorFactory (dictionary)          .../EqualsPredicateEvaluatorFactory.java:71-102
//   NotEqualsPredicateEvaluatorFactory (dictionary)       .../NotEqualsPredicateEvaluatorFactory.java:71-127
//   InPredicateEvaluatorFactory (dictionary)              .../InPredicateEvaluatorFactory.java:83-127
//   NotInPredicateEvaluatorFactory (dictionary)           .../NotInPredicateEvaluatorFactory.java:83-145
//   RangePredicateEvaluatorFactory (offline dictionary)   .../RangePredicateEvaluatorFactory.java:79-158
//   RangePredicate string parsing                         PC/common/predicate/RangePredicate.java:41-67
//   ImmutableDictionaryReader.binarySearch                PC/segment/index/readers/ImmutableDictionaryReader.java:80-180
//   FilterPlanNode.constructPhysicalOperator              PC/plan/FilterPlanNode.java:70-126
//   FilterOperatorUtils.getLeaf/And/OrFilterOperator      PC/operator/filter/FilterOperatorUtils.java:43-161
#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdlib>

#include "engine.h"

namespace pinot {

// Integer.parseInt / Long.parseLong: optional sign, decimal digits, range-checked.
int64_t java_parse_integer(const std::string &s, int64_t lo, int64_t hi) {
  require(!s.empty(), PINOT_ERR_BAD_QUERY, "NumberFormatException: empty literal");
  size_t i = 0;
  bool neg = false;
  if (s[0] == '-' || s[0] == '+') {
    neg = s[0] == '-';
    i = 1;
    require(s.size() > 1, PINOT_ERR_BAD_QUERY, "NumberFormatException: " + s);
  }
  __int128 v = 0;
  for (; i < s.size(); i++) {
    require(s[i] >= '0' && s[i] <= '9', PINOT_ERR_BAD_QUERY, "NumberFormatException: For input string: \"" + s + "\"");
    v = v * 10 + (s[i] - '0');
    require(v <= (__int128)hi + 1, PINOT_ERR_BAD_QUERY, "NumberFormatException: out of range: " + s);
  }
  if (neg) v = -v;
  require(v >= lo && v <= hi, PINOT_ERR_BAD_QUERY, "NumberFormatException: out of range: " + s);
  return (int64_t)v;
}

// Double.parseDouble / Float.parseFloat (leading/trailing whitespace allowed, optional f/F/d/D suffix). as_float:
// the decimal rounded straight to float (strtof), as Float.parseFloat does, not through a double.
double java_parse_double(const std::string &raw, bool as_float) {
  size_t b = raw.find_first_not_of(" \t\n\r\f\v");
  size_t e = raw.find_last_not_of(" \t\n\r\f\v");
  require(b != std::string::npos, PINOT_ERR_BAD_QUERY, "NumberFormatException: empty literal");
  std::string s = raw.substr(b, e - b + 1);
  const std::string bad = "NumberFormatException: For input string: \"" + raw + "\"";
  const size_t sign = (s[0] == '+' || s[0] == '-') ? 1 : 0;
  const bool neg = s[0] == '-';
  if (s.compare(sign, std::string::npos, "NaN") == 0) return NAN;
  if (s.compare(sign, std::string::npos, "Infinity") == 0) return neg ? -INFINITY : INFINITY;
  if (s.back() == 'f' || s.back() == 'F' || s.back() == 'd' || s.back() == 'D') s.pop_back();
  // FloatingDecimal.readJavaFormatString's decimal grammar: digits [. digits] (a digit somewhere) [e|E [+|-] digits].
  // Hexadecimal literals and C's "inf" / "nan" spellings are not accepted (strtod alone would take them).
  size_t i = sign, digits = 0;
  while (i < s.size() && s[i] >= '0' && s[i] <= '9') i++, digits++;
  if (i < s.size() && s[i] == '.') {
    i++;
    while (i < s.size() && s[i] >= '0' && s[i] <= '9') i++, digits++;
  }
  require(digits > 0, PINOT_ERR_BAD_QUERY, bad);
  if (i < s.size() && (s[i] == 'e' || s[i] == 'E')) {
    i++;
    if (i < s.size() && (s[i] == '+' || s[i] == '-')) i++;
    size_t ed = 0;
    while (i < s.size() && s[i] >= '0' && s[i] <= '9') i++, ed++;
    require(ed > 0, PINOT_ERR_BAD_QUERY, bad);
  }
  require(i == s.size(), PINOT_ERR_BAD_QUERY, bad);
  char *end = nullptr;
  errno = 0;
  // correctly rounded, like FloatingDecimal; overflow -> +-inf
  const double v = as_float ? (double)std::strtof(s.c_str(), &end) : std::strtod(s.c_str(), &end);
  require(end && *end == 0, PINOT_ERR_BAD_QUERY, bad);
  return v;
}

// RangePredicate(lhs, rhs) (PC/common/predicate/RangePredicate.java:41-67): "(lo\t\thi]" with "*" for unbounded;
// "(" / ")" exclusive unless that bound is "*".
RangeBounds parse_range(const std::string &value) {
  std::string s = value;
  size_t b = s.find_first_not_of(" \t\n\r");
  size_t e = s.find_last_not_of(" \t\n\r");
  require(b != std::string::npos, PINOT_ERR_BAD_QUERY, "empty RANGE");
  s = s.substr(b, e - b + 1);
  size_t d = s.find("\t\t");
  require(d != std::string::npos && s.size() >= 2, PINOT_ERR_BAD_QUERY, "malformed RANGE: " + s);
  RangeBounds r;
  r.lower = s.substr(1, d - 1);
  r.upper = s.substr(d + 2, s.size() - d - 3);
  r.inc_lower = !(s[0] == '(') || r.lower == "*";
  r.inc_upper = !(s.back() == ')') || r.upper == "*";
  return r;
}

namespace {

// Returns insertionIndexOf(raw): index if found, else -(insertion point + 1).
int64_t insertion_index_of(const ColumnData &c, const std::string &raw) {
  int64_t low = 0, high = (int64_t)c.card - 1;
  auto search = [&](auto cmp) -> int64_t {
    while (low <= high) {
      int64_t mid = (low + high) >> 1;
      int r = cmp(mid);
      if (r < 0) low = mid + 1;
      else if (r > 0) high = mid - 1;
      else return mid;
    }
    return -(low + 1);
  };
  switch (c.data_type) {
    case PINOT_INT: {
      const int64_t v = java_parse_integer(raw, INT32_MIN, INT32_MAX);
      return search([&](int64_t m) { return c.dict_int[m] < v ? -1 : c.dict_int[m] > v ? 1 : 0; });
    }
    case PINOT_LONG: {
      const int64_t v = java_parse_integer(raw, INT64_MIN, INT64_MAX);
      return search([&](int64_t m) { return c.dict_int[m] < v ? -1 : c.dict_int[m] > v ? 1 : 0; });
    }
    case PINOT_FLOAT: {
      const double v = java_parse_double(raw, true);  // compared as float
      return search([&](int64_t m) { return c.dict_dbl[m] < v ? -1 : c.dict_dbl[m] > v ? 1 : 0; });
    }
    case PINOT_DOUBLE: {
      const double v = java_parse_double(raw);
      return search([&](int64_t m) { return c.dict_dbl[m] < v ? -1 : c.dict_dbl[m] > v ? 1 : 0; });
    }
    default: {
      // String.compareTo; byte order == code-point order for UTF-8. Padding byte 0: unpadded values. Any other
      // padding (legacy '%' segments): the value padded to the width against the full-width entries
      // (ImmutableDictionaryReader.binarySearch / padString, ImmutableDictionaryReader.java:152-216).
      if (c.string_pad == 0)
        return search([&](int64_t m) {
          int r = c.dict_str[m].compare(raw);
          return r < 0 ? -1 : r > 0 ? 1 : 0;
        });
      const size_t w = (size_t)c.string_width;
      std::string padded = raw;
      if (padded.size() < w) padded.append(w - padded.size(), (char)c.string_pad);
      return search([&](int64_t m) {
        const std::string entry(reinterpret_cast<const char *>(c.dict_be.data()) + (size_t)m * w, w);
        int r = entry.compare(padded);
        return r < 0 ? -1 : r > 0 ? 1 : 0;
      });
    }
  }
}

int64_t index_of(const ColumnData &c, const std::string &raw) {
  int64_t i = insertion_index_of(c, raw);
  return i >= 0 ? i : -1;
}

std::vector<std::string> split_values(const std::vector<std::string> &values) {
  // BaseInPredicate.getValues: a single value is split on "\t\t" (String.split drops trailing empties)
  if (values.size() != 1) return values;
  std::vector<std::string> out;
  const std::string &s = values[0];
  size_t start = 0;
  while (true) {
    size_t p = s.find("\t\t", start);
    if (p == std::string::npos) {
      out.push_back(s.substr(start));
      break;
    }
    out.push_back(s.substr(start, p - start));
    start = p + 2;
  }
  while (out.size() > 1 && out.back().empty()) out.pop_back();
  return out;
}

// A raw FLOAT / DOUBLE column's RawValueBased evaluators compare primitives (FloatRawValueBasedEqPredicateEvaluator
// `_matchingValue == value`, the range evaluators `value >= lower` ...): -0.0 equals 0.0, and NaN (as literal or value)
// compares false, where the transcoded dictionary (Double.compare order) keeps -0.0 < 0.0 and sorts NaN last. The
// dictionary evaluator above is right for every other entry, so only the NaN entry and the zero entries are
// re-evaluated with the primitive rules — unless a RANGE bound is NaN (nothing compares true), which re-evaluates all.
void raw_fp_semantics(const ColumnData &c, int op, const std::vector<std::string> &values, Evaluator &ev) {
  const bool f32 = c.data_type == PINOT_FLOAT;
  const int64_t card = c.card;
  if (card == 0) return;
  auto lit = [&](const std::string &s) { return java_parse_double(s, f32); };
  std::vector<double> set;
  RangeBounds rb;
  bool lo_set = false, hi_set = false;
  double lo = 0, hi = 0;
  if (op == PINOT_FILTER_IN || op == PINOT_FILTER_NOT_IN) {
    for (const auto &v : split_values(values)) set.push_back(lit(v));
  } else if (op == PINOT_FILTER_RANGE) {
    rb = parse_range(values[0]);
    if (rb.lower != "*") { lo_set = true; lo = lit(rb.lower); }
    if (rb.upper != "*") { hi_set = true; hi = lit(rb.upper); }
  } else {
    set.push_back(lit(values[0]));
  }
  auto match = [&](double v) -> bool {
    switch (op) {
      case PINOT_FILTER_EQUALITY: return v == set[0];
      case PINOT_FILTER_NOT: return v != set[0];
      case PINOT_FILTER_IN: for (double x : set) if (v == x) return true; return false;
      case PINOT_FILTER_NOT_IN: for (double x : set) if (v == x) return false; return true;
      default:
        return (!lo_set || (rb.inc_lower ? v >= lo : v > lo)) && (!hi_set || (rb.inc_upper ? v <= hi : v < hi));
    }
  };
  std::vector<int64_t> ids;
  if (op == PINOT_FILTER_RANGE && ((lo_set && std::isnan(lo)) || (hi_set && std::isnan(hi)))) {
    for (int64_t i = 0; i < card; i++) ids.push_back(i);
  } else {
    const bool nan_last = std::isnan(c.double_value(card - 1));
    if (nan_last) ids.push_back(card - 1);
    int64_t l = 0, r = card - (nan_last ? 1 : 0);  // the zero entries (-0.0, 0.0) are adjacent
    while (l < r) {
      const int64_t m = (l + r) / 2;
      if (c.double_value(m) < 0.0) l = m + 1; else r = m;
    }
    for (int64_t i = l; i < card - (nan_last ? 1 : 0) && c.double_value(i) == 0.0; i++) ids.push_back(i);
  }
  for (int64_t i : ids) {
    const uint8_t m = match(c.double_value(i)) ? 1 : 0;
    ev.num_matching += (int64_t)m - (int64_t)ev.matching[i];
    ev.matching[i] = m;
  }
  ev.always_true = ev.num_matching == card;
  ev.always_false = ev.num_matching == 0;
}

}  // namespace

Evaluator make_evaluator(const ColumnData &c, int op, const std::vector<std::string> &values) {
  Evaluator ev;
  const int64_t card = c.card;
  ev.matching.assign(card, 0);
  require(!values.empty(), PINOT_ERR_BAD_QUERY, "predicate on " + c.name + " has no value");
  switch (op) {
    case PINOT_FILTER_EQUALITY: {
      ev.kind = Evaluator::EQ;
      const int64_t id = index_of(c, values[0]);
      if (id >= 0) {
        ev.matching[id] = 1;
        ev.num_matching = 1;
        ev.always_true = card == 1;
      } else {
        ev.always_false = true;
      }
      break;
    }
    case PINOT_FILTER_NOT: {
      ev.kind = Evaluator::NEQ;
      const int64_t id = index_of(c, values[0]);
      std::fill(ev.matching.begin(), ev.matching.end(), 1);
      ev.num_matching = card;
      if (id >= 0) {
        ev.matching[id] = 0;
        ev.num_matching--;
        ev.always_false = card == 1;
      } else {
        ev.always_true = true;
      }
      break;
    }
    case PINOT_FILTER_IN:
    case PINOT_FILTER_NOT_IN: {
      int64_t n = 0;
      for (const auto &v : split_values(values)) {
        const int64_t id = index_of(c, v);
        if (id >= 0 && !ev.matching[id]) {
          ev.matching[id] = 1;
          n++;
        }
      }
      if (op == PINOT_FILTER_IN) {
        ev.kind = Evaluator::IN;
        ev.num_matching = n;
        ev.always_false = n == 0;
        ev.always_true = n == card;
      } else {
        ev.kind = Evaluator::NOT_IN;
        for (auto &m : ev.matching) m ^= 1;
        ev.num_matching = card - n;
        ev.always_true = n == 0;
        ev.always_false = n == card;
      }
      break;
    }
    case PINOT_FILTER_RANGE: {
      ev.kind = Evaluator::RANGE;
      const RangeBounds rb = parse_range(values[0]);
      const std::string &lower = rb.lower, &upper = rb.upper;
      const bool inc_lower = rb.inc_lower, inc_upper = rb.inc_upper;
      int64_t start, end;
      if (lower == "*") {
        start = 0;
      } else {
        int64_t ii = insertion_index_of(c, lower);
        start = ii < 0 ? -(ii + 1) : (inc_lower ? ii : ii + 1);
      }
      if (upper == "*") {
        end = card;
      } else {
        int64_t ii = insertion_index_of(c, upper);
        end = ii < 0 ? -(ii + 1) : (inc_upper ? ii + 1 : ii);
      }
      const int64_t n = end - start;
      if (n <= 0) {
        ev.always_false = true;
      } else {
        std::fill(ev.matching.begin() + start, ev.matching.begin() + end, 1);
        ev.num_matching = n;
        ev.always_true = n == card;
      }
      break;
    }
    default:
      throw Error(PINOT_ERR_UNSUPPORTED, "unsupported predicate operator");
  }
  if (c.raw && (c.data_type == PINOT_FLOAT || c.data_type == PINOT_DOUBLE)) raw_fp_semantics(c, op, values, ev);
  return ev;
}

FilterTreeInput decode_filter(int32_t n, const pinot_filter_node *nodes) {
  std::vector<FilterTreeInput> stack;
  for (int32_t i = 0; i < n; i++) {
    const pinot_filter_node &nd = nodes[i];
    FilterTreeInput t;
    t.op = nd.op;
    if (nd.op == PINOT_FILTER_AND || nd.op == PINOT_FILTER_OR) {
      require(nd.num_children >= 1 && (size_t)nd.num_children <= stack.size(), PINOT_ERR_BAD_ARG,
              "malformed postfix filter");
      t.children.assign(std::make_move_iterator(stack.end() - nd.num_children), std::make_move_iterator(stack.end()));
      stack.resize(stack.size() - nd.num_children);
    } else {
      require(nd.op >= PINOT_FILTER_EQUALITY && nd.op <= PINOT_FILTER_NOT_IN, PINOT_ERR_UNSUPPORTED,
              "unsupported filter operator");
      require(nd.column != nullptr, PINOT_ERR_BAD_ARG, "filter leaf without column");
      t.column = nd.column;
      for (int32_t k = 0; k < nd.num_values; k++) t.values.emplace_back(nd.values[k] ? nd.values[k] : "");
    }
    stack.push_back(std::move(t));
  }
  require(stack.size() == 1, PINOT_ERR_BAD_ARG, "filter must reduce to exactly one tree");
  return std::move(stack[0]);
}

namespace {

// FilterOperatorUtils.reorderAndFilterChildOperators (:130-161): sorted, bitmap, AND, OR, scan; a multi-value scan
// after the single-value ones (getScanBasedFilterPriority)
int and_priority(const SegmentData &seg, const FilterNode &n) {
  switch (n.type) {
    case FilterNode::SORTED: return 0;
    case FilterNode::BITMAP: return 1;
    case FilterNode::AND: return 2;
    case FilterNode::OR: return 3;
    default: return n.col >= 0 && seg.cols[n.col]->mv ? 5 : 4;
  }
}

FilterNode construct(const SegmentData &seg, const FilterTreeInput &t) {
  if (t.op == PINOT_FILTER_AND || t.op == PINOT_FILTER_OR) {
    const bool is_and = t.op == PINOT_FILTER_AND;
    FilterNode out;
    out.type = is_and ? FilterNode::AND : FilterNode::OR;
    for (const auto &ct : t.children) {
      FilterNode c = construct(seg, ct);
      if (is_and) {
        if (c.type == FilterNode::EMPTY) return FilterNode{FilterNode::EMPTY};
        if (c.type != FilterNode::MATCH_ALL) out.children.push_back(std::move(c));
      } else {
        if (c.type == FilterNode::MATCH_ALL) return FilterNode{FilterNode::MATCH_ALL};
        if (c.type != FilterNode::EMPTY) out.children.push_back(std::move(c));
      }
    }
    if (out.children.empty()) return FilterNode{is_and ? FilterNode::MATCH_ALL : FilterNode::EMPTY};
    if (out.children.size() == 1) return std::move(out.children[0]);
    if (is_and)
      std::stable_sort(out.children.begin(), out.children.end(),
                       [&](const FilterNode &a, const FilterNode &b) {
                         return and_priority(seg, a) < and_priority(seg, b);
                       });
    return out;
  }
  const int ci = seg.by_name.count(t.column) ? seg.by_name.at(t.column) : -1;
  require(ci >= 0, PINOT_ERR_BAD_QUERY, "unknown filter column: " + t.column);
  const ColumnData &col = *seg.cols[ci];
  auto ev = std::make_shared<Evaluator>(make_evaluator(col, t.op, t.values));
  if (ev->always_false) return FilterNode{FilterNode::EMPTY};
  if (ev->always_true) return FilterNode{FilterNode::MATCH_ALL};
  FilterNode leaf;
  leaf.col = ci;
  leaf.ev = ev;
  // getLeafFilterOperator: inverted index && !RANGE -> sorted / bitmap operator, else scan
  if (col.has_inverted && ev->kind != Evaluator::RANGE) {
    leaf.type = col.is_sorted ? FilterNode::SORTED : FilterNode::BITMAP;
  } else {
    leaf.type = FilterNode::SCAN;
  }
  return leaf;
}

}  // namespace

FilterNode plan_filter(const SegmentData &seg, const FilterTreeInput *tree) {
  if (tree == nullptr) return FilterNode{FilterNode::MATCH_ALL};
  return construct(seg, *tree);
}

}  // namespace pinot
