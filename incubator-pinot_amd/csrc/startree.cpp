// Star-tree v2 (PC/startree/v2; PC = pinot-core/src/main/java/org/apache/pinot/core): the index a segment carries
// beside its columns, and the plan that answers a query from its pre-aggregated documents.
//
//   attach_star_tree   OffHeapStarTree (PC/startree/OffHeapStarTree.java:38-70) parsed and checked (little-endian
//                      header, 7-int nodes, children in range and sorted, doc ranges inside the star docs); the star
//                      docs registered as their own device segment (dimension columns over the segment's
//                      dictionaries, metric columns "count__*" / "sum__x" / "min__x" / "max__x" and the AvgPair halves
//                      "avg__x.sum" / "avg__x.count" transcoded like raw columns; the HyperLogLog columns
//                      "distinctCountHLL__x" decoded into u8 register rows); the dimensions' dictIds kept on the host
//                      for the traversal's remaining predicates.
//   star_tree_fits     StarTreeUtils.isFitForStarTree (PC/startree/StarTreeUtils.java:50-95).
//   star_tree_match    StarTreeFilterOperator (PC/startree/operator/StarTreeFilterOperator.java): evaluators on the
//                      segment's dictionaries, the BFS over the tree, then the remaining predicates ANDed over the
//                      matched star docs — a host pass over a tree of a few thousand nodes and the matched docs'
//                      dictIds; the aggregation over the matched docs runs on the device (executor.cpp).
#include <algorithm>
#include <cstring>
#include <deque>
#include <map>
#include <set>

#include "engine.h"

namespace pinot {
namespace {

constexpr uint64_t kStarTreeMagic = 0xBADDA55B00DAD00Dull;
constexpr int32_t kAll = -1;

uint32_t le32(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }
uint64_t le64(const uint8_t *p) { return (uint64_t)le32(p) | ((uint64_t)le32(p + 4) << 32); }

uint32_t read_bits(const uint8_t *fwd, int bits, uint64_t i) {  // PinotDataBitSet.readInt
  uint64_t pos = i * (uint64_t)bits;
  uint32_t v = 0;
  for (int b = 0; b < bits; b++, pos++) v = (v << 1) | ((fwd[pos >> 3] >> (7 - (pos & 7))) & 1u);
  return v;
}

void collect_leaves(const FilterTreeInput &t, std::vector<const FilterTreeInput *> &out, bool &has_or) {
  if (t.op == PINOT_FILTER_AND || t.op == PINOT_FILTER_OR) {
    has_or = has_or || t.op == PINOT_FILTER_OR;
    for (const auto &c : t.children) collect_leaves(c, out, has_or);
    return;
  }
  out.push_back(&t);
}

}  // namespace

std::string star_pair_column(const pinot_agg_spec &a) {
  const std::string col = a.column ? a.column : "*";
  switch (a.function) {
    case PINOT_AGG_COUNT: return "count__*";
    case PINOT_AGG_SUM: return "sum__" + col;
    case PINOT_AGG_MIN: return "min__" + col;
    case PINOT_AGG_MAX: return "max__" + col;
    case PINOT_AGG_AVG: return "avg__" + col;  // the AvgPair column, as "avg__x.sum" + "avg__x.count"
    case PINOT_AGG_DISTINCTCOUNTHLL: return "distinctCountHLL__" + col;
    default: return "";
  }
}

void attach_star_tree(Engine &e, SegmentData &seg, const pinot_star_tree_desc &d) {
  require(d.tree && d.docs, PINOT_ERR_BAD_ARG, seg.name + ": star-tree without tree bytes or documents");
  const uint8_t *b = d.tree;
  const uint64_t n = d.tree_len;
  require(n >= 24 && le64(b) == kStarTreeMagic, PINOT_ERR_BAD_ARG, seg.name + ": invalid star-tree magic marker");
  require(le32(b + 8) == 1, PINOT_ERR_BAD_ARG, seg.name + ": star-tree version");
  const uint64_t header = le32(b + 12), ndims = le32(b + 16);
  require(ndims >= 1 && ndims < 1024 && header <= n, PINOT_ERR_BAD_ARG, seg.name + ": star-tree header");
  auto st = std::make_unique<StarTreeData>();
  st->dims.assign(ndims, "");
  uint64_t off = 20;
  for (uint64_t i = 0; i < ndims; i++) {
    require(off + 8 <= header, PINOT_ERR_BAD_ARG, seg.name + ": star-tree header truncated");
    const uint32_t idx = le32(b + off), len = le32(b + off + 4);
    off += 8;
    require(idx < ndims && off + len <= header && st->dims[idx].empty(), PINOT_ERR_BAD_ARG,
            seg.name + ": star-tree dimension entry");
    st->dims[idx].assign(reinterpret_cast<const char *>(b + off), len);
    off += len;
  }
  require(off + 4 == header, PINOT_ERR_BAD_ARG, seg.name + ": star-tree header length mis-match");
  const uint64_t nnodes = le32(b + off);
  require(header + nnodes * 28 == n && nnodes >= 1, PINOT_ERR_BAD_ARG, seg.name + ": star-tree buffer size mis-match");
  const int32_t ndocs = d.docs->num_docs;
  st->nodes.resize(nnodes);
  for (uint64_t i = 0; i < nnodes; i++) {
    const uint8_t *p = b + header + 28 * i;
    StarTreeNodeRec &r = st->nodes[i];
    int32_t *f = &r.dim;
    for (int k = 0; k < 7; k++) f[k] = (int32_t)le32(p + 4 * k);
  }
  for (uint64_t i = 0; i < nnodes; i++) {  // everything the traversal dereferences
    const StarTreeNodeRec &r = st->nodes[i];
    require(r.agg >= -1 && r.agg < ndocs, PINOT_ERR_BAD_ARG, seg.name + ": star-tree aggregated doc out of range");
    if (r.first == -1) {
      require(r.start >= 0 && r.start <= r.end && r.end <= ndocs, PINOT_ERR_BAD_ARG,
              seg.name + ": star-tree leaf doc range");
      continue;
    }
    require(r.first > (int64_t)i && r.first <= r.last && (uint64_t)r.last < nnodes, PINOT_ERR_BAD_ARG,
            seg.name + ": star-tree child range");
    const int32_t cd = st->nodes[r.first].dim;
    require(cd >= 0 && (uint64_t)cd < ndims, PINOT_ERR_BAD_ARG, seg.name + ": star-tree child dimension");
    for (int32_t c = r.first; c <= r.last; c++) {
      require(st->nodes[c].dim == cd, PINOT_ERR_BAD_ARG, seg.name + ": star-tree children on different dimensions");
      require(c == r.first || st->nodes[c].value > st->nodes[c - 1].value, PINOT_ERR_BAD_ARG,
              seg.name + ": star-tree children not sorted by dimension value");
    }
  }
  // the star docs: dimensions over the segment's dictionaries, metric pairs
  for (const std::string &dn : st->dims) {
    const ColumnData &pc = *seg.column(dn);
    require(!pc.mv && !pc.raw, PINOT_ERR_UNSUPPORTED, seg.name + ": star-tree dimension " + dn + " is not a dictionary SV column");
    const pinot_column_desc *cd = nullptr;
    for (int32_t k = 0; k < d.docs->num_columns; k++)
      if (d.docs->columns[k].name && dn == d.docs->columns[k].name) cd = &d.docs->columns[k];
    require(cd && cd->cardinality == pc.card && cd->bits_per_value == pc.bits && cd->data_type == pc.data_type,
            PINOT_ERR_BAD_ARG, seg.name + ": star-tree dimension " + dn + " must use the segment column's dictionary");
    require(cd->forward_index && cd->forward_index_len >= ((uint64_t)ndocs * pc.bits + 7) / 8 && !cd->is_sorted,
            PINOT_ERR_BAD_ARG, seg.name + ": star-tree dimension " + dn + " forward index");
    std::vector<uint32_t> ids((size_t)ndocs);
    for (int32_t i = 0; i < ndocs; i++) ids[i] = read_bits(cd->forward_index, pc.bits, (uint64_t)i);
    st->host_dims.push_back(std::move(ids));
  }
  // HyperLogLog pair columns ("distinctCountHLL__x": HyperLogLog.getBytes per star doc, raw var-byte layout) become
  // u8 register rows on the device; the other columns register as the star docs' segment
  std::vector<pinot_column_desc> plain;
  for (int32_t k = 0; k < d.docs->num_columns; k++) {
    const pinot_column_desc &c = d.docs->columns[k];
    const std::string cn = c.name ? c.name : "";
    if (cn.rfind("distinctCountHLL__", 0) != 0) {
      plain.push_back(c);
      continue;
    }
    require(c.data_type == PINOT_STRING && c.encoding == PINOT_ENCODING_RAW && c.forward_index &&
                c.forward_index_len >= ((uint64_t)ndocs + 1) * 4,
            PINOT_ERR_BAD_ARG, seg.name + ": star-tree HyperLogLog column " + cn + " must be raw bytes");
    require(!st->regs.count(cn), PINOT_ERR_BAD_ARG, seg.name + ": duplicate star-tree column " + cn);
    const uint8_t *f = c.forward_index;
    auto be32 = [](const uint8_t *q) { return ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3]; };
    const uint64_t body = ((uint64_t)ndocs + 1) * 4;
    std::vector<uint8_t> regs((size_t)ndocs * 256);
    for (int32_t i = 0; i < ndocs; i++) {
      const uint64_t o = be32(f + 4 * (uint64_t)i), e2 = be32(f + 4 * ((uint64_t)i + 1));
      require(e2 >= o && e2 - o == 180 && body + e2 <= c.forward_index_len, PINOT_ERR_BAD_ARG,
              seg.name + ": " + cn + ": a HyperLogLog value is not 180 bytes (log2m 8)");
      const uint8_t *h = f + body + o;  // HyperLogLog.getBytes: log2m, size in bytes, RegisterSet words
      require(be32(h) == 8 && be32(h + 4) == 172, PINOT_ERR_UNSUPPORTED, seg.name + ": " + cn + ": log2m other than 8");
      for (int p = 0; p < 256; p++) regs[(size_t)i * 256 + p] = (uint8_t)((be32(h + 8 + 4 * (p / 6)) >> (5 * (p % 6))) & 31u);
    }
    DeviceBuffer &db = st->regs[cn];
    db.alloc(regs.size() + 16);
    PINOT_HIP(hipMemcpy(db.get(), regs.data(), regs.size(), hipMemcpyHostToDevice));
    seg.device_bytes += regs.size();
  }
  pinot_segment_desc plain_desc = *d.docs;
  plain_desc.columns = plain.data();
  plain_desc.num_columns = (int32_t)plain.size();
  st->docs = register_segment(e, plain_desc);
  // ValueAggregatorFactory's value types: COUNT (and AvgPair's count half) LONG, SUM / MIN / MAX (and AvgPair's sum
  // half) DOUBLE — the star aggregation reads the counts as exact integers and the others as doubles
  auto ends_with = [](const std::string &a, const char *b) {
    const size_t n = strlen(b);
    return a.size() >= n && a.compare(a.size() - n, n, b) == 0;
  };
  auto is_metric = [](const std::string &n) {  // function-column pair columns: "<function>__<column>" (+ ".sum" / ".count")
    for (const char *f : {"count__", "sum__", "min__", "max__", "avg__"})
      if (n.rfind(f, 0) == 0) return true;
    return false;
  };
  for (auto &c : st->docs->cols)
    if (is_metric(c->name)) {  // a dimension whose name merely contains "__" keeps its own type
      require(c->numeric(), PINOT_ERR_BAD_ARG, seg.name + ": star-tree metric " + c->name + " must be numeric");
      const bool count = c->name.rfind("count__", 0) == 0 || ends_with(c->name, ".count");
      require(count ? c->data_type == PINOT_LONG : c->data_type == PINOT_DOUBLE, PINOT_ERR_BAD_ARG,
              seg.name + ": star-tree metric " + c->name + (count ? " must be LONG" : " must be DOUBLE"));
    }
  seg.device_bytes += st->docs->device_bytes;
  seg.star = std::move(st);
}

bool star_tree_fits(const SegmentData &seg, const pinot_query &q) {
  if (!seg.star) return false;
  const StarTreeData &st = *seg.star;
  const std::set<std::string> dims(st.dims.begin(), st.dims.end());
  for (int a = 0; a < q.num_aggregations; a++) {
    const std::string p = star_pair_column(q.aggregations[a]);
    if (p.empty()) return false;
    if (q.aggregations[a].function == PINOT_AGG_AVG) {
      if (!st.docs->by_name.count(p + ".sum") || !st.docs->by_name.count(p + ".count")) return false;
    } else if (q.aggregations[a].function == PINOT_AGG_DISTINCTCOUNTHLL) {
      if (!st.regs.count(p)) return false;
    } else if (!st.docs->by_name.count(p)) {
      return false;
    }
  }
  for (int j = 0; j < q.num_group_by; j++)
    if (!dims.count(q.group_by[j])) return false;
  if (q.num_filter_nodes == 0) return true;
  const FilterTreeInput t = decode_filter(q.num_filter_nodes, q.filter);
  std::vector<const FilterTreeInput *> leaves;
  bool has_or = false;
  collect_leaves(t, leaves, has_or);
  if (has_or) return false;
  for (auto *l : leaves)
    if (!dims.count(l->column)) return false;
  return true;
}

StarMatch star_tree_match(const SegmentData &seg, const pinot_query &q, const FilterTreeInput *tree) {
  const StarTreeData &st = *seg.star;
  StarMatch out;
  const int32_t ndocs = st.docs->num_docs;
  std::map<std::string, std::vector<uint8_t>> matching;  // per filtered column: AND of its evaluators
  std::set<std::string> group;
  for (int j = 0; j < q.num_group_by; j++) group.insert(q.group_by[j]);
  if (tree) {
    std::vector<const FilterTreeInput *> leaves;
    bool has_or = false;
    collect_leaves(*tree, leaves, has_or);
    for (auto *l : leaves) {
      const ColumnData &c = *seg.column(l->column);
      const Evaluator ev = make_evaluator(c, l->op, l->values);
      if (ev.always_false) {
        out.empty = true;
        return out;
      }
      if (ev.always_true) continue;
      auto it = matching.find(l->column);
      if (it == matching.end()) {
        matching[l->column] = ev.matching;
      } else {
        for (size_t i = 0; i < ev.matching.size(); i++) it->second[i] &= ev.matching[i];
      }
    }
  }
  for (auto &m : matching) group.erase(m.first);
  std::map<std::string, int> dim_index;
  for (size_t i = 0; i < st.dims.size(); i++) dim_index[st.dims[i]] = (int)i;
  out.bits.assign(((size_t)ndocs + 63) / 64, 0);
  auto set_doc = [&](int32_t d) { out.bits[(size_t)d >> 6] |= 1ull << (d & 63); };
  std::set<std::string> remaining_cols;
  struct Entry {
    int32_t node;
    std::set<std::string> pred, grp;
  };
  std::deque<Entry> queue;
  std::set<std::string> all_pred;
  for (auto &m : matching) all_pred.insert(m.first);
  queue.push_back({0, all_pred, group});
  while (!queue.empty()) {
    Entry en = std::move(queue.front());
    queue.pop_front();
    const StarTreeNodeRec &nd = st.nodes[en.node];
    if (en.pred.empty() && en.grp.empty()) {
      require(nd.agg >= 0, PINOT_ERR_BAD_ARG, seg.name + ": star-tree node without an aggregated doc");
      set_doc(nd.agg);
      continue;
    }
    if (nd.first == -1) {
      for (int32_t d = nd.start; d < nd.end; d++) set_doc(d);
      remaining_cols.insert(en.pred.begin(), en.pred.end());
      continue;
    }
    const std::string &next = st.dims[st.nodes[nd.first].dim];
    if (en.pred.count(next)) {
      const std::vector<uint8_t> &m = matching[next];
      if (std::find(m.begin(), m.end(), 1) == m.end()) {  // getMatchingDictIds empty: no result
        out.empty = true;
        return out;
      }
      std::set<std::string> np = en.pred;
      np.erase(next);
      for (int32_t c = nd.first; c <= nd.last; c++) {
        const int32_t v = st.nodes[c].value;
        if (v != kAll && v >= 0 && (size_t)v < m.size() && m[v]) queue.push_back({c, np, en.grp});
      }
    } else {
      std::set<std::string> ng = en.grp;
      if (!en.grp.count(next)) {
        if (st.nodes[nd.first].value == kAll) {  // the star child (sorted first)
          queue.push_back({nd.first, en.pred, en.grp});
          continue;
        }
      } else {
        ng.erase(next);
      }
      for (int32_t c = nd.first; c <= nd.last; c++)
        if (st.nodes[c].value != kAll) queue.push_back({c, en.pred, ng});
    }
  }
  // the remaining predicates: a bitmap operator AND scan operators over the star docs (applyAnd counts the answer)
  for (const std::string &col : remaining_cols) {
    const std::vector<uint8_t> &m = matching[col];
    const std::vector<uint32_t> &ids = st.host_dims[dim_index[col]];
    for (size_t w = 0; w < out.bits.size(); w++) {
      uint64_t x = out.bits[w], keep = 0;
      while (x) {
        const int bit = __builtin_ctzll(x);
        x &= x - 1;
        const size_t d = w * 64 + bit;
        out.entries_in_filter++;
        if (m[ids[d]]) keep |= 1ull << bit;
      }
      out.bits[w] = keep;
    }
  }
  for (uint64_t w : out.bits) out.docs += __builtin_popcountll(w);
  return out;
}

}  // namespace pinot
