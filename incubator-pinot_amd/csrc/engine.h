// Host-side engine: device-resident segments, query planning, execution.
#pragma once
#include <chrono>
#include <cmath>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "bloom.h"
#include "common.h"
#include "kernels.h"

namespace pinot {

// ------------------------------------------------------------------ segments
struct ColumnData {
  std::string name;
  int data_type = PINOT_INT;
  int32_t card = 0;
  int32_t bits = 0;
  bool is_sorted = false;
  bool has_inverted = false;
  int32_t string_width = 0;
  int32_t string_pad = 0;             // STRING padding byte (0 = '\0'; legacy segments '%')
  int32_t num_docs = 0;
  bool raw = false;                   // registered from a raw (no-dictionary) forward index, transcoded
  bool has_minmax = false;            // metadata minValue / maxValue present (the segment pruner's only input)
  std::string min_value, max_value;
  bool mv = false;                    // multi-value column: fwd packs its entries, mv_offsets[doc] = first entry
  int64_t num_values = 0;             // totalNumberOfEntries (MV)
  int32_t max_mv = 0;                 // longest row (MV)
  uint64_t mv_raw_offset = 0;         // byte offset of the packed entries in the descriptor's forward_index
  std::vector<uint32_t> mv_offsets_host;  // numDocs + 1 row starts (host copy: oracle-free checks, key strings)
  DeviceBuffer mv_offsets;            // u32 [numDocs + 1]
  BloomFilter bloom;                  // empty: none (ColumnValueSegmentPruner's EQUALITY test)
  int partition_fn = PF_NONE;         // PartitionFunctionKind of the partition metadata (PartitionSegmentPruner)
  int32_t num_partitions = 0;
  std::vector<int32_t> partitions;    // the partitions the segment holds, sorted

  // host copies (dictionary-sized; used for predicate evaluation and key materialisation)
  std::vector<uint8_t> dict_be;        // raw BE dictionary bytes
  std::vector<int64_t> dict_int;       // INT / LONG values
  std::vector<double> dict_dbl;        // FLOAT / DOUBLE values (float widened exactly)
  std::vector<std::string> dict_str;   // STRING values (unpadded)
  std::vector<int32_t> sorted_start, sorted_end;  // sorted columns
  std::vector<int32_t> inv_dir;        // per dictId [dir[i], dir[i+1]) into containers
  std::vector<uint16_t> inv_keys;      // per container its roaring key (the fused plan's per-key container lists)
  std::vector<uint64_t> inv_bytes;     // serialized roaring bytes per dictId (cost model)
  // INT/LONG dictionary that is an arithmetic progression value(id) = affine_base + affine_step * id:
  // SUM/AVG then need Σ dictId only (no dictionary gather)
  bool affine = false;
  int64_t affine_base = 0, affine_step = 0;

  // device
  DeviceBuffer fwd;             // packed forward index (synthesised for sorted columns)
  uint64_t fwd_bytes = 0;       // ceil(N*b/8)
  DeviceBuffer dict_dev;        // int32 (INT) / int64 (LONG) / double (FLOAT, DOUBLE); none for STRING
  DeviceBuffer inv_payload, inv_containers, inv_dir_dev;
  DeviceBuffer hll_lut;         // u16 per dictId, built lazily

  DevColumn dev() const { return DevColumn{fwd.get<uint8_t>(), bits, card}; }
  int value_kind() const {  // 0 int32, 1 int64, 2 double
    return data_type == PINOT_INT ? 0 : data_type == PINOT_LONG ? 1 : 2;
  }
  bool numeric() const { return data_type != PINOT_STRING; }
  std::string string_value(int32_t id) const;  // Dictionary.getStringValue
  double double_value(int32_t id) const;
};

// Host-side products of parse_column that register_column uploads.
struct ParsedIndexes {
  std::vector<int32_t> sorted_starts;         // sorted column: card + 1 range starts (last = numDocs)
  std::vector<RoaringContainer> containers;   // inverted index: container directory of every dictId
};
// segment_parse.cpp: validates and decodes one column descriptor on the host (no device work).
void parse_column(ColumnData &c, const pinot_column_desc &d, int32_t num_docs, ParsedIndexes &out);
// A raw column's descriptor transcoded to the dictionary-encoded form (sorted distinct values + packed dictIds);
// false (out untouched) for a dictionary column. out.desc points into out's buffers.
struct TranscodedColumn {
  pinot_column_desc desc{};
  std::vector<uint8_t> dictionary, forward_index;
};
bool transcode_raw(const pinot_column_desc &d, int32_t num_docs, TranscodedColumn &out);
// The checks every raw column passes; the value width (4 / 8) of a raw numeric column, 0 for STRING or dictionary.
int raw_numeric_width(const pinot_column_desc &d, int32_t num_docs);
// out.dictionary and out.desc from the distinct order-preserving keys (ascending); out.forward_index set by the caller.
void transcoded_numeric_finish(const pinot_column_desc &d, const uint64_t *uniq, int64_t card, TranscodedColumn &out);
struct Engine;
// segment.cpp: a raw column's dictionary form as registration builds it (numeric on the device when e.raw_device).
bool transcode_column(Engine &e, const pinot_column_desc &d, int32_t num_docs, TranscodedColumn &tc);
// Same, on `threads` host threads (0: one per 1 M docs, at most 16); the output does not depend on the count.
bool transcode_raw_threads(const pinot_column_desc &d, int32_t num_docs, TranscodedColumn &out, size_t threads);
void validate_segment(const pinot_segment_desc &d);
// The pruning metadata of a column descriptor (bloom filter bytes or creation from the decoded dictionary, partition
// metadata) into c; c's dictionary must be decoded already (parse_column calls it).
void parse_pruning_metadata(ColumnData &c, const pinot_column_desc &d);
void parse_dictionary_only(ColumnData &c, const pinot_column_desc &d);  // dictionary + pruning metadata only
// FixedByteChunkSingleValueReader over a .sv.raw.fwd file: the docs' values back to back, big-endian (segment_reader.cpp)
std::vector<uint8_t> read_raw_chunks(const uint8_t *b, uint64_t n, int64_t num_docs, int entry_size, const std::string &what);
void parse_multi_value(ColumnData &c, const pinot_column_desc &d, int32_t num_docs);
std::string java_double_to_string(double v);  // Double.toString
std::string java_float_to_string(float v);    // Float.toString

// segment_reader.cpp: a Pinot segment directory (v1 / v2 files, or v3 columns.psf + index_map) mapped read-only
// and described as a pinot_segment_desc (ImmutableSegmentLoader.load's inputs).
struct MappedFile {
  const uint8_t *data = nullptr;
  size_t size = 0;
  explicit MappedFile(const std::string &path);
  ~MappedFile();
  MappedFile(const MappedFile &) = delete;
  MappedFile &operator=(const MappedFile &) = delete;
};
struct SegmentDirData {
  std::string name;
  int32_t num_docs = 0;
  std::vector<std::string> column_names, skipped;  // served columns; multi-value / raw / BYTES columns left out
  std::vector<pinot_column_desc> cols;
  std::vector<std::unique_ptr<MappedFile>> files;
  std::vector<std::vector<uint8_t>> owned;  // raw columns: the decompressed chunk values
  std::deque<std::string> strings;          // min / max values the descriptors point at (stable addresses)
  std::deque<std::vector<int32_t>> ints;    // partition values the descriptors point at
  std::string time_column;                  // segment.time.column.name
  pinot_segment_desc desc() const;
  // star-tree v2 index (the first tree, startree.v2.0.*): the tree bytes and the star docs' columns
  bool has_star = false;
  const uint8_t *star_tree = nullptr;
  uint64_t star_tree_len = 0;
  int32_t star_num_docs = 0;
  std::vector<pinot_column_desc> star_cols;
  std::deque<std::string> star_names;
  pinot_segment_desc star_desc() const;
};
void read_segment_dir(const std::string &index_dir, SegmentDirData &out);
// segment.name (metadata.properties) and creation.meta's CRC (false when the directory has no creation.meta)
bool read_segment_identity(const std::string &index_dir, std::string &name, int64_t &crc);
uint64_t next_segment_uid();

struct SegmentData;
// A segment's star-tree v2 (startree.cpp): the tree (OffHeapStarTreeNode fields), the split order, the star docs as a
// registered segment (dimension columns + metric columns) and the dimensions' dictIds on the host for the traversal's
// remaining predicates.
struct StarTreeNodeRec {
  int32_t dim, value, start, end, agg, first, last;
};
struct StarTreeData {
  std::vector<StarTreeNodeRec> nodes;
  std::vector<std::string> dims;                  // split order
  std::vector<std::vector<uint32_t>> host_dims;   // [dim][star doc] dictIds
  std::unique_ptr<SegmentData> docs;
  std::map<std::string, DeviceBuffer> regs;       // "distinctCountHLL__x" -> u8 registers [star doc][256]
};

struct SegmentData {
  std::string name;
  std::unique_ptr<StarTreeData> star;  // star-tree v2 index, when attached
  uint64_t uid = 0;                 // process-unique (never reused, unlike addresses): plan cache keys
  int32_t num_docs = 0;
  std::vector<std::unique_ptr<ColumnData>> cols;
  std::unordered_map<std::string, int> by_name;
  std::vector<std::string> unserved;  // columns the segment has but the engine does not serve (loader's left-outs)
  uint64_t device_bytes = 0;

  ColumnData *column(const std::string &n) const {
    auto it = by_name.find(n);
    if (it == by_name.end()) throw Error(PINOT_ERR_BAD_QUERY, "unknown column: " + n);
    return cols[it->second].get();
  }
  int64_t nwords() const { return ceil_div(num_docs, 64); }
};

// ------------------------------------------------------------------ predicate evaluation
// Dictionary-based predicate evaluator (PredicateEvaluatorProvider.java:37-80).
struct Evaluator {
  enum Kind { EQ, NEQ, IN, NOT_IN, RANGE } kind;
  std::vector<uint8_t> matching;  // per dictId
  int64_t num_matching = 0;
  bool always_true = false, always_false = false;
  bool exclusive() const { return kind == NEQ || kind == NOT_IN; }
};

Evaluator make_evaluator(const ColumnData &col, int op, const std::vector<std::string> &values);

// Physical filter plan for one segment (FilterPlanNode.constructPhysicalOperator +
// FilterOperatorUtils.getLeafFilterOperator/getAndFilterOperator/getOrFilterOperator).
struct FilterNode {
  enum Type { EMPTY, MATCH_ALL, SCAN, SORTED, BITMAP, AND, OR } type;
  int col = -1;
  std::shared_ptr<Evaluator> ev;
  std::vector<FilterNode> children;
};

struct FilterTreeInput {  // decoded pinot_filter_node (postfix) as a tree
  int op;
  std::string column;
  std::vector<std::string> values;
  std::vector<FilterTreeInput> children;
};

FilterTreeInput decode_filter(int32_t n, const pinot_filter_node *nodes);
FilterNode plan_filter(const SegmentData &seg, const FilterTreeInput *tree);

// Literals as FieldSpec.DataType.convert reads them (Integer/Long.valueOf, Float/Double.valueOf) and RANGE strings
// as RangePredicate splits them (planner.cpp).
int64_t java_parse_integer(const std::string &s, int64_t lo, int64_t hi);
double java_parse_double(const std::string &raw, bool as_float = false);
struct RangeBounds {
  std::string lower, upper;  // "*" = unbounded
  bool inc_lower = true, inc_upper = true;
};
RangeBounds parse_range(const std::string &value);

// Segment pruning before the plan (pruner.cpp): SegmentPrunerService.prune with the pruners of `mask`
// (PINOT_PRUNER_* bits), applied in the server's default order.
bool prune_segment(const SegmentData &s, const pinot_query &q, const FilterTreeInput *tree, int32_t mask);
bool prune_segment_desc(const pinot_segment_desc &d, const pinot_query &q, const FilterTreeInput *tree, int32_t mask);

// ------------------------------------------------------------------ engine
struct Engine {
  int device = 0;
  hipStream_t stream = nullptr;
  // result D2H fan-out (d2h.streams): the group-by result arrays copied on parallel streams (one SDMA queue each)
  bool compact_d2h = false;   // d2h.compact: key bitmap + u32 read-back (config 4: 1.26 vs 1.19 ms, no gain: off)
  PinnedBuffer compact_host;  // its host staging
  int d2h_streams = 1;         // measured on config 4: 1 / 2 / 4 streams all ~1.15 ms for 32 MB (PCIe-bound)
  std::vector<hipStream_t> copy_streams;
  hipEvent_t ev_copy = nullptr;
  std::mutex mu;
  int64_t next_handle = 1;
  std::unordered_map<int64_t, std::unique_ptr<SegmentData>> segments;
  // device segment cache: segment name -> (creation.meta CRC, handle) (pinot_gpu_segment_acquire)
  std::unordered_map<std::string, std::pair<int64_t, int64_t>> segment_cache;
  std::unordered_map<int64_t, int64_t> acquire_refs;  // handle -> references taken by pinot_gpu_segment_acquire

  // configuration
  int num_groups_limit = 100000;
  std::string force_filter;   // "", "scan", "index": planner override for tests
  bool use_affine = true;     // agg.affine: arithmetic-progression dictionary SUM shortcut
  bool use_fused = true;      // exec.fused: one k_scan_query launch per aggregation query when the shape allows
  bool use_star_tree = true;  // startree.use: star-tree plans for the queries a segment's tree fits
  bool stats_exact = false;   // stats.exact: numEntriesScannedInFilter replayed per the iterator protocol (host)
  std::vector<const SegmentData *> star_answered;  // the current query's segments answered on their star-trees
  bool use_nt = true;         // exec.nt: non-temporal policy on the streamed column DMA (measured: config-2
                              // k_scan_query 0.733 -> 0.702 ms)
  bool use_pipe = false;      // exec.pipe: double-buffered whole-chunk staging (k_scan_query_pipe) when a chunk fits
  bool timing = false;
  std::string group_mode;     // group.mode: "" (auto) | lds | global | partition (tests force a sink)
  bool use_plan_cache = true;  // plan.cache: a repeated fused aggregation reuses its host plan
  std::shared_ptr<void> fused_plan;  // executor.cpp FusedPlan of the last fused aggregation
  uint64_t config_epoch = 0;  // bumped by every configuration change (plan cache key)
  bool sync_flag = true;      // sync.flag: fused aggregation waits on its kernel's mapped completion flag
  uint32_t fused_seq = 0;     // last completion sequence number handed to k_scan_query
  int64_t wall_clock_khz = 100000;  // hipDeviceAttributeWallClockRate (device-side kernel timing)
  bool sync_poll = false;     // sync.poll: busy-poll the stream instead of hipStreamSynchronize
  bool host_phases = false;
  int group_nt_store = 0;     // group.nt_store: partitioned records stored non-temporally
  bool group_prefetch = true; // group.prefetch: partitioned plan loads every column of a word batch at once
  int group_pshift = -1;      // group.pshift: cap on log2 keys per partition (tests: many small partitions)
  int group_split = -1;       // group.split: log2 sub-partitions per emitted run (-1 auto, 0 single-level)
  bool use_shortcut_plans = true;  // plan.shortcut: metadata / dictionary plans for unfiltered COUNT / MIN / MAX
  int group_emit_block = 512;  // group.emit_block: 512 | 1024 threads per bucketed lane-owns-quarter EMIT block
  int group_lds_block = 512;   // group.lds_block: 256 | 512 threads per lane-owns-quarter GB_LDS block
  bool group_aligned = false; // group.aligned: bucketed EMIT runs padded to 64-B buckets (measured: EMIT -1.6%, reduce slower)
  int group_lw = 2;           // group.lw: partitioned plan reads 0 per doc, 1 each lane's 64-doc word, 2 contiguous quarters
  bool group_bucket = true;   // group.bucket: partitioned plan EMITs through LDS buckets into the final layout
  bool group_ring = true;     // group.ring: large dense key spaces take the ring plan (no histogram pass; group_ring.hip);
                              // 0: the counted plan (COUNT -> scan -> EMIT2 -> k_partition_reduce)
  bool raw_device = true;     // raw.device: raw numeric columns transcoded on the device at registration (transcode.h)
  int64_t raw_device_columns = 0;  // columns the device transcoded
  int64_t raw_host_fallbacks = 0;  // raw numeric columns transcoded on the host for want of free HBM
  bool group_lds_qfilter = false;  // group.lds_qfilter: the LDS group-by evaluates a one-leaf filter per quarter
                                   // (measured slower than the staged chunk filter: 1.47 vs 1.15 ms, off by default)
  bool group_ring_hll = true;      // group.ring_hll: the ring scatter computes HLL (register, rank) fields (affine columns)
  bool group_ring_rec6 = false;    // group.ring_rec6: 6-byte ring records when the fields fit 48 bits (measured slower)
  bool group_ring_qfilter = true;  // group.ring_qfilter: the ring kernel evaluates simple filters itself (else GB_FILTER)
  int32_t trim_top_n = 0;      // per call (pinot_gpu_group_by_top): trim the group-by on the device for this TOP n
  int64_t ring_queries = 0;    // group-bys launched on the ring plan
  int64_t last_group_instance = 0;  // the last fused group-by's main kernel instance (group.last_instance)
  int64_t last_pre_segments = 0;  // segments of the last fused query whose filter needed a `pre` bitset (launch sequence)
  int64_t ring_last_rec_bytes = 0;  // the last ring query's record bytes (6 / 8) and its scatter-side HLL field (0 / 1)
  int64_t ring_last_hll_slot = 0;
  int64_t ring_last_status = 0;   // the status bits that sent the last fallen-back ring query to the counted plan
  int64_t ring_qfilter_queries = 0;  // ... of them with the filter evaluated inside k_group_ring (no GB_FILTER pass)
  int64_t ring_fallbacks = 0;  // ring-plan queries re-answered on the counted plan (a region overflowed: skewed keys)
  int num_cus = 256;          // multiProcessorCount of the device

  // scratch (grow-only)
  DeviceBuffer bitsets;       // filter bitset slots (slot 0 = final)
  DeviceBuffer small;         // per-query arena: ranges, ids, LUTs
  DeviceBuffer partials;      // per-block partial slots
  DeviceBuffer reduced;       // per-segment reduced slots + HLL registers
  DeviceBuffer group_scratch;  // dense group-by accumulators (+ per-segment matched counts)
  DeviceBuffer group_part;     // partitioned plan: histogram, offsets, partition starts, scan temp
  DeviceBuffer group_records;  // partitioned plan: (local key | dictIds) records, partition-major
  DeviceBuffer group_runs;     // two-level plan: the same records in coarse (run, block) order
  DeviceBuffer group_filter;   // bucketed plan: the COUNT pass's filter words per segment (read back by GB_EMIT2)
  DeviceBuffer group_final;    // ordered non-empty keys + compaction scratch
  DeviceBuffer group_out;      // per-group outputs (counts, accumulators, HLL sums, keys) for the D2H
  DeviceBuffer group_gather;   // multi-GPU root: every rank's per-group outputs, gathered
  PinnedBuffer group_host;     // their pinned host copy
  std::vector<std::shared_ptr<DeviceBuffer>> hll_pool;  // gathered HLL registers, reused once results are released
  std::shared_ptr<DeviceBuffer> hll_ser;  // HyperLogLog.getBytes rows of a device-trimmed result (copied back at once)
  DeviceBuffer group_trim;     // device trim: union keys, per-group function bits, sort / scan scratch
  DeviceBuffer group_hash;     // hashed key spaces: fingerprint table + representative docs
  DeviceBuffer group_admit;    // num.groups.limit admission: first docs [S][G], admitted bitmaps [S][G/32], sort scratch
  PinnedBuffer host_arena;    // staging of the per-query arena (H2D)
  std::vector<uint8_t> arena_shadow;  // bytes last copied into `small` (upload_arena skips identical programs)
  uint64_t arena_dev_gen = 0;
  bool arena_dev_valid = false;
  PinnedBuffer host_result;   // staging of the reduced results (D2H)
  PinnedBuffer d2h_small;     // pinned landing of the group-by's small status reads (a pageable target makes each copy
                              // a staged, synchronous one: ~20-35 us apiece)
  DeviceBuffer fused_ctl;     // k_scan_query: u32 arrival counter + [kMaxHll][256] HLL registers, kept zeroed
  MappedBuffer fused_result;  // k_scan_query's last block writes the reduced per-segment slots + HLL here

  // per-call query budget (pinot_query.timeout_ms): waits on the stream give up at the deadline
  bool has_deadline = false;
  std::chrono::steady_clock::time_point deadline;

  // timing
  hipEvent_t ev_start = nullptr, ev_stop = nullptr;
  DeviceBuffer hll_linear;    // device copy of hll_linear_counting_table() (k_group_final)
  std::vector<hipEvent_t> kev;  // per-kernel event pairs (timing mode)
  double last_ms[2] = {0, 0};
  int64_t last_launches[2] = {0, 0};

  ~Engine();
  SegmentData &seg(int64_t h);
};

// Deadline of a query call (ServerQueryExecutorV1Impl.java:113-126: remaining = timeout - scheduling wait).
void check_deadline(const Engine &e, const char *phase);
struct DeadlineScope {
  Engine &e;
  DeadlineScope(Engine &en, int32_t timeout_ms);
  ~DeadlineScope() { e.has_deadline = false; }
};

// execution entry points (executor.cpp)
void exec_filter(Engine &e, SegmentData &s, const FilterTreeInput *tree, uint64_t *bitset_out, int64_t *count);
// numEntriesScannedInFilter of one segment as the reference's iterator protocol counts it (filter_stats.cpp;
// stats.exact=1)
int64_t filter_entries_scanned(Engine &e, SegmentData &s, const FilterTreeInput *tree);
void exec_aggregate(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q, pinot_agg_result *out,
                    pinot_exec_stats *stats);

struct HllPart {
  int device = 0;
  std::shared_ptr<DeviceBuffer> buf;
  std::vector<size_t> off;        // per fn: byte offset of its [num_groups][256] registers
  int64_t group_begin = 0, num_groups = 0;
};

// The non-empty groups of a key range on the device, array-major, as the host result will hold them (the output of
// the owner finalize before its D2H; what a multi-GPU group-by gathers to its root rank). Per function fn: values[fn]
// (nullptr-free; read back only where derive[fn] == -1), cards[fn] (kind 4), HLL registers [n][256] at hll_off[fn].
struct DenseOut {
  unsigned long long n = 0;
  std::vector<int> kind;            // accumulator kind per fn
  std::vector<int> derive;          // -1: read back; -2: from the HLL cardinalities; >= 0: copy of that fn's values
  long long *keys = nullptr, *counts = nullptr;
  std::vector<double *> values;
  std::vector<long long *> cards;
  std::shared_ptr<DeviceBuffer> hll;
  std::vector<size_t> hll_off;
  // device-trimmed results: each HLL function's HyperLogLog.getBytes rows ([n][180] B, hll_serde.hip) in hll_ser at
  // hll_ser_off[fn], copied back with the other arrays
  std::shared_ptr<DeviceBuffer> hll_ser;
  std::vector<size_t> hll_ser_off;
  int32_t *key_ids = nullptr;       // device-trimmed results: [n][gcols] global ids of each kept key (trim.h)
  // compact read-back (dense, non-hashed key spaces of >= 64 K groups): the non-empty keys as a bitmap over [0, G),
  // counts and HLL cardinalities as u32 (overflow flag -> the 64-bit arrays), widened on the host
  const uint64_t *key_bits = nullptr;
  int64_t key_words = 0;
  long long key_base = 0;
  unsigned int *counts32 = nullptr;
  std::vector<unsigned int *> cards32;
  unsigned int *overflow = nullptr;
};

// The single-value function whose intermediate result / merge / final result a multi-value function shares
// (CountMVAggregationFunction extends CountAggregationFunction, etc.).
inline int sv_function(int f) { return f >= PINOT_AGG_COUNTMV && f <= PINOT_AGG_DISTINCTCOUNTHLLMV ? f - PINOT_AGG_COUNTMV : f; }

// A pinned host vector whose resize leaves new elements uninitialised (a D2H copy fills them: no zero pass over
// megabytes first).
template <typename T>
struct PinnedNoInitAllocator : PinnedAllocator<T> {
  template <typename U>
  struct rebind {
    using other = PinnedNoInitAllocator<U>;
  };
  PinnedNoInitAllocator() = default;
  template <typename U>
  PinnedNoInitAllocator(const PinnedNoInitAllocator<U> &) {}
  template <typename U>
  void construct(U *p) noexcept {
    ::new (static_cast<void *>(p)) U;
  }
  template <typename U, typename... A>
  void construct(U *p, A &&...a) {
    ::new (static_cast<void *>(p)) U(std::forward<A>(a)...);
  }
};
template <typename T>
using HostVecNoInit = std::vector<T, PinnedNoInitAllocator<T>>;

struct GroupByResult {
  GroupByResult() = default;
  GroupByResult(GroupByResult &&) = default;
  GroupByResult &operator=(GroupByResult &&) = default;
  ~GroupByResult();  // returns its large result arrays to a process-wide pool (no page faults on the next query)
  HostVec<int64_t> raw_keys;                  // ascending raw keys (mixed radix over global ids, column 0 least significant)
  int32_t num_columns = 0;
  std::vector<int> functions;
  std::vector<HostVec<int64_t>> counts;       // per fn (counts_shared: one vector, counts[0], for every fn)
  bool counts_shared = false;
  std::vector<HostVec<double>> values;        // per fn
  // group key strings ('\t'-joined Dictionary.getStringValue), built on first access
  std::vector<std::vector<std::string>> gvalues;  // [gcol] global id -> string
  std::vector<int64_t> gcard;
  std::vector<int32_t> key_ids;               // hashed key spaces: [groups][gcols] global ids
  mutable std::vector<std::string> keys;
  mutable std::vector<uint8_t> key_built;
  const std::string &key(int64_t g) const;
  // all key strings back to back (offsets[n + 1]); built in parallel on first use
  mutable std::vector<int64_t> key_offsets;
  uint64_t export_keys(char *buf, uint64_t buf_len, int64_t *offsets) const;
  // AggregationGroupByTrimmingService: the groups of function fn's trimmed map (ascending)
  std::vector<int64_t> trim(int32_t top_n, int32_t fn) const;
  // trimmed on the device (pinot_gpu_group_by_top): the result holds the union of the functions' trimmed maps and
  // fn_kept[fn] lists fn's groups; 0 = not trimmed (every group)
  int32_t trimmed_top_n = 0;
  int64_t merged_groups = -1;  // groups of the merged map before a device trim (-1: raw_keys.size())
  std::vector<std::vector<int64_t>> fn_kept;
  // DISTINCTCOUNTHLL: cardinalities per fn; registers on the host (hll[fn]) or on the device in parts (one per
  // GPU that finalized a key range: [groups][256] u8 at off[fn], copied on request)
  std::vector<HostVec<int64_t>> hll_card;
  std::vector<std::vector<uint8_t>> hll;
  std::vector<HllPart> hll_parts;
  // device-trimmed results (pinot_gpu_group_by_top): per HLL function its groups' HyperLogLog.getBytes, [n][180] B
  // (empty: not prepared; the DataTable writer then packs the registers itself)
  std::vector<HostVecNoInit<uint8_t>> hll_bytes;
  // pinot_datatable_group_by's bytes, one buffer per call: every pointer handed out stays valid until the result is
  // freed (a caller may hold a zero-copy view of an earlier call's bytes)
  mutable std::deque<std::vector<uint8_t>> datatables;
};
// all groups' u8 HLL registers of function fn ([groups][256]) into host memory, from the device parts or the host copy
void group_by_hll_registers(const GroupByResult &r, int fn, uint8_t *registers, bool pinned_dst = false);
// Host task pool (executor.cpp): pause instructions its threads spin after a job before sleeping (engine key host.spin).
void set_host_spin(int pauses);

// DataTable bytes (datatable.cpp)
std::vector<uint8_t> aggregation_datatable(const pinot_query &q, const pinot_agg_result *r, const pinot_exec_stats &s,
                                           const pinot_datatable_server *srv);
std::vector<uint8_t> group_by_datatable(const pinot_query &q, const GroupByResult &r, const int64_t *const *fn_groups,
                                        const int64_t *fn_num_groups, const pinot_exec_stats &s,
                                        const pinot_datatable_server *srv);
// DataTableBuilder.buildEmptyDataTable + the metadata processQuery puts on it when every segment was pruned
std::vector<uint8_t> empty_datatable(const pinot_query &q, int64_t total_docs, const pinot_datatable_server *srv);
// BrokerReduceService over the servers' DataTable bytes -> BrokerResponseNative JSON (broker.cpp)
std::string broker_reduce(const pinot_query &q, int32_t n, const uint8_t *const *tables, const uint64_t *lens,
                          int32_t top_n);
std::unique_ptr<GroupByResult> exec_group_by(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q,
                                             pinot_exec_stats *stats);

// multi-GPU partials
void exec_group_by_layout(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q,
                          pinot_partial_layout *layout);
void exec_group_by_partial(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q,
                           int64_t *counts_dev, void *const *accs_dev, pinot_exec_stats *stats);
std::unique_ptr<GroupByResult> exec_group_by_finalize(Engine &e, const std::vector<SegmentData *> &segs,
                                                      const pinot_query &q, const int64_t *counts_dev,
                                                      void *const *accs_dev);

// segments (segment.cpp)
std::unique_ptr<SegmentData> register_segment(Engine &e, const pinot_segment_desc &d);
// Star-tree v2 (startree.cpp): attach (parse + check + register the star docs), fit test, traversal.
void attach_star_tree(Engine &e, SegmentData &seg, const pinot_star_tree_desc &d);
bool star_tree_fits(const SegmentData &seg, const pinot_query &q);
bool star_plan_fits(const Engine &e, const SegmentData &seg, const pinot_query &q);  // startree.use && the tree fits
std::string star_pair_column(const pinot_agg_spec &a);  // "count__*", "sum__x", ... ("" when no pair exists)
struct StarMatch {
  bool empty = false;                  // a predicate matches nothing
  std::vector<uint64_t> bits;          // matched star docs
  int64_t docs = 0;
  int64_t entries_in_filter = 0;       // remaining predicates' scanned entries (applyAnd over the bitmap answer)
};
StarMatch star_tree_match(const SegmentData &seg, const pinot_query &q, const FilterTreeInput *tree);
std::unique_ptr<SegmentData> register_synthetic(Engine &e, const char *name, int32_t num_docs, int32_t ncols,
                                                const char *const *names, const int32_t *cards, uint64_t seed,
                                                const int32_t *kinds = nullptr);
void ensure_hll_lut(Engine &e, ColumnData &c);

// stream-lib HyperLogLog(log2m=8) helpers (hll.cpp)
uint32_t murmur_hash_long(int64_t v);
uint32_t murmur_hash_bytes(const uint8_t *data, int len);
uint16_t hll_register_rank(uint32_t h);  // (register << 8) | rank
int64_t hll_cardinality(const uint8_t *regs);
// HyperLogLog.cardinality() from the exact register sum Σ 2^(32 - reg) and the zero-register count.
int64_t hll_cardinality_from_sum(unsigned long long sum_fixed32, uint32_t zeros);
const double *hll_linear_counting_table();  // [257]: m * log(m / z), z = 0 -> +inf
double hll_alpha_mm();

// ------------------------------------------------------------------ multi-GPU server (server.cpp)
// One engine per local GPU + RCCL communicators created once (ncclCommInitAll over the local devices, or one
// rank of a multi-process communicator: ncclCommInitRank). Queries over segments of several engines run each
// engine's part concurrently and merge on the device: reduce-scatter of the dense group-by partials, owner
// finalize per key range (CombineGroupByOperator.java:104-228), host merge (single process) or an all-reduce
// (multi process) of aggregation partials (CombineOperator.java:75-196).
struct ServerImpl;
struct SegmentRef {
  int engine;
  int64_t handle;
};
ServerImpl *server_create(const int32_t *devices, int32_t n, const char *config);
ServerImpl *server_create_rank(int32_t device, int32_t nranks, int32_t rank, const uint8_t *id,
                             const char *config);
void server_unique_id(uint8_t *id);
void server_destroy(ServerImpl *s);
constexpr int kServerPhases = 8;
void server_last_phases(const ServerImpl &s, double *ms, int n);
int server_num_engines(const ServerImpl &s);
Engine *server_engine(ServerImpl &s, int i);
void server_aggregate(ServerImpl &s, const std::vector<SegmentRef> &refs, const pinot_query &q, pinot_agg_result *out,
                      pinot_exec_stats *stats);
// top_n > 0: the server's trimmed answer (pinot_gpu_server_group_by_top)
std::unique_ptr<GroupByResult> server_group_by(ServerImpl &s, const std::vector<SegmentRef> &refs, const pinot_query &q,
                                               pinot_exec_stats *stats, int32_t top_n = 0);

// the multi-device partial step of one engine (executor.cpp): dense partials over [0, G) of the given key space
// into counts / accs (allow_admission: per-segment num.groups.limit admission inside the partial, when the caller
// has established that the inter-segment cap cannot bind)
// The server's num.groups.limit inter-segment cap across ranks (CombineGroupByOperator.java:80,147 over every rank's
// segments): mode 1 exports each local segment's first-appearance admitted keys ([segments][words] u32 bitmaps over
// the global key space, DictionaryBasedGroupKeyGenerator's per-segment holder rule applied, no cap) and runs no
// group-by; mode 2 imports the capped bitmaps and runs the partial with them.
struct AdmissionIO {
  int mode = 0;
  int64_t words = 0;
  std::vector<uint32_t> bitmaps;
};
void exec_group_by_partial_ks(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q,
                              const std::vector<int64_t> &gcard, const std::vector<std::vector<std::string>> &gvalues,
                              const std::vector<std::vector<std::vector<int32_t>>> &remap, int64_t *counts_dev,
                              void *const *accs_dev, pinot_exec_stats *stats, AdmissionIO *aio = nullptr,
                              bool hll_sum_room = false, bool *hll_sums_written = nullptr);
// (hll_sum_room: each HLL array holds u64 [G] after its registers, where the ring plan leaves the packed register
// sums — set in *hll_sums_written — so a one-rank owner finalize reads cardinalities without the registers)
// CombineGroupByOperator's cap over [S][words] admitted bitmaps in segment order: keys enter until `cap` are in
void inter_segment_cap(std::vector<uint32_t> &bm, size_t S, int64_t words, int64_t cap);
// Multi-value group-by (MV group columns or *MV functions): the extended function list (a hidden CountMV after the
// functions for every AvgMV, whose entry count it carries), and the fold of those counts into the final result.
std::vector<pinot_agg_spec> mv_extended_specs(const pinot_query &q, std::vector<int> &hidden);
void fold_mv_counts(GroupByResult &res, const pinot_query &q, const std::vector<int> &hidden);
bool touches_mv_group_by(const std::vector<SegmentData *> &segs, const pinot_query &q);
struct MvPartial {  // the server's MV partial step: global key space, its dense arrays (extended function list)
  const std::vector<int64_t> *gcard;
  const std::vector<std::vector<std::string>> *gvalues;
  const std::vector<std::vector<std::vector<int32_t>>> *remap;
  int64_t *counts;
  void *const *accs;
  AdmissionIO *aio;
};
void exec_group_by_mv_partial(Engine &e, const std::vector<SegmentData *> &segs, const pinot_query &q,
                              const MvPartial &mp, pinot_exec_stats *stats);
// owner finalize of one key range [key_base, key_base + G) of merged dense arrays, device half: ordered compaction
// of the non-empty keys (one sync for their count) and the group outputs on the device
DenseOut slice_outputs(Engine &e, const pinot_query &q, const std::vector<int> &acc_kind, unsigned long long *counts,
                       const std::vector<void *> &accs, int64_t G, int64_t key_base);
// slice_outputs in two halves (a server's trimmed answer all-gathers the ranges' group counts between them): the
// range's ordered non-empty keys (device) and their count, then the outputs of those keys — top_n > 0: of the range's
// trimSize best groups per function only (AggregationGroupByTrimmingService, every group when the range holds no
// more), with each kept group's mask of the functions that keep it in `flags`. gcard (the whole key space's, the
// range being all of it): the DataTable's per-column ids and serialized HLLs made on the device as the engine's own
// result has them; hll_sum: per aggregation, the ring plan's packed register sums (or null)
unsigned long long slice_compact(Engine &e, const unsigned long long *counts, int64_t G, long long *&keys_dev);
DenseOut slice_outputs_keys(Engine &e, const pinot_query &q, const std::vector<int> &acc_kind, unsigned long long *counts,
                            const std::vector<void *> &accs, int64_t G, int64_t key_base, const long long *keys_dev,
                            unsigned long long n, int32_t top_n, std::vector<uint32_t> &flags,
                            const std::vector<int64_t> *gcard = nullptr, const std::vector<const void *> *hll_sum = nullptr);
// The server trim over the ranges' candidates (flags: per gathered group, the functions whose range trim kept it):
// each function keeps its trimSize best candidates — the merged map's trimSize best, as every group's range kept the
// range's best — and the result becomes a device-trimmed one (fn_kept, trimmed_top_n, merged_groups).
void server_trim_select(GroupByResult &r, int32_t top_n, const std::vector<uint32_t> &flags, int64_t merged_groups);
// the device arrays of n gathered groups, in e's gather buffers, laid out as slice_outputs lays them out
DenseOut slice_alloc(Engine &e, const pinot_query &q, const std::vector<int> &acc_kind, unsigned long long n);
// rank 0's gathered trimmed answer, after the gather on the same stream: the DataTable's per-column ids and serialized
// HLLs on the device, as dense_outputs makes them for a one-GPU trimmed result
void slice_serialize(Engine &e, const pinot_query &q, const std::vector<int64_t> &gcard, DenseOut &o);
// the gatherable arrays of a DenseOut in a fixed order: (device pointer, bytes per group)
std::vector<std::pair<void *, size_t>> slice_arrays(const DenseOut &o);
// host half: the D2H into a result
std::unique_ptr<GroupByResult> slice_result(Engine &e, const pinot_query &q, const std::vector<int64_t> &gcard,
                                            const std::vector<std::vector<std::string>> &gvalues, const DenseOut &o);
// The multi-GPU group-by key space. Each rank serializes, per group-by column, the union of its segments'
// dictionary values (sorted, unique; an empty list of unknown type for a rank without segments); every rank merges
// all ranks' lists into the same global dictionaries: global id = rank of the value in the union (value order:
// integers, doubles by Double.compare, strings by bytes), and each local segment gets a dictId -> global id remap
// (empty where its dictionary IS the union). The reference merges by string key instead because dictionaries
// differ per segment (CombineGroupByOperator.java:142-161).
std::vector<uint8_t> local_group_dictionaries(const std::vector<SegmentData *> &segs, const pinot_query &q);
struct GlobalKeySpace {
  std::vector<int64_t> gcard;
  std::vector<std::vector<std::string>> gvalues;
  std::vector<std::vector<std::vector<int32_t>>> remap;  // [local segment][gcol]
  int64_t G = 1;
  bool hashed = false;  // Π cardinalities beyond the dense limit
  uint64_t fingerprint = 0;
};
GlobalKeySpace global_key_space(const std::vector<SegmentData *> &segs, const pinot_query &q,
                                const std::vector<std::vector<uint8_t>> &rank_dicts);
std::vector<int> group_acc_kind_list(const SegmentData &s, const pinot_query &q);
bool admission_cap_can_bind(const std::vector<SegmentData *> &segs, const pinot_query &q, const Engine &e, int64_t G);
uint64_t dictionary_fingerprint(const ColumnData &c);
// SegmentPrunerService over one call's segments with the query's pruners (pinot_query.pruners; 0: all kept)
std::vector<SegmentData *> prune_for_query(const std::vector<SegmentData *> &segs, const pinot_query &q);
// the aggregation result of no segment (identities: MIN +inf, MAX -inf, exact zero sums, zero HLL registers)
void agg_identities(const pinot_query &q, pinot_agg_result *out);
// the group-by result of no segment (no group)
std::unique_ptr<GroupByResult> empty_group_result(const pinot_query &q);
// keys the num.groups.limit admission can let in over these segments (the 2 x limit inter-segment cap binds when
// the total over every GPU's segments exceeds it)
int64_t admission_possible(const std::vector<SegmentData *> &segs, const pinot_query &q, const Engine &e);
// Math.min / Math.max (NaN wins, -0.0 < 0.0)
inline double java_min(double a, double b) {
  if (a != a) return a;
  if (b != b) return b;
  if (a == 0.0 && b == 0.0) return std::signbit(a) ? a : b;
  return a < b ? a : b;
}
inline double java_max(double a, double b) {
  if (a != a) return a;
  if (b != b) return b;
  if (a == 0.0 && b == 0.0) return std::signbit(a) ? b : a;
  return a > b ? a : b;
}
// CombineService.mergeTwoBlocks over per-engine aggregation results (host)
void merge_agg_parts(const pinot_query &q, const std::vector<const pinot_agg_result *> &parts, pinot_agg_result *out);

}  // namespace pinot

struct pinot_engine : pinot::Engine {};
struct pinot_groupby_result : pinot::GroupByResult {};

namespace pinot {
std::unique_ptr<pinot_engine> create_engine(int32_t device, const char *config);
}  // namespace pinot
