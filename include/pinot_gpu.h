/*
 * pinot_gpu.h — C-ABI of the MI355X-native Pinot segment query executor.
 *
 * This is the drop-in boundary between Pinot's Java operator layer and the
 * HIP/CDNA4 kernels. A JNI shim binds these symbols; the
 * tests and bench bind them through ctypes. No C++/torch types cross the ABI:
 * plain structs, pointers and sizes only. Every entry point returns a
 * pinot_status (0 = ok); on failure pinot_gpu_last_error() holds a thread-local
 * message. Nothing aborts across the ABI.
 *
 * Reference interfaces replaced (PC = pinot-core/src/main/java/org/apache/pinot/core):
 *   pinot_gpu_engine_create / destroy   QueryExecutor.init/start/shutDown   (PC/query/executor/QueryExecutor.java:32-62)
 *   pinot_gpu_segment_register          ImmutableSegmentLoader.load + PhysicalColumnIndexContainer
 *                                       (PC/indexsegment/immutable/ImmutableSegmentLoader.java:59-153,
 *                                        PC/segment/index/column/PhysicalColumnIndexContainer.java:63-121)
 *   pinot_gpu_segment_release           SegmentDataManager release / IndexSegment.destroy
 *                                       (ServerQueryExecutorV1Impl.java:231-233)
 *   pinot_gpu_filter                    BaseFilterOperator.nextBlock().getBlockDocIdSet()
 *                                       (PC/plan/FilterPlanNode.java:70-126, PC/operator/filter/)
 *   pinot_gpu_aggregate                 AggregationOperator + CombineOperator
 *                                       (PC/operator/query/AggregationOperator.java:56-82,
 *                                        PC/operator/CombineOperator.java:75-196)
 *   pinot_gpu_group_by                  AggregationGroupByOperator + CombineGroupByOperator
 *                                       (PC/operator/query/AggregationGroupByOperator.java:64-94,
 *                                        PC/operator/CombineGroupByOperator.java:104-228)
 *   pinot_gpu_prune_segments            ServerQueryExecutorV1Impl.pruneSegments + SegmentPrunerService.prune
 *                                       (PC/query/executor/ServerQueryExecutorV1Impl.java:183-216, :270-294,
 *                                        PC/query/pruner/SegmentPrunerService.java:52-60)
 *   pinot_broker_reduce                 BrokerReduceService.reduceOnDataTable (PC/query/reduce/BrokerReduceService.java:69-530)
 *   pinot_datatable_*                   IntermediateResultsBlock.getDataTable / DataTableBuilder.buildEmptyDataTable
 *                                       (PC/operator/blocks/IntermediateResultsBlock.java:206-317,
 *                                        PC/common/datatable/DataTableBuilder.java:292-370)
 */
#ifndef PINOT_GPU_H_
#define PINOT_GPU_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PINOT_GPU_ABI_VERSION 14

/* ------------------------------------------------------------------ status */
typedef enum {
  PINOT_OK = 0,
  PINOT_ERR_BAD_ARG = 1,      /* malformed descriptor / query (maps to QueryException.QUERY_EXECUTION_ERROR) */
  PINOT_ERR_OOM = 2,          /* HBM allocation failed: caller falls back to the CPU operator */
  PINOT_ERR_DEVICE = 3,       /* HIP runtime / kernel error */
  PINOT_ERR_UNSUPPORTED = 4,  /* query shape not handled on the GPU: caller falls back */
  PINOT_ERR_BAD_QUERY = 5,    /* bad literal, unknown column (BadQueryRequestException) */
  PINOT_ERR_TIMEOUT = 6       /* query budget exhausted: QUERY_SCHEDULING_TIMEOUT_ERROR when it was spent before
                                 the call (ServerQueryExecutorV1Impl.java:116-126), else the combine timeout
                                 (CombineGroupByOperator.java:174-181); device work already queued still drains */
} pinot_status;

/* ------------------------------------------------------------------ segment */
typedef enum {
  PINOT_INT = 0, PINOT_LONG = 1, PINOT_FLOAT = 2, PINOT_DOUBLE = 3, PINOT_STRING = 4
} pinot_data_type;

/* Raw (no-dictionary) numeric columns are transcoded once at registration: the sorted distinct values become the
 * dictionary and every doc's dictId is fixed-bit packed, so the device path reads one format. Predicates, MIN / MAX
 * and SUM give the reference's raw-value results (RawValueBased*PredicateEvaluator) except for signed zeros and NaN
 * in FLOAT / DOUBLE columns, which a dictionary keeps apart / orders last. The dictionary-based MIN / MAX plan is
 * not used for them (InstancePlanMakerImplV2 requires a dictionary). Raw STRING (var-byte) columns are transcoded to
 * a dictionary sorted in UTF-8 byte order (String.compareTo's order for text without supplementary characters). */
typedef enum { PINOT_ENCODING_DICTIONARY = 0, PINOT_ENCODING_RAW = 1 } pinot_column_encoding;

/* One single-value dictionary-encoded column, exactly as the segment files hold it
 * (all multi-byte fields big-endian, as PinotDataBuffer serves them). Host pointers are
 * only read during pinot_gpu_segment_register; nothing is retained. */
typedef struct {
  const char *name;
  int32_t data_type;           /* pinot_data_type */
  int32_t cardinality;         /* dictionary length */
  int32_t bits_per_value;      /* PinotDataBitSet.getNumBitsPerValue(card - 1) */
  int32_t is_sorted;           /* sorted column: sorted_index present, forward_index absent */
  int32_t has_inverted_index;  /* bitmap inverted index present (unsorted columns) */
  int32_t string_width;        /* STRING dictionary: bytes per padded value */
  int32_t padding_byte;        /* STRING dictionary padding (segment.padding.character; '%' on legacy segments,
                                  ColumnMetadata.java:111-115): values end at the first such byte, and a non-zero
                                  padding compares predicate values padded (ImmutableDictionaryReader.java:152-180) */
  int32_t encoding;            /* PINOT_ENCODING_DICTIONARY (0) or PINOT_ENCODING_RAW (1): a no-dictionary column
                                  (PhysicalColumnIndexContainer.java:101-106); forward_index then holds the N values
                                  themselves, BE fixed width (INT / FLOAT 4 bytes, LONG / DOUBLE 8), as the
                                  decompressed chunks of FixedByteChunkSingleValueReader hold them; STRING: N + 1
                                  BE int32 offsets then the UTF-8 bytes (value i = bytes [off[i], off[i+1]), offsets
                                  counted from the first byte after the offsets; what VarByteChunkSingleValueReader
                                  .getBytes returns per doc); cardinality, bits_per_value, dictionary and the
                                  indexes are ignored (0 / NULL). */
  const uint8_t *dictionary;   uint64_t dictionary_len;     /* card * width BE values */
  const uint8_t *forward_index; uint64_t forward_index_len; /* ceil(N*b/8) bytes, MSB-first */
  const uint8_t *sorted_index; uint64_t sorted_index_len;   /* 2*card BE int32 [start,end] */
  const uint8_t *inverted_index; uint64_t inverted_index_len; /* (card+1) BE int32 offsets + portable roaring */
  /* column.<c>.minValue / maxValue as the segment metadata holds them (ColumnMetadata.java:155-156; NULL = absent,
     as in segments whose loader did not generate them: ColumnMinMaxValueGenerator, default mode TIME). Read only by
     the segment pruner; parsed with the column's data type. */
  const char *min_value;
  const char *max_value;
  /* Bloom filter (ABI >= 8): the column's .bloom bytes as BloomFilterReader reads them (BE int type = 1, BE int
     version = 1, then Guava's BloomFilter.writeTo: byte strategy, byte numHashFunctions, BE int words, BE longs;
     BloomFilterReader.java:36-50), or create_bloom_filter = 1 to build it at registration from the dictionary as
     BloomFilterHandler does at load (BloomFilterHandler.java:107-116; dictionary columns only). Read only by the
     COLUMN_VALUE pruner's EQUALITY test (ColumnValueSegmentPruner.java:140-144). */
  const uint8_t *bloom_filter; uint64_t bloom_filter_len;
  int32_t create_bloom_filter;
  /* Partition metadata (ABI >= 8; column.<c>.partitionFunction / numPartitions / partitionValues,
     ColumnMetadata.java:184-194): function name (Modulo / Murmur / ByteArray / HashCode, any case; NULL = none), the
     partition count and the partitions this segment holds (ranges already expanded,
     ColumnPartitionMetadata.extractPartitions), or num_partition_values = -1 to take the partitions of every dictionary
     value, as the segment creator records them. Read only by the PARTITION pruner. */
  int32_t num_partitions;
  const char *partition_function;
  const int32_t *partition_values; int32_t num_partition_values;
  /* Multi-value columns (ABI >= 9; column.<c>.isSingleValues = false): forward_index then holds the
     FixedBitMultiValueReader layout (PC/io/reader/impl/v1/FixedBitMultiValueReader.java:30-74): BE int chunk offsets
     (one per ceil(2048 / (entries / rows)) rows), a bitmap of entries marking each row's first value (MSB first),
     then the entries' dictIds fixed-bit packed. total_number_of_entries / max_number_of_multi_values are the
     metadata's totalNumberOfEntries / maxNumberOfMultiValues. Dictionary columns only; never sorted. */
  int32_t multi_value;
  int32_t max_number_of_multi_values;
  int64_t total_number_of_entries;
} pinot_column_desc;

typedef struct {
  const char *name;
  int32_t num_docs;            /* totalRawDocs, < 2^31 */
  int32_t num_columns;
  const pinot_column_desc *columns;
} pinot_segment_desc;

typedef struct pinot_engine pinot_engine;   /* one per GPU (HIP device) */
typedef int64_t pinot_segment_handle;

/* ------------------------------------------------------------------ query */
/* Filter tree as Thrift FilterQuery nodes in POSTFIX order: leaves carry the
 * operator, column and value strings exactly as the PQL compiler emits them
 * (RANGE: one "(lo\t\thi]" string; IN/NOT_IN: values, or one "\t\t"-joined string). */
typedef enum {
  PINOT_FILTER_AND = 0, PINOT_FILTER_OR = 1,
  PINOT_FILTER_EQUALITY = 2, PINOT_FILTER_NOT = 3, PINOT_FILTER_RANGE = 4,
  PINOT_FILTER_IN = 5, PINOT_FILTER_NOT_IN = 6
} pinot_filter_op;

typedef struct {
  int32_t op;                  /* pinot_filter_op */
  int32_t num_children;        /* AND/OR: number of immediately preceding subtrees */
  const char *column;          /* leaf only */
  int32_t num_values;          /* leaf only */
  const char *const *values;   /* leaf only */
} pinot_filter_node;

typedef enum {
  PINOT_AGG_COUNT = 0, PINOT_AGG_SUM = 1, PINOT_AGG_MIN = 2, PINOT_AGG_MAX = 3,
  PINOT_AGG_AVG = 4, PINOT_AGG_DISTINCTCOUNTHLL = 5,
  /* multi-value variants (PC/query/aggregation/function/...MVAggregationFunction.java): over every entry of the
     matching docs' values; COUNTMV counts entries, AVGMV's count is entries */
  PINOT_AGG_COUNTMV = 6, PINOT_AGG_SUMMV = 7, PINOT_AGG_MINMV = 8, PINOT_AGG_MAXMV = 9,
  PINOT_AGG_AVGMV = 10, PINOT_AGG_DISTINCTCOUNTHLLMV = 11
} pinot_agg_function;

typedef struct {
  int32_t function;            /* pinot_agg_function */
  const char *column;          /* NULL or "*" for COUNT(*) */
} pinot_agg_spec;

typedef struct {
  int32_t num_filter_nodes;    /* 0 = no WHERE clause */
  const pinot_filter_node *filter;
  int32_t num_aggregations;
  const pinot_agg_spec *aggregations;
  int32_t num_group_by;        /* 0 = aggregation-only */
  const char *const *group_by;
  int32_t num_groups_limit;    /* num.groups.limit, default 100000 (InstancePlanMakerImplV2.java:55-58) */
  int32_t max_init_group_holder_capacity; /* array-holder threshold, default 10000 */
  int32_t timeout_ms;          /* remaining query budget = table timeout - scheduling wait
                                  (ServerQueryExecutorV1Impl.java:113-114); 0 = none, < 0 = already spent */
  int32_t pruners;             /* pinot_pruner bits: the query entry points (pinot_gpu_aggregate / _group_by and the
                                  server's) first drop the segments these pruners reject, as processQuery does
                                  (ServerQueryExecutorV1Impl.java:183-216): numSegmentsProcessed counts the rest,
                                  totalDocs every segment; every segment pruned gives the empty result (identities /
                                  no group). 0 = no pruning (ABI <= 6: the reserved field) */
} pinot_query;

/* Per-query statistics (ExecutionStatistics.java:35-43). num_entries_scanned_in_filter
 * is this engine's own count (every scan leaf reads every doc), not the reference's. */
typedef struct {
  int64_t num_docs_scanned;
  int64_t num_entries_scanned_in_filter;
  int64_t num_entries_scanned_post_filter;
  int64_t num_total_raw_docs;
  int64_t num_segments_processed;
  double device_ms;            /* HIP-event time of the device work of the call */
  double host_ms;              /* wall time from C-ABI entry to return (results on the host) */
  int64_t num_segments_matched; /* segments with at least one matching doc (ExecutionStatistics.java:42) */
} pinot_exec_stats;

/* Intermediate result of one aggregation function over a set of segments (already
 * combined, i.e. what CombineOperator hands to the DataTable):
 *   COUNT:  count
 *   SUM:    value (double, = Σ values; exact for integer columns below 2^53)
 *   MIN/MAX: value (+inf / -inf when no doc matched)
 *   AVG:    value = sum, count  (AvgPair)
 *   DISTINCTCOUNTHLL: hll_registers (merged), hll_cardinality = HyperLogLog.cardinality()
 * exact_sum / has_exact_sum: the int64 sum the device computed for INT columns. */
typedef struct {
  int64_t count;
  double value;
  int64_t exact_sum;
  int32_t has_exact_sum;
  int32_t reserved;
  int64_t hll_cardinality;
  uint8_t hll_registers[256];
} pinot_agg_result;

typedef struct pinot_groupby_result pinot_groupby_result;

/* ------------------------------------------------------------------ engine */
const char *pinot_gpu_last_error(void);
int32_t pinot_gpu_abi_version(void);
int32_t pinot_gpu_device_count(void);

/* config: "key=value;key=value" (keys: num.groups.limit, device.scratch.mb), may be NULL */
pinot_status pinot_gpu_engine_create(int32_t device, const char *config, pinot_engine **out);
pinot_status pinot_gpu_engine_destroy(pinot_engine *engine);
/* Change configuration keys at run time (e.g. "timing=1" to record per-kernel HIP events). Plan keys (defaults are
 * the measured-fastest plans; the others stay for experiments and parity tests): exec.fused, filter.force,
 * group.mode (lds | global | partition), group.ring (1: the ring-partitioned group-by plan), group.lds_block
 * (256 | 512), group.emit_block, stats.exact, startree.use; diagnostics: debug.host_phases (stderr phase times),
 * debug.ring (ring-kernel timing modes, wrong results). */
pinot_status pinot_gpu_engine_set_config(pinot_engine *engine, const char *config);

/* Copies the column buffers into HBM (one-time, cold path). */
pinot_status pinot_gpu_segment_register(pinot_engine *engine, const pinot_segment_desc *desc,
                                        pinot_segment_handle *out);
pinot_status pinot_gpu_segment_release(pinot_engine *engine, pinot_segment_handle handle);
/* ImmutableSegmentLoader.load (PC/indexsegment/immutable/ImmutableSegmentLoader.java:59-153) of a segment
 * directory as Pinot writes it: v1/v2 (one file per index) or v3 (v3/columns.psf + v3/index_map), metadata from
 * metadata.properties (SegmentMetadataImpl / ColumnMetadata; V1Constants.java:54-146). The files are memory-mapped,
 * checked like pinot_gpu_segment_register's descriptors and copied to HBM. Raw (no-dictionary) INT / LONG / FLOAT /
 * DOUBLE columns are read from their chunked .sv.raw.fwd index (PASS_THROUGH or Snappy chunks,
 * BaseChunkSingleValueReader.java:57-147), raw STRING columns from their var-byte chunks (.sv.raw.fwd,
 * VarByteChunkSingleValueReader.java:40-115), and registered as PINOT_ENCODING_RAW; multi-value dictionary columns
 * from <col>.mv.fwd (FixedBitMultiValueReader). Raw multi-value and BYTES columns are not served and are left out. */
pinot_status pinot_gpu_segment_load(pinot_engine *engine, const char *index_dir, pinot_segment_handle *out);
/* The engine's device segment cache (a server's SegmentDataManager map keyed by segment name, refreshed when the
 * segment's CRC changes: creation.meta's crc, SegmentMetadataImpl.java:204-210, V1Constants.java:27,97). A
 * directory whose segment name and CRC match a cached device copy returns that copy's handle (*cache_hit = 1; only
 * metadata.properties and creation.meta are read); otherwise the directory is loaded as pinot_gpu_segment_load does,
 * a cached copy of the same name with another CRC is released (the segment was replaced), and the new copy is
 * cached (*cache_hit = 0). A directory without creation.meta is loaded and never cached. Acquires are reference-counted
 * like SegmentDataManager.increaseReferenceCount / releaseSegment (BaseTableDataManager.java): every acquire of a
 * handle takes one reference, pinot_gpu_segment_release returns one, and the device copy is dropped when the last
 * reference returns. A replaced copy (new CRC) leaves the cache at once but stays valid for its holders until they
 * release it. */
pinot_status pinot_gpu_segment_acquire(pinot_engine *engine, const char *index_dir, pinot_segment_handle *out,
                                       int32_t *cache_hit);
/* The same read and checks on the host only (no engine, no GPU): docs, served columns, left-out columns. */
pinot_status pinot_gpu_segment_dir_info(const char *index_dir, int32_t *num_docs, int32_t *num_columns,
                                        int32_t *num_skipped);
/* A raw (no-dictionary) fixed-width forward index file's values, host only: FixedByteChunkSingleValueReader over the
 * file's bytes (BaseChunkSingleValueReader.java:57-96 header, version 1 always Snappy, version 2 PASS_THROUGH or
 * Snappy chunks; FixedByteChunkSingleValueReader.getInt / getLong / getFloat / getDouble), as the segment loader reads
 * .sv.raw.fwd. data_type INT / LONG / FLOAT / DOUBLE; values receives num_docs native-endian values. */
pinot_status pinot_segment_read_raw_forward_index(const uint8_t *bytes, uint64_t len, int32_t data_type, int32_t num_docs,
                                          void *values);
/* A raw (no-dictionary) column's dictionary form exactly as pinot_gpu_segment_register builds it before upload
 * (replaces the reference's raw-value reads, PhysicalColumnIndexContainer.java:101-106 / FixedByteChunkSingleValueReader,
 * with the dictionary plans' input): numeric columns radix-sorted on the engine's GPU when on_device is 1 (config key
 * raw.device, default on), on the host otherwise; STRING columns on the host. Outputs the cardinality, the bits per
 * dictId, the dictionary (cardinality big-endian values, STRING zero-padded to the longest) and the MSB-first packed
 * forward index; null buffers report the lengths only. PINOT_ERR_BAD_ARG for a dictionary-encoded column. */
pinot_status pinot_gpu_transcode_raw(pinot_engine *engine, const pinot_column_desc *column, int32_t num_docs,
                                     int32_t on_device, int32_t *cardinality, int32_t *bits_per_value,
                                     uint8_t *dictionary, uint64_t dictionary_cap, uint64_t *dictionary_len,
                                     uint8_t *forward_index, uint64_t forward_cap, uint64_t *forward_len);
/* Every check pinot_gpu_segment_register makes on the descriptor's bytes (dictionaries, forward-index
 * length, sorted-index tiling, inverted-index offsets and roaring containers), on the host only: no engine,
 * no GPU. PINOT_ERR_BAD_ARG + pinot_gpu_last_error() name the first bad column. */
pinot_status pinot_gpu_segment_validate(const pinot_segment_desc *desc);
/* Bytes of HBM held by a segment. */
/* A segment's star-tree v2 index (PC/startree/v2, StarTreeLoaderUtils.java:60-110): the tree as OffHeapStarTree
 * reads it (little-endian: magic 0xBADDA55B00DAD00D, version 1, header size, (index, name) per dimension, node count,
 * 7 int32 per node in BFS order: dimension id, dimension value (-1 = star), start doc, end doc, aggregated doc, first
 * child, last child), and its documents as a segment descriptor: one dictionary column per split-order dimension
 * named like the segment's column (the segment's own dictionary bytes, the star-tree's fixed-bit forward index at
 * the segment column's bits per element, STAR stored as 0) and one raw column per function-column pair, named as
 * AggregationFunctionColumnPair.toColumnName ("count__*" LONG; "sum__x", "min__x", "max__x" DOUBLE; AVG's AvgPair
 * BYTES column "avg__x" as its two halves "avg__x.sum" DOUBLE + "avg__x.count" LONG; DISTINCTCOUNTHLL's
 * "distinctCountHLL__x" as a raw STRING-layout column of HyperLogLog.getBytes values, log2m 8). Queries the tree fits
 * (StarTreeUtils.isFitForStarTree: COUNT / SUM / MIN / MAX / AVG / DISTINCTCOUNTHLL with their pairs, group-by and
 * filter columns in
 * the split order, no OR) then run on the star-tree (StarTreeFilterOperator's traversal + the pre-aggregated
 * functions) when every queried segment has one; engine config startree.use=0 disables it (the reference's
 * useStarTree=false debug option). */
typedef struct {
  const uint8_t *tree;
  uint64_t tree_len;
  const pinot_segment_desc *docs;
} pinot_star_tree_desc;
pinot_status pinot_gpu_segment_attach_star_tree(pinot_engine *engine, pinot_segment_handle handle,
                                                const pinot_star_tree_desc *desc);
pinot_status pinot_gpu_segment_device_bytes(pinot_engine *engine, pinot_segment_handle handle, uint64_t *out);

/* Filter one segment: writes the dense doc bitset (bit d of word d/64 = doc d, LSB first;
 * caller provides ceil(N/64) words, may be NULL to only count) and the matching doc count. */
pinot_status pinot_gpu_filter(pinot_engine *engine, pinot_segment_handle segment,
                              int32_t num_filter_nodes, const pinot_filter_node *filter,
                              uint64_t *bitset_out, int64_t *count_out);

/* Aggregation-only query over segments on this engine's GPU; out has num_aggregations entries. */
pinot_status pinot_gpu_aggregate(pinot_engine *engine, const pinot_segment_handle *segments,
                                 int32_t num_segments, const pinot_query *query,
                                 pinot_agg_result *out, pinot_exec_stats *stats);

/* Group-by query over segments; the result object lists the non-empty groups. */
pinot_status pinot_gpu_group_by(pinot_engine *engine, const pinot_segment_handle *segments,
                                int32_t num_segments, const pinot_query *query,
                                pinot_groupby_result **out, pinot_exec_stats *stats);
/* The group-by as the server hands it to the DataTable: CombineGroupByOperator's trim
 * (AggregationGroupByTrimmingService.trimIntermediateResultsMap, :71-116; CombineGroupByOperator.java:184-215) runs on
 * the device before any group leaves it. Above 4 x trimSize groups (trimSize = max(5 * top_n, 5000)) the result holds
 * only the union of the functions' trimmed maps (pinot_groupby_trim with the same top_n lists each function's groups;
 * another top_n is PINOT_ERR_BAD_ARG); otherwise every group, as pinot_gpu_group_by. Ties: lower raw key first. The
 * device trim applies to dense key spaces; hashed, multi-value and star-tree group-bys return every group and trim
 * on the host (pinot_groupby_trim). */
pinot_status pinot_gpu_group_by_top(pinot_engine *engine, const pinot_segment_handle *segments,
                                    int32_t num_segments, const pinot_query *query, int32_t top_n,
                                    pinot_groupby_result **out, pinot_exec_stats *stats);
int64_t pinot_groupby_num_groups(const pinot_groupby_result *r);
int32_t pinot_groupby_num_columns(const pinot_groupby_result *r);
/* '\t'-joined group key string (DictionaryBasedGroupKeyGenerator.getGroupKey); NUL-terminated. */
const char *pinot_groupby_key(const pinot_groupby_result *r, int64_t group);
/* Per group: count (COUNT / AVG count), value (SUM / MIN / MAX / AVG sum) for function fn. */
pinot_status pinot_groupby_values(const pinot_groupby_result *r, int32_t fn, int64_t *counts, double *values);
/* DISTINCTCOUNTHLL: 256 registers per group (num_groups*256 bytes) and/or final cardinalities. */
pinot_status pinot_groupby_hll(const pinot_groupby_result *r, int32_t fn, uint8_t *registers, int64_t *cardinalities);
/* Raw dense keys in the query's global key space (column 0 least significant). */
pinot_status pinot_groupby_raw_keys(const pinot_groupby_result *r, int64_t *keys);
/* Every group key string in one call (what a JNI caller copies into one byte[] + int[] pair): group g's bytes
   are buf[offsets[g], offsets[g + 1]) (no terminator); offsets has num_groups + 1 entries. buf == NULL (or too
   short) only sets *bytes_needed. */
pinot_status pinot_groupby_export_keys(const pinot_groupby_result *r, char *buf, uint64_t buf_len, int64_t *offsets,
                                       uint64_t *bytes_needed);
/* AggregationGroupByTrimmingService.trimIntermediateResultsMap (:71-116) for function fn: the groups of fn's
   trimmed map, ascending group index. trimSize = max(5 * top_n, 5000); trimming happens only above
   4 * trimSize groups, keeping the trimSize best final values (MIN ascending, every other function descending,
   :160-176; ties: lower raw key first, where the reference's heap order is arbitrary). groups == NULL only sets
   *num_out. */
pinot_status pinot_groupby_trim(const pinot_groupby_result *r, int32_t top_n, int32_t fn, int64_t *groups,
                                int64_t *num_out);
void pinot_groupby_free(pinot_groupby_result *r);

/* ------------------------------------------------------------------ segment pruning
 * The step before the plan: processQuery drops segments the query cannot match and runs the plan on the rest
 * (ServerQueryExecutorV1Impl.java:183-216). Pruners (bit mask; applied in the server's default order,
 * DefaultHelixStarterServerConfig.java:60-64):
 *   DATA_SCHEMA   a query column (filter, non-COUNT aggregation, group-by) missing from the segment
 *                 (DataSchemaSegmentPruner.java:38-41)
 *   COLUMN_VALUE  EQUALITY / RANGE leaves outside the column's [minValue, maxValue] metadata (a column without
 *                 them never prunes; a loaded segment's time column gets its dictionary's ends, as the default
 *                 ColumnMinMaxValueGenerator mode TIME does at load), and an EQUALITY value the column's bloom
 *                 filter rules out (:140-144); AND prunes when any child does, OR when all do
 *                 (ColumnValueSegmentPruner.java:49-200, AbstractSegmentPruner.java:56-90)
 *   VALID         an empty segment (ValidSegmentPruner.java:47-58)
 *   PARTITION     an EQUALITY value whose partition (the column's partition function) the segment does not hold
 *                 (PartitionSegmentPruner.java:73-111); the default list has it last
 *                 (DefaultHelixStarterServerConfig.java:60-65)
 * A bad literal in an EQUALITY / RANGE leaf is PINOT_ERR_BAD_QUERY (AbstractSegmentPruner.getValue); a query column
 * the engine left out of a loaded segment (multi-value / raw / BYTES) is PINOT_ERR_UNSUPPORTED; a query whose budget
 * is already spent (timeout_ms < 0) is PINOT_ERR_TIMEOUT, checked before pruning as processQuery does (:116-126). */
typedef enum {
  PINOT_PRUNER_DATA_SCHEMA = 1, PINOT_PRUNER_COLUMN_VALUE = 2, PINOT_PRUNER_VALID = 4, PINOT_PRUNER_PARTITION = 8,
  PINOT_PRUNER_DEFAULT = 15
} pinot_pruner;

/* pruned[i] = 1 when segment i is dropped, else 0; *total_raw_docs = the docs of ALL the segments, pruned or not
 * (the totalDocs processQuery reports, :214-215). */
pinot_status pinot_gpu_prune_segments(pinot_engine *engine, const pinot_segment_handle *segments, int32_t num_segments,
                                      const pinot_query *query, int32_t pruners, uint8_t *pruned,
                                      int64_t *total_raw_docs);
/* The same decision for one segment descriptor, on the host only (no engine, no GPU). */
pinot_status pinot_segment_prune(const pinot_segment_desc *desc, const pinot_query *query, int32_t pruners,
                                 int32_t *pruned);

/* ------------------------------------------------------------------ DataTable (server -> broker bytes)
 * IntermediateResultsBlock.getDataTable (PC/operator/blocks/IntermediateResultsBlock.java:206-317) serialized as
 * DataTableImplV2.toBytes (PC/common/datatable/DataTableImplV2.java:233-347), object cells per ObjectSerDeUtils
 * (PC/common/ObjectSerDeUtils.java). Metadata: the block's statistics (attachMetadataToDataTable :298-317) and,
 * when `server` is given, the server's own keys (ServerQueryExecutorV1Impl.java:244-245). */
typedef struct {
  int64_t num_segments_queried;
  int64_t time_used_ms;
  int64_t request_id;          /* < 0: no requestId key */
} pinot_datatable_server;

/* Aggregation-only result (getAggregationResultDataTable :234-270): *out_len = size; bytes copied when buf_len
 * suffices (buf == NULL: size only), else PINOT_ERR_BAD_ARG. */
pinot_status pinot_datatable_aggregation(const pinot_query *query, const pinot_agg_result *results,
                                         const pinot_exec_stats *stats, const pinot_datatable_server *server,
                                         uint8_t *buf, uint64_t buf_len, uint64_t *out_len);
/* Group-by result (getAggregationGroupByResultDataTable :272-292): one row per function, its map restricted to
 * fn_groups[fn] (fn_num_groups[fn] group indexes, e.g. pinot_groupby_trim's output) when fn_groups and
 * fn_groups[fn] are non-NULL. The bytes are owned by the result: each call's *data stays valid until
 * pinot_groupby_free (a later call on the same result writes a new buffer). */
pinot_status pinot_datatable_group_by(const pinot_query *query, const pinot_groupby_result *result,
                                      const int64_t *const *fn_groups, const int64_t *fn_num_groups,
                                      const pinot_exec_stats *stats, const pinot_datatable_server *server,
                                      const uint8_t **data, uint64_t *len);

/* Every segment pruned (ServerQueryExecutorV1Impl.java:187-196): DataTableBuilder.buildEmptyDataTable (:292-370;
 * aggregation-only: one row of the functions' empty results, group-by: one empty map per function) with totalDocs
 * = total_docs and every other statistic 0. Buffer protocol as pinot_datatable_aggregation. */
pinot_status pinot_datatable_empty(const pinot_query *query, int64_t total_docs, const pinot_datatable_server *server,
                                   uint8_t *buf, uint64_t buf_len, uint64_t *out_len);

/* ------------------------------------------------------------------ broker reduce
 * BrokerReduceService.reduceOnDataTable (PC/query/reduce/BrokerReduceService.java:69-270, :347-530) over the
 * servers' DataTable bytes for an aggregation-only or group-by query (no HAVING, no selection): statistics summed
 * from the metadata, intermediate results merged per function (group maps by key), final results extracted, the
 * group-by top_n kept per function (AggregationGroupByTrimmingService.trimFinalResults :123-149: MIN ascending,
 * others descending; ties by group key) and every value formatted by AggregationFunctionUtils.formatValue
 * (:113-128, "%1.5f" rounded half-up on the shortest digits). Writes the BrokerResponseNative JSON
 * (BrokerResponseNative.java:42 field order; timeUsedMs 0, numServersQueried / Responded = num_tables). Buffer
 * protocol as pinot_datatable_aggregation. */
pinot_status pinot_broker_reduce(const pinot_query *query, int32_t num_tables, const uint8_t *const *tables,
                                 const uint64_t *lens, int32_t top_n, char *buf, uint64_t buf_len, uint64_t *out_len);

/* ------------------------------------------------------------------ multi-GPU partials
 * Group-by over a GLOBAL dense key space, for segment sharding across ranks: each rank
 * accumulates its segments into caller-provided DEVICE arrays (one set per rank, same
 * shape everywhere), the caller all-reduces them over RCCL (sum for counts/sums, max for
 * HLL registers, min/max for MIN/MAX), then pinot_gpu_group_by_finalize reads the merged
 * arrays. The key space is the product of the group-by columns' cardinalities, which must
 * be identical dictionaries on every segment (checked). */
typedef struct {
  int64_t num_keys;            /* G = Π cardinalities */
  int32_t num_aggregations;
  int32_t reserved;
  /* per aggregation f: accumulator kind and element size, so the caller can allocate:
     kind 0 = int64 sum, 1 = double sum, 2 = uint64 ordered-min, 3 = uint64 ordered-max,
     4 = uint8 HLL registers (256 bytes per key: an all-reduce MAX over uint8 moves G*256 bytes),
     5 = none (COUNT uses the shared count array) */
  int32_t acc_kind[8];
  uint64_t group_dictionary_fingerprint; /* FNV-1a of the group-by columns' dictionaries: ranks compare it
                                            before merging (raw keys mean the same groups only when equal) */
} pinot_partial_layout;

pinot_status pinot_gpu_group_by_layout(pinot_engine *engine, const pinot_segment_handle *segments,
                                       int32_t num_segments, const pinot_query *query,
                                       pinot_partial_layout *layout);
/* counts: int64[G] device; accs[f]: device array per acc_kind (NULL for kind 5). Arrays are
 * zero/identity-initialised by this call. */
pinot_status pinot_gpu_group_by_partial(pinot_engine *engine, const pinot_segment_handle *segments,
                                        int32_t num_segments, const pinot_query *query,
                                        int64_t *counts_dev, void *const *accs_dev,
                                        pinot_exec_stats *stats);
pinot_status pinot_gpu_group_by_finalize(pinot_engine *engine, const pinot_segment_handle *segments,
                                         int32_t num_segments, const pinot_query *query,
                                         const int64_t *counts_dev, void *const *accs_dev,
                                         pinot_groupby_result **out);

/* ------------------------------------------------------------------ multi-GPU server
 * One server per node process: QueryExecutor.init with a device mask. It owns one engine per GPU and
 * the RCCL communicators, created once (ncclCommInitAll). Segments are registered on its engines
 * (pinot_gpu_server_engine; never pass those to pinot_gpu_engine_destroy) and queried together: the result is the
 * combine over every GPU, as CombineOperator / CombineGroupByOperator return it (CombineOperator.java:75-196,
 * CombineGroupByOperator.java:104-228). Group-by merges dense partials over the query's global key space (the
 * union of every GPU's dictionaries: per-segment dictionaries may differ) with a reduce-scatter, finalizes each key
 * range on its GPU and gathers the ranges to the first GPU. Not handled across GPUs (PINOT_ERR_UNSUPPORTED: run on
 * one engine): hashed key spaces (LONG_MAP / ARRAY_MAP) and queries where the 2 x num.groups.limit inter-segment cap
 * can bind. */
typedef struct pinot_server pinot_server;
typedef struct {
  int32_t engine;              /* index of the server engine that holds the segment */
  int32_t reserved;
  pinot_segment_handle handle; /* that engine's handle */
} pinot_segment_ref;

pinot_status pinot_gpu_server_create(const int32_t *devices, int32_t num_devices, const char *config, pinot_server **out);
/* Multi-process form (one process per GPU): rank 0 makes a 128-byte id, shares it out of band; every rank then
 * creates its server with (device, nranks, rank, id). Every rank calls each query, with its own segments (none, or
 * all pruned, is fine: it contributes identities). Group-by dictionaries may differ across ranks and segments: the
 * ranks exchange their dictionaries and merge over the union. Aggregation results are complete on every rank; the
 * group-by result is complete on rank 0 (the key ranges gathered there) and empty on the others, or with
 * "server.gather=0" each rank's own key range (ranges disjoint and ascending). Any rank's failure (bad literal,
 * timeout, unsupported shape) fails every rank with that status: no rank is left waiting in a collective.
 * Server config keys (besides the engines'): server.gather=0|1, server.loopback=1 (every rank of the communicator
 * in this process on ONE device, the collectives done by an in-library device reduce / copy: the multi-GPU merge
 * protocol on one GPU; with pinot_gpu_server_create the devices must repeat one device, with _create_rank every
 * rank passes the same id and device from its own thread), server.timeout_ms (in-process rendezvous timeout). */
pinot_status pinot_gpu_server_unique_id(uint8_t *unique_id);
pinot_status pinot_gpu_server_create_rank(int32_t device, int32_t nranks, int32_t rank, const uint8_t *unique_id,
                                          const char *config, pinot_server **out);
pinot_status pinot_gpu_server_destroy(pinot_server *server);
int32_t pinot_gpu_server_num_engines(const pinot_server *server);
pinot_status pinot_gpu_server_engine(pinot_server *server, int32_t index, pinot_engine **out);
pinot_status pinot_gpu_server_aggregate(pinot_server *server, const pinot_segment_ref *segments, int32_t num_segments,
                                        const pinot_query *query, pinot_agg_result *out, pinot_exec_stats *stats);
pinot_status pinot_gpu_server_group_by(pinot_server *server, const pinot_segment_ref *segments, int32_t num_segments,
                                       const pinot_query *query, pinot_groupby_result **out, pinot_exec_stats *stats);
/* (ABI >= 14) The server's trimmed answer, as pinot_gpu_group_by_top is the engine's: CombineGroupByOperator's
 * AggregationGroupByTrimmingService (CombineGroupByOperator.java:184-187, AggregationGroupByTrimmingService.java:71-116)
 * across the GPUs. After the reduce-scatter each rank owns a disjoint key range; the ranks all-gather their ranges'
 * group counts, and when the merged map exceeds 4 x trimSize (trimSize = max(5 * top_n, 5000)) each rank keeps only its
 * range's trimSize best groups per function before the gather to rank 0, which picks each function's trimSize best
 * among them (the merged map's best, the ranges being disjoint). The result is device-trimmed (pinot_groupby_trim
 * returns each function's list; top_n must match). With server.gather=0 and several ranks, or AvgMV functions, the
 * result is returned untrimmed. */
pinot_status pinot_gpu_server_group_by_top(pinot_server *server, const pinot_segment_ref *segments,
                                           int32_t num_segments, const pinot_query *query, int32_t top_n,
                                           pinot_groupby_result **out, pinot_exec_stats *stats);
/* Host wall time (ms) of the phases of the server's last query as its first engine's rank ran it (n <= 8 values):
 *   [0] local work (aggregation: prune + plan + run; group-by: prune + dictionaries)  [1] all-gather of the ranks'
 *   headers (aggregation: of their results) + the global key space  [2] group-by partials on the device
 *   [3] agreement after the partials  [4] reduce-scatter (its device time when the engine has timing=1, else the
 *   launch)  [5] owner finalize (compaction + outputs)  [6] gather to rank 0 + D2H  [7] total. */
pinot_status pinot_gpu_server_last_phases(const pinot_server *server, double *ms, int32_t n);
/* pinot_gpu_prune_segments over segments spread across the server's engines. */
pinot_status pinot_gpu_server_prune_segments(pinot_server *server, const pinot_segment_ref *segments,
                                             int32_t num_segments, const pinot_query *query, int32_t pruners,
                                             uint8_t *pruned, int64_t *total_raw_docs);

/* ------------------------------------------------------------------ benchmark tooling
 * NOT part of the Java drop-in path: builds a synthetic dictionary-encoded column
 * directly in HBM (seeded splitmix64; docs [0, card) hold values 0..card-1 so every
 * segment has the identity dictionary [0, card)). Used by bench.py to avoid 15 GB of
 * host→device copies; the same generator is restated on the host in oracle/. */
pinot_status pinot_gpu_segment_register_synthetic(pinot_engine *engine, const char *name,
                                                  int32_t num_docs, int32_t num_columns,
                                                  const char *const *column_names,
                                                  const int32_t *cardinalities, uint64_t seed,
                                                  pinot_segment_handle *out);
/* Same, with a kind per column (NULL = all PINOT_SYNTH_RANDOM): SORTED = value v on the docs
 * [v*N/card, (v+1)*N/card) with a sorted index; INVERTED = the RANDOM values with a bitmap inverted index
 * (both built on the host in Pinot's file layout and registered like a loaded segment). */
typedef enum { PINOT_SYNTH_RANDOM = 0, PINOT_SYNTH_SORTED = 1, PINOT_SYNTH_INVERTED = 2 } pinot_synth_kind;
pinot_status pinot_gpu_segment_register_synthetic_ex(pinot_engine *engine, const char *name,
                                                     int32_t num_docs, int32_t num_columns,
                                                     const char *const *column_names,
                                                     const int32_t *cardinalities, const int32_t *kinds,
                                                     uint64_t seed, pinot_segment_handle *out);

/* Synchronise the engine's stream (bench timing brackets). */
pinot_status pinot_gpu_synchronize(pinot_engine *engine);
/* Device time (ms) of the named kernel class in the last call, for the roofline report:
 * kind 0 = scan/filter kernel, 1 = aggregation kernel. */
pinot_status pinot_gpu_last_kernel_ms(pinot_engine *engine, int32_t kind, double *ms, int64_t *launches);
/* Engine counters (diagnostics, no Java counterpart): "group.ring_queries" = group-bys answered on the ring plan,
 * "group.ring_fallbacks" = ring-plan group-bys re-answered on the counted plan (a region overflowed: skewed keys),
 * "group.ring_waits" / "group.ring_sleeps" = ring-sink rounds that waited for a ring half to drain / their spins
 * (counted under debug.ring only),
 * "exec.last_pre_segments" = segments of the last fused query whose filter was built as a dense `pre` bitset by the
 * launch sequence instead of inside the fused kernel's register program. */
pinot_status pinot_gpu_engine_stat(pinot_engine *engine, const char *name, int64_t *value);

#ifdef __cplusplus
}
#endif
#endif /* PINOT_GPU_H_ */
