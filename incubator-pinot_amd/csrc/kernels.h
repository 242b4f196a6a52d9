// Kernel argument blocks and launch entry points (scan.hip, kernels.hip).
//
// HBM layout of a segment:
//   forward index  : the segment's own big-endian MSB-first fixed-bit stream, copied as-is,
//                    zero-padded by >= 256 bytes so a 64-doc super-word load never leaves the
//                    allocation. Doc d occupies bits [d*b, d*b+b) of the stream; the 64 docs of
//                    word w occupy exactly the 8*b bytes at offset 8*b*w (8-byte aligned).
//   dictionary     : INT -> int32, LONG -> int64, FLOAT/DOUBLE -> double (little-endian).
//   filter bitsets : u64 words, bit (d & 63) of word d >> 6 = doc d.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace pinot {

constexpr int kMaxProgramColumns = 24;
constexpr int kMaxProgramInstr = 48;
constexpr int kMaxStack = 8;
constexpr int kMaxAggs = 8;
constexpr int kMaxHll = 4;
constexpr int kMaxGroupCols = 16;
constexpr int kBlock = 256;

struct DevColumn {
  const uint8_t *fwd;  // packed forward index (BE, MSB-first)
  int32_t bits;
  int32_t card;
};

constexpr int kMaxScanGrid = 2048;  // blocks per streaming launch (8 per CU); grid-stride beyond

// ---------------------------------------------------------------- streaming kernels (scan.hip)
enum LeafKind : int32_t { LEAF_RANGE = 0, LEAF_LUT64 = 1, LEAF_LUT = 2 };
enum CombineMode : int32_t { CM_WRITE = 0, CM_AND = 1, CM_OR = 2 };

// Filter leaf on one segment column: m = pred(dictId) per doc, optionally negated, then written to /
// AND-ed into / OR-ed into dst.
struct LeafArgs {
  const uint8_t *fwd;
  int64_t nwords;
  int32_t num_docs;
  int32_t negate;
  uint32_t lo, span;          // LEAF_RANGE: lo <= id < lo + span
  uint64_t lut64;             // LEAF_LUT64: bit id (cardinality <= 64)
  const uint32_t *lut;        // LEAF_LUT: bit id of the membership bitmap
  int32_t mode;               // CombineMode
  int32_t reserved;
  uint64_t *dst;
};
void launch_leaf(int bits, int kind, const LeafArgs &a, hipStream_t stream);

// Multi-value scan leaf (MVScanDocIdIterator, PC/operator/dociditerators/MVScanDocIdIterator.java:108-123, with
// BaseDictionaryBasedPredicateEvaluator.applyMV :103-121): a doc matches when ANY entry's dictId is in lut, or for an
// exclusive predicate (all = 1) when EVERY entry's is; written to / AND-ed into / OR-ed into dst like LeafArgs.
struct MvLeafArgs {
  const uint8_t *fwd;          // packed entries
  const uint32_t *offsets;     // [num_docs + 1] row starts
  const uint32_t *lut;         // bit dictId = applySV(dictId)
  int64_t nwords;
  int32_t num_docs, bits;
  int32_t all, mode;
  uint64_t *dst;
};
void launch_mv_leaf(const MvLeafArgs &a, hipStream_t stream);

// Aggregations of a query that touches multi-value columns (the *MVAggregationFunction aggregate() loops, and the
// single-value functions beside them): one lane per doc over the doc's entries. Per aggregation the kernel keeps
// out[5 * a + k]: k = 0 entries (COUNT*: docs), 1 int64 sum, 2 double sum bits, 3 / 4 min / max as order-preserving
// u64 images of the double value; HLL registers in hll[a * 256 + r] (atomicMax).
// MVA_REGS: a star-tree's HyperLogLog column — 256 u8 registers per doc at dict + doc * 256, max-merged.
enum MvAggKind : int32_t { MVA_COUNT_DOCS = 0, MVA_VALUES = 1, MVA_HLL = 2, MVA_REGS = 3 };
struct MvAggSpec {
  const uint8_t *fwd;          // packed forward index (entries for MV columns)
  const uint32_t *offsets;     // MV: [num_docs + 1] row starts; null: single-value column
  const void *dict;            // int32 / int64 / double dictionary values
  const uint16_t *hll_lut;     // MVA_HLL: (register << 8 | rank) per dictId
  int32_t bits, kind, value_kind, numeric;
};
struct MvAggArgs {
  const uint64_t *bitset;      // matching docs; null = all
  int64_t nwords;
  int32_t num_docs, n;
  MvAggSpec specs[kMaxAggs];
  unsigned long long *out;     // [kMaxAggs][5], identities on entry (0, 0, +0.0, ~0, 0)
  uint32_t *hll;               // [kMaxAggs][256]
  unsigned long long *docs;    // matching docs (one counter)
};
void launch_mv_aggregate(const MvAggArgs &a, hipStream_t stream);

enum ColAggOps : int32_t { COLAGG_IDSUM = 1, COLAGG_MINMAX = 2 };
// Per-column fold over the docs of `bitset` (null = all): per-block partials of COUNT, Σ dictId, min/max dictId.
struct ColAggArgs {
  const uint8_t *fwd;
  const uint64_t *bitset;
  int64_t nwords;
  int32_t num_docs;
  int32_t reserved;
  unsigned long long *out_count, *out_idsum, *out_minmax;  // [grid] each
};
void launch_colagg(int bits, int ops, const ColAggArgs &a, hipStream_t stream);

enum GatherKind : int32_t { GA_SUM_I32 = 0, GA_SUM_I64 = 1, GA_SUM_F64 = 2, GA_HLL = 3 };
struct GatherSpec {
  int32_t kind;
  int32_t bits;
  int32_t hll_slot;
  int32_t reserved;
  const uint8_t *fwd;
  const void *table;            // int32 / int64 / double dictionary or u16 HLL (register << 8 | rank) LUT
  unsigned long long *out;      // [grid] per-block partials (sums)
  uint32_t *hll_out;            // 256 registers (atomicMax)
};
struct GatherArgs {
  const uint64_t *bitset;
  int64_t nwords;
  int32_t num_docs;
  int32_t n;
  unsigned long long *out_count;  // [grid]
  GatherSpec specs[kMaxAggs];
};
void launch_gather_agg(const GatherArgs &a, hipStream_t stream);
void launch_popcount(const uint64_t *bitset, int64_t nwords, int32_t num_docs, unsigned long long *out,
                     hipStream_t stream);

enum SlotKind : int32_t { SLOT_SUM_U64 = 0, SLOT_SUM_F64 = 1, SLOT_MINMAX = 2 };
constexpr int kMaxSlots = 64;
// Reduces slot s (grid partials at in + s * stride) into out[out_index[s]], fixed order.
struct ReduceArgs {
  const unsigned long long *in;
  int64_t stride;
  int32_t grid;
  int32_t reserved;
  unsigned long long *out;
  int32_t kinds[kMaxSlots];
  int32_t out_index[kMaxSlots];
};
void launch_reduce_slots(const ReduceArgs &a, int nslots, hipStream_t stream);
int scan_grid(int64_t nwords);

// ---------------------------------------------------------------- fused query kernel (scan.hip)
// ONE launch evaluates an aggregation-only query over every segment on the GPU: per 4096-doc chunk a
// wave AND-s the scan leaves of the filter into a 64-bit mask per lane (held in registers, never
// written to HBM), optionally starting from a `pre` bitset (index leaves / OR subtrees, evaluated by
// the kernels below), skips the rest of the chunk as soon as the wave's mask is empty, then folds
// the aggregated columns of the matching docs.
enum FusedKind : int32_t {
  FK_LEAF_RANGE = 0, FK_LEAF_LUT64 = 1, FK_LEAF_LUT = 2, FK_FOLD = 3,
  FK_LEAF_RANGES = 4,   // sorted-index leaf: inclusive [start, end] doc ranges (table, n = lo)
  FK_LEAF_ROARING = 5,  // bitmap-index leaf: OR of the dictIds' roaring bitmaps (fwd = payload, aux0 = containers,
                        // aux1 = per-dictId container directory, table = dictIds, n = lo), negate = exclusive;
                        // ops = 1 (more than 256 dictIds): aux1 = per-key directory [lo + 1] into table = the dictIds'
                        // container indices bucketed by roaring key (lo = keys)
  FK_OP = 6             // nested AND / OR: term = (popped entry) op term, op in `join` (JOIN_AND / JOIN_OR)
};
// How a leaf joins the filter program (the top-level conjunction of terms, a term = an AND / OR tree of leaves in
// postfix): JOIN_NEW starts a term (the previous one is AND-ed into the mask), JOIN_OR / JOIN_AND combine the leaf
// into the running term, JOIN_PUSH pushes the running term onto a register stack and starts a nested one (an FK_OP
// step pops it and combines). kMaxFusedStack entries below the running term.
enum FusedJoin : int32_t { JOIN_NEW = 0, JOIN_OR = 1, JOIN_AND = 2, JOIN_PUSH = 3 };
constexpr int kMaxFusedStack = 4;       // k_scan_query's register stack
constexpr int kMaxFusedStackGroup = 3;  // the group-by kernels' (one 64-bit entry less: their registers are spoken for)
enum FoldOps : int32_t { FOLD_IDSUM = 1, FOLD_MINMAX = 2, FOLD_DICT32 = 4, FOLD_HLL = 8 };
constexpr int kMaxFusedFolds = 6;                      // distinct aggregated columns per query
constexpr int kMaxFusedSlots = 1 + 2 * kMaxFusedFolds; // slot 0 count; fold f: 1 + 2f sum, 2 + 2f min/max

struct FusedStep {           // one (segment, leaf or fold) pair, built on the host per query
  const uint8_t *fwd;        // packed forward index of the column
  const void *table;         // FK_LEAF_LUT: u32 membership words; FOLD_DICT32: int32 dictionary
  const uint16_t *hll_lut;   // FOLD_HLL: (register << 8 | rank) per dictId
  uint64_t lut64;            // FK_LEAF_LUT64
  uint32_t lo, span;         // FK_LEAF_RANGE: lo <= id < lo + span
  int32_t bits, kind, negate, ops;
  int32_t fold, hll_set;     // FK_FOLD: fold index (slots 1 + 2f, 2 + 2f), HLL register set
  int32_t stage_off;         // pipelined kernel: byte offset of this step's chunk within the wave's LDS slot
  int32_t join;              // leaves: FusedJoin
  const void *aux0, *aux1;   // FK_LEAF_ROARING: containers, directory
};

struct FusedSegment {
  const uint64_t *pre;       // AND-ed in before the leaves; null = all docs
  int64_t nwords;            // 0 = skip the segment (EMPTY filter)
  int32_t num_docs;
  int32_t first_step;        // leaves [first, first + n_leaves), then folds
  int32_t n_leaves;
  int32_t n_folds;
  int64_t ch_begin, ch_end;  // chunk window: a top-level sorted-index term bounds the candidate docs
};

struct FusedArgs {
  const FusedSegment *segs;
  const FusedStep *steps;
  unsigned long long *acc;   // [nsegs][res_stride] accumulators (identity between launches: sums 0,
                             // min/max slots min = 0xFFFFFFFF / max = 0), reset by the last block
  uint32_t *hll_out;         // [kMaxHll][256] registers, atomicMax (zero on entry; re-zeroed by the last block)
  int32_t nsegs, bps;        // block b serves segment b / bps
  int32_t nslots;            // 1 + 2 * folds
  int32_t stage_bytes;       // stepwise: LDS bytes per wave = staged_chunk_bytes(max bits);
                             // pipelined: bytes of ONE chunk slot (all steps), two slots per wave
  int32_t n_hll;
  int32_t nt;                // pipelined: non-temporal policy on the column DMA (exec.nt)
  int32_t res_stride;        // u64 slots per segment in `result`
  uint32_t *done;            // arrival counter (0 between launches; the last block resets it)
  unsigned long long *result;  // host-mapped: [nsegs][res_stride] slots, then [kMaxHll][256] u32 HLL registers
  int64_t result_hll_off;    // byte offset of the HLL registers in `result`
  // completion flag: the last block writes {elapsed wall-clock ticks, seq} at result_tail_off after every
  // result, behind a system-scope release, so the host can spin on mapped memory instead of waiting for the
  // runtime's completion signal (seq 0: no flag)
  int64_t result_tail_off;
  unsigned long long *clock_start;  // device: earliest block start (wall_clock64); ~0 between launches
  uint32_t seq;
  int32_t reserved;
};
// Largest chunk slot the pipelined kernel double-buffers in LDS: 512 B of `pre` words + every step's
// 1-KiB pieces; 4 waves x 2 slots x 18.5 KiB + the block's FusedLds fit the 160 KiB of a CU.
constexpr int kPipePreBytes = 512;
// A staged chunk's 1-KiB DMA pieces sit kPiecePad bytes apart in LDS: the per-lane super-word reads of the
// decoders (lane stride 8*B bytes) then spread over all 64 banks for every width but 16 and 32 (2-way),
// where back-to-back pieces left B = 8, 12, 20, 24, 28 2-8-way conflicted (fused_common.h decode_half).
constexpr int kPiecePad = 8;
constexpr int kPieceStride = 1024 + kPiecePad;
constexpr int staged_chunk_bytes(int bits) { return kPieceStride * ((bits + 1) / 2); }
constexpr int kMaxPipeSlotBytes = 18 * kPieceStride + kPipePreBytes;
// gathers: the program has memory-LUT leaves, FOLD_DICT32 or FOLD_HLL (selects the gather instance).
// pipelined: whole-chunk double-buffered staging (stage_bytes = slot <= kMaxPipeSlotBytes), else stepwise.
void launch_scan_query(const FusedArgs &a, bool gathers, bool pipelined, hipStream_t stream);
// Resident blocks of k_scan_query per CU for a stage size (occupancy API), cached.
int scan_query_blocks_per_cu(int stage_bytes, bool gathers, bool pipelined);

// ---------------------------------------------------------------- fused group-by (fused.hip)
// ONE launch per group-by query over every segment on the GPU: the filter leaves are evaluated exactly
// as in k_scan_query (LDS-staged chunks, register masks, `pre` bitsets), then every matching doc's raw
// group key (mixed radix over the global ids of the group columns) and aggregated dictIds are read
// straight from the packed forward indexes (one doc per lane: the 64 lanes of a wave read 8*b
// contiguous bytes per column) and handed to a sink:
//   GB_GLOBAL  HBM atomics into dense per-key accumulators (medium key spaces)
//   GB_LDS     LDS-privatised per-block accumulators, flushed with HBM atomics (small key spaces)
//   GB_COUNT   pass 1 of the partitioned plan: per-block histogram of partitions (key >> shift)
//   GB_EMIT    pass 2: (local key | dictId fields) u64 records scattered into partition runs;
//              k_partition_reduce then owns one partition per block (accumulators in LDS, no atomics
//              to HBM) — the large key spaces (config 4: 1 M keys with HLL)
//   GB_VERIFY  hashed key spaces: re-reads every matching doc's tuple and checks it against its hash
//              slot's representative doc (a 64-bit fingerprint collision is detected, never merged)
//   GB_FIRST   num.groups.limit admission: first_doc[segment][key] = smallest matching doc of the key
//              (a plain read first; atomicMin only when the doc is earlier)
//   GB_EMIT2   pass 2 of the bucketed partitioned plan: the filter words GB_COUNT wrote (no filter re-evaluation),
//              records appended to per-block LDS buckets of kBucketRecs records per partition and written out
//              whole into the FINAL partition layout (offsets from GB_COUNT's histogram): no split pass
//   GB_FILTER  the ring plan's first pass for filters k_group_ring does not evaluate itself (group_ring.hip): the
//              filter program alone, its words per segment into filter_out
enum GroupMode : int32_t { GB_GLOBAL = 0, GB_LDS = 1, GB_COUNT = 2, GB_EMIT = 3, GB_VERIFY = 4, GB_FIRST = 5, GB_EMIT2 = 6,
                           GB_FILTER = 7 };
constexpr int kBucketRecs = 8;                                   // 64-B bucket flushes
constexpr unsigned long long kRecInvalid = ~0ull;                // padding slot of an aligned run (bit 63 set)
constexpr int kRecPartShift = 52;  // GB_EMIT2 records carry their partition in bits [52, 63) (bucketed plan: <= 52 record bits)
constexpr int kBucketMaxPartitions = 2040;  // P x (3 x 4 + 8 x 8) B + 4 KiB of flush lists per block <= 160 KiB
// accumulator kinds (acc_kind): 0 int64 sum, 1 double sum, 2 ordered-u64 min, 3 ordered-u64 max,
// 4 HLL registers (u8 [G][256]), 5 none (COUNT / AVG count share `counts`)
constexpr int kMaxGroupAggs = 8;

struct GroupColDev {
  const uint8_t *fwd;
  const int32_t *remap;      // dictId -> global id (null = identity)
  long long stride;          // Π global cardinalities of the previous group columns
  int32_t bits;
  int32_t reserved;
};

struct GroupAggDev {
  const uint8_t *fwd;
  const void *dict;          // int32 / int64 / double dictionary values
  const uint16_t *hll_lut;   // acc_kind 4: (register << 8 | rank) per dictId
  void *acc;                 // dense global accumulator array
  int32_t bits, acc_kind, value_kind;
  int32_t field_shift;       // GB_EMIT: bit position of this column's dictId in the record
  int32_t lds_off;           // GB_LDS / k_partition_reduce: byte offset of its LDS accumulator array
  int32_t affine;            // INT/LONG dictionary value(id) = affine_base + affine_step * id: k_partition_reduce
                             // sums dictIds (SUM) and hashes the value arithmetically (HLL) — no gathers
  long long affine_base, affine_step;
};

struct GroupSegment {
  const uint64_t *pre;       // AND-ed in before the leaves; null = all docs
  int64_t nwords;            // 0 = skip (EMPTY filter)
  int32_t num_docs;
  int32_t first_leaf, n_leaves;
  int32_t first_gcol, first_agg;
  int32_t reserved;
  int64_t ch_begin, ch_end;  // chunk window (see FusedSegment)
  const uint32_t *admitted;  // num.groups.limit: bitmap over keys admitted for THIS segment, null = all
};

struct GroupArgs {
  const GroupSegment *segs;
  const FusedStep *leaves;
  const GroupColDev *gcols;
  const GroupAggDev *aggs;
  int32_t nsegs, bps, n_gcols, n_aggs;
  int32_t mode, stage_bytes;  // stage: LDS bytes per wave for the leaves (staged_chunk_bytes(max leaf bits))
  long long G;
  unsigned long long *counts;  // u64 [G]
  unsigned long long *matched; // u64 [nsegs]: docs passing the filter per segment (numDocsScanned)
  uint32_t *first_doc;         // GB_FIRST: [nsegs][G] smallest matching doc per key (0xFFFFFFFF = absent)
  int32_t lds_acc_bytes;       // GB_LDS: per-block accumulator bytes (counts u32 [G] at 0, aggs at lds_off)
  int32_t shift;               // GB_COUNT / GB_EMIT: partition = key >> shift, local key = low bits
  int32_t P;                   // partitions
  int32_t split;               // GB_EMIT two-level: log2 partitions per coarse run (0 = records go straight to
                               // their partition runs); a block emits into run (key >> (shift + split))
  uint32_t *hist;              // GB_COUNT: [P][nblk] per-block partition counts (partition-major)
  const uint32_t *offsets;     // GB_EMIT: [P][nblk] exclusive record offsets
  const uint32_t *pstart;      // GB_EMIT two-level: [P + 1] partition starts (coarse run starts derive from them)
  unsigned long long *emit;    // GB_EMIT: records (two-level: in coarse (run, block) order)
  // hashed key space (LONG_MAP / ARRAY_MAP shapes: Π cardinalities too large for dense arrays): the key
  // is the slot of the tuple's 64-bit fingerprint in an open-addressing table of hcap (power of 2) slots
  unsigned long long *htable;  // [hcap] fingerprints, 0 = empty
  unsigned long long *reps;    // [hcap] first (segment << 32 | doc) of the slot (atomicMin)
  long long hcap;
  unsigned long long hseed;
  uint32_t *verify_err;        // GB_VERIFY: set when a doc's tuple differs from its slot's representative
  int32_t hashed;
  // GB_COUNT / GB_EMIT column prefetch: every column a doc needs (group columns, then the aggregated
  // columns pf_agg[c] for slots c >= n_gcols) is loaded for kGroupPfUnroll words before any is decoded;
  // pf_nc = number of slots (<= kGroupPfCols), 0 = off (per-column loop)
  int32_t pf_nc;
  int32_t pf_agg[4];
  int32_t nt_store;            // GB_EMIT / split: records stored with the non-temporal (streaming) policy
  int32_t lw;                  // GB_COUNT / GB_EMIT / GB_EMIT2 with pf_nc > 0: lane-owns-word reads (G < 2^32)
  uint64_t *filter_out;        // GB_COUNT: writes each segment's filter words here (GB_EMIT2 reads them back)
  int32_t aligned_runs;        // GB_EMIT2 (lane-owns-quarter sink): runs padded to multiples of kBucketRecs records
                               // (offsets from the padded counts): bucket flushes advance from the run start in
                               // aligned 64-B pieces, records that find their bucket full fill from the run end
                               // backwards, and the padding slots are written with kRecInvalid
  int32_t emit_block;          // GB_EMIT2 lane-owns-quarter: threads per block (512, or 1024 = group.emit_block)
  int64_t filter_stride;       // words per segment in filter_out
  // GB_LDS lane-owns-quarter: the doc count rides in the high bits of aggregation lds_pack's affine dictId sum
  // ((1 << lds_sbits) + dictId per doc: one LDS atomic for both); -1 = separate u32 counts
  int32_t lds_pack, lds_sbits;
  // GB_LDS lane-owns-quarter, <= 3 read columns: every segment's filter is at most one scan leaf of <= 12 bits (RANGE /
  // LUT64 / LUT, AND-ed with `pre`), evaluated on each quarter from its own lane-owns-quarter loads beside the group and
  // aggregated columns' (no LDS chunk staging and no wait for it; stage_bytes = 0)
  int32_t qfilter;
};
constexpr int kGroupPfCols = 4;
constexpr int kGroupLwMaxBits = 20;  // widest column the lane-owns-word decode handles
void launch_group_query(const GroupArgs &a, hipStream_t stream);
// Grid (blocks per segment x segments) the host sizes `hist` / `offsets` for.
int group_query_blocks_per_cu(const GroupArgs &a);
size_t group_query_lds_bytes(const GroupArgs &a);

struct PartitionReduceArgs {
  const unsigned long long *records;
  const uint32_t *pstart;      // [P + 1] first record of each partition
  int32_t P, shift, n_aggs, lds_bytes;
  int32_t wave_cnt_off;        // LDS byte offset of the per-wave count copies (8 waves x K u32)
  int32_t skip_invalid;        // records may be kRecInvalid padding (GB_EMIT2 aligned runs): skipped
  long long G;
  unsigned long long *counts;
  GroupAggDev aggs[kMaxGroupAggs];  // fwd unused; dict / hll_lut / acc / lds_off / acc_kind / field_shift / bits
};
void launch_partition_reduce(const PartitionReduceArgs &a, hipStream_t stream);

// ---------------------------------------------------------------- ring plan (group_ring.hip)
// Large dense key spaces without a histogram pass: k_group_ring (records into fixed-capacity regions [P][nblk][C],
// C for the busiest block's docs all matching; the filter evaluated per quarter, or GB_FILTER's words first) ->
// k_ring_reduce (one block per partition of 2^shift keys).
struct RingArgs {
  const GroupSegment *segs;
  const GroupColDev *gcols;
  const GroupAggDev *aggs;
  const FusedStep *leaves;       // nf > 0: each segment's top-level conjunction of nf scan leaves (quarter form)
  const int64_t *cstart;         // [nsegs + 1]: first global chunk of each segment's chunk window
  const uint64_t *filter;        // nf == 0: GB_FILTER's words, [nsegs][filter_stride]
  int64_t filter_stride;
  int64_t total_chunks;
  long long G;
  int32_t nsegs, n_gcols, nc, P;  // nc: columns read per doc (the group columns, then the pf_agg fields)
  int32_t pf_agg[4];
  int32_t shift, nblk;            // nblk: blocks of the launch (one per CU): block b owns chunks [T b / nblk, T (b+1) / nblk)
  uint32_t cap;                   // C: records per region
  int32_t nf;                     // < 0: the filter words; else at most nf scan leaves evaluated per quarter
  int32_t rec_bytes;              // 8, or 6 when the record fields fit 48 bits (the low 48 bits of each record stored)
  int32_t hll;                    // 1: the records leave the block with the field [hll_shift, + hll_bits) (an HLL column's
                                  // dictId, over an affine dictionary base + step * id with values in [0, 2^32)) replaced
                                  // by register << 5 | rank of its value (the flushers hash; the reduce does not)
  int32_t hll_shift, hll_bits;
  uint32_t hll_base, hll_step;
  uint8_t *records;               // [P][nblk][C] records of rec_bytes (local key | fields)
  uint32_t *hist;                 // [P][nblk] records claimed per region (> C: overflow)
  uint32_t *status;               // |= 1 a region overflowed, 2 a spin bound was hit, 4 HLL exception list full
  uint32_t *region;               // C, written by block 0 (read by k_ring_reduce)
  unsigned long long *matched;    // nf >= 0: [nsegs] docs passing the filter (numDocsScanned), added by the decoders
};
constexpr int kRingMaxQuarterLeaves = 2;
struct RingReduceArgs {
  const uint8_t *records;            // RingArgs.records
  int32_t rec_bytes;
  int32_t hll_pre;                   // bit g: aggregation g's field is the scatter's HLL register << 5 | rank
  const uint32_t *hist;
  const uint32_t *region;
  int32_t P, shift, n_aggs, nblk;
  int32_t lds_bytes, lds_zero_bytes;
  int32_t cnt_off, hist_off, exc_off;  // LDS: counts u32 [K], hist row u32 [nblk], exceptions (count + entries)
  int32_t hll_sums;  // 1: each HLL aggregation's array holds u64 [G] after its registers: Σ 2^(32 - register) in bits
                     // 0..47, the zero registers' count in bits 48..63 (k_group_final kind 9 reads them, not the registers)
  long long G;
  unsigned long long *counts;
  uint32_t *status;
  GroupAggDev aggs[kMaxGroupAggs];  // lds_off / acc_kind / field_shift / bits / dict / hll_lut / affine / acc
};
__host__ __device__ uint32_t ring_region_records(uint64_t max_block_docs, int64_t K, int64_t G, uint32_t cap);
size_t ring_lds_bytes(int P);  // k_group_ring's dynamic LDS
void launch_group_ring(const RingArgs &a, hipStream_t stream);
void launch_ring_reduce(const RingReduceArgs &a, hipStream_t stream);
int ring_reduce_exceptions();  // LDS exception entries per partition
// Two-level partitioned plan, second level: coarse run (q, b) of `runs` (2^split partitions' records
// emitted by block b) is split into the partitions' final slots offsets[p][b]... of `records`.
void launch_partition_split(const uint32_t *hist, const uint32_t *offsets, const uint32_t *pstart, int32_t P,
                            int32_t nblk, int32_t shift, int32_t split, const unsigned long long *runs,
                            unsigned long long *records, int nt_store, hipStream_t stream);
// pstart[p] = offsets[p * nblk] (partition-major exclusive offsets), pstart[P] = total records.
void launch_partition_starts(const uint32_t *offsets, const uint32_t *hist, int32_t P, int32_t nblk, uint32_t *pstart,
                             hipStream_t stream);
// out[i] = in[i] rounded up to a multiple of kBucketRecs (aligned runs of the bucketed EMIT)
void launch_pad_counts(const uint32_t *in, long long n, uint32_t *out, hipStream_t stream);
// Hashed key spaces: the global-id tuple of each listed slot's representative doc, ids[i * n_gcols + j].
void launch_hash_tuples(const GroupArgs &a, const long long *slots, long long n, int32_t *ids, hipStream_t stream);
// HLL registers of the listed keys: out[i * 256 + r] = regs[keys[i] * 256 + r].
void launch_gather_hll(const uint8_t *regs, const long long *keys, long long n, uint8_t *out, hipStream_t stream);
// out[i] = in[i] for n HLL registers (n % 4 == 0): the u8 multi-GPU partial layout <-> the bitset path's u32
void launch_widen_u8(const uint8_t *in, long long n, int32_t *out, hipStream_t stream);
void launch_narrow_u32(const uint32_t *in, long long n, uint8_t *out, hipStream_t stream);

// Device finalize of dense accumulators: ordered list of the non-empty keys (flags + exclusive scan +
// scatter; `scratch` holds 4 * (G + 1) bytes + the scan's temporary storage) and per-group outputs.
size_t compact_keys_scratch_bytes(long long G);
void launch_compact_keys_ordered(long long G, const unsigned long long *counts, long long *keys_out,
                                 unsigned long long *n_out, void *scratch, size_t scratch_bytes, hipStream_t stream);
// Final per-group arrays in the host result layout (k_group_final): out_keys[i] = keys[i] + key_base, out_counts,
// out_values[fn] (the function's intermediate value as a double) and out_card[fn] (DISTINCTCOUNTHLL cardinality,
// bit-identical to the host's hll_cardinality_from_sum). kind: 0 i64 sum, 1 f64 sum, 2/3 ordered min / max,
// 4 HLL u8 registers [G][256], 5 the count; acc: the accumulator the function reads (its primary's for aliases).
struct GroupFinalArgs {
  int32_t n;
  int32_t kind[kMaxGroupAggs];  // accumulator kinds; 9: an HLL's packed register sums (RingReduceArgs.hll_sums)
  const void *acc[kMaxGroupAggs];
  double *out_values[kMaxGroupAggs];
  long long *out_card[kMaxGroupAggs];
  long long *out_keys, *out_counts;
  long long key_base;
  double alpha_mm;
  const double *linear;  // device copy of m * log(m / z), z = 0..256 (z = 0: +inf)
  // compact read-back (optional): counts and cardinalities also as u32, *overflow set when one does not fit
  unsigned int *out_counts32;
  unsigned int *out_card32[kMaxGroupAggs];
  unsigned int *overflow;
};
// Server-side trimming on the device (AggregationGroupByTrimmingService.trimIntermediateResultsMap :71-116): per function,
// flags[g] |= bit for the T best groups of its comparable values (vals = k_group_final's out_values; avg: / counts;
// asc: MIN), ties in ascending group order; then the union of flagged groups compacted in group order.
size_t trim_scratch_bytes(long long n);
void launch_trim_select(const double *vals, const long long *counts, int avg, int asc, long long n, long long T,
                        uint32_t bit, uint32_t *flags, void *scratch, size_t scratch_bytes, hipStream_t stream);
void launch_trim_union(const uint32_t *flags, const long long *keys, long long n, long long *keys_out,
                       uint32_t *flags_out, unsigned long long *n_out, void *scratch, size_t scratch_bytes,
                       hipStream_t stream);
// bit k of bits[k >> 6] = counts[k] != 0 (the non-empty keys the compaction lists, as a bitmap)
void launch_key_bitmap(const unsigned long long *counts, long long G, uint64_t *bits, hipStream_t stream);
void launch_group_final(const unsigned long long *counts, const long long *keys, long long n, const GroupFinalArgs &f,
                        hipStream_t stream);
// num.groups.limit admission (DictionaryBasedGroupKeyGenerator IntMapBasedHolder.getGroupId, first appearance):
// segment s admits the upper[s] keys with the smallest first_doc[s][k] (first_doc values of distinct keys are
// distinct docs). bitmaps[s] (words u32 each) gets bit k for every admitted key; upper[s] >= G admits every present
// key. One radix sort of first_doc[s] per limited segment; the threshold never leaves the device.
size_t admission_scratch_bytes(long long G);
void launch_admission_bitmaps(const uint32_t *first_doc, int S, long long G, const long long *upper, uint32_t *bitmaps,
                              long long words, void *scratch, size_t scratch_bytes, hipStream_t stream);

// Exclusive prefix sum of n u32 (hipcub); returns the temporary storage it needs when tmp == null.
size_t exclusive_sum_u32(const uint32_t *in, uint32_t *out, long long n, void *tmp, size_t tmp_bytes,
                         hipStream_t stream);

// Sorted-index leaf: ranges (inclusive [start, end], sorted, disjoint) -> bitset (combine mode as k_leaf).
void launch_ranges_to_bitset(const int32_t *ranges, int32_t nranges, int64_t nwords, int32_t num_docs,
                             int32_t mode, uint64_t *out, hipStream_t stream);

// Roaring container descriptor, built on the host at segment registration.
struct RoaringContainer {
  uint64_t payload_offset;  // byte offset into the inverted-index payload
  uint32_t cardinality;
  uint16_t key;             // high 16 bits of the docIds
  uint16_t type;            // 0 array, 1 bitmap, 2 run (runs: cardinality = run count)
};

// Bitmap-inverted-index leaf: OR of the containers of `ids` (exclusive: flip), combined into out by mode.
void launch_roaring_expand(const uint8_t *payload, const RoaringContainer *containers, const int32_t *dir,
                           const int32_t *ids, int32_t nids, int exclusive, int64_t nwords, int32_t num_docs,
                           int32_t mode, uint64_t *out, hipStream_t stream);
// Bitset algebra: dst = dst (op) src, or a fill (all-ones / zeros) for MATCH_ALL / EMPTY children.
void launch_bitset_combine(uint64_t *dst, const uint64_t *src, int64_t nwords, int32_t num_docs, int32_t mode,
                           int32_t fill, hipStream_t stream);

struct AggSpecDev {
  int32_t kind;
  int32_t col;            // index into GroupByProgram::cols
  const void *dict;       // int32 / int64 / double dictionary
  const uint16_t *hll_lut;
};

// Group-by over docs selected by bitset (null = all docs).
struct GroupByProgram {
  int32_t n_gcols;
  int32_t n_aggs;
  int32_t n_cols;
  DevColumn cols[kMaxProgramColumns];
  int32_t gcol[kMaxGroupCols];          // column index of group column j (j = 0 least significant)
  const int32_t *remap[kMaxGroupCols];  // dictId -> global id (null = identity)
  long long stride[kMaxGroupCols];      // Π_{k<j} global card_k
  AggSpecDev aggs[kMaxAggs];
  const uint32_t *admitted;             // bitmap over keys (null = all admitted)
  unsigned long long *counts;           // u64[G]
  void *acc[kMaxAggs];                  // per agg accumulator array
  int32_t acc_kind[kMaxAggs];           // 0 i64 sum, 1 f64 sum, 2 ordered min, 3 ordered max, 4 HLL u32[256], 5 none
  int32_t value_kind[kMaxAggs];         // dictionary type: 0 int32, 1 int64, 2 double
};
void launch_group_by(const GroupByProgram &prog, const uint64_t *bitset, int64_t nwords, int32_t num_docs,
                     hipStream_t stream);
// Group-by over multi-value group columns and / or MV aggregations (DefaultGroupByExecutor.process with
// DictionaryBasedGroupKeyGenerator.generateKeysForBlock(MV), :213-240, and aggregateGroupByMV): one lane per doc;
// the doc's group keys are the cartesian product of its group columns' entries (duplicates included); every key
// takes count + 1 and each function folds all entries of its column. acc_kind 6 adds the doc's entry count
// (CountMV). Columns are (packed fwd, bits, row starts or null for single-value).
struct MvGroupArgs {
  int32_t n_gcols, n_aggs;
  const uint8_t *gfwd[kMaxGroupCols];
  const uint32_t *goff[kMaxGroupCols];
  int32_t gbits[kMaxGroupCols];
  const int32_t *remap[kMaxGroupCols];
  long long stride[kMaxGroupCols];
  const uint8_t *afwd[kMaxAggs];
  const uint32_t *aoff[kMaxAggs];
  int32_t abits[kMaxAggs];
  const void *dict[kMaxAggs];
  const uint16_t *hll_lut[kMaxAggs];
  int32_t acc_kind[kMaxAggs];   // 0 i64 sum (INT), 1 f64 sum, 2 ordered min, 3 ordered max, 4 HLL u32[256], 5 none,
                                // 6 entry count, 7 i64 sum (int64 dictionary)
  int32_t value_kind[kMaxAggs];
  unsigned long long *counts;
  void *acc[kMaxAggs];
  const uint64_t *bitset;       // null = all docs
  int64_t nwords;
  int32_t num_docs;
  int32_t reserved;
  const uint32_t *admitted;     // num.groups.limit: keys admitted for this segment (bitmap), null = all
};
void launch_group_by_mv(const MvGroupArgs &a, hipStream_t stream);
// MV first appearance (DictionaryBasedGroupKeyGenerator IntMapBasedHolder.processMultiValue :282-300 over getIntRawKeys
// :344-410): first_pos[key] = min over matching docs of (doc << 32 | position of the key in the doc's raw-key list),
// the list ordered as getIntRawKeys builds it (the highest-index multi-value column fastest).
void launch_first_pos_mv(const MvGroupArgs &a, unsigned long long *first_pos, hipStream_t stream);
// admitted bit k = first_pos[k] among the `upper` smallest (every present key when upper >= G); one radix sort
size_t admission_scratch_bytes_u64(long long G);
void launch_admission_bitmap_u64(const unsigned long long *first_pos, long long G, long long upper, uint32_t *bitmap,
                                 long long words, void *scratch, size_t scratch_bytes, hipStream_t stream);
// First matching doc per key (atomicMin), for the num.groups.limit first-appearance rule.
void launch_first_doc(const GroupByProgram &prog, const uint64_t *bitset, int64_t nwords, int32_t num_docs,
                      uint32_t *first_doc, hipStream_t stream);
// Gather counts / 64-bit accumulators (out_acc[a * n + i]) / HLL registers (u8, out_hll[(h * n + i) * 256]).
void launch_gather_groups(const GroupByProgram &prog, const long long *keys, int64_t n, unsigned long long *out_counts,
                          unsigned long long *out_acc, uint8_t *out_hll, hipStream_t stream);
// Compact non-empty keys: writes keys[] (unordered) and *n.
void launch_compact_keys(int64_t G, const unsigned long long *counts, long long *keys_out,
                         unsigned long long *n_out, hipStream_t stream);

// Synthetic column (bench tooling): value(d) = d < card ? d : splitmix64(seed ^ d*phi) % card, packed.
void launch_synth_column(uint64_t seed, int32_t card, int32_t bits, int32_t num_docs, uint8_t *out,
                         hipStream_t stream);
// Sorted column -> packed forward index from per-dictId start docs (starts[card] = num_docs).
void launch_sorted_to_fwd(const int32_t *starts, int32_t card, int32_t bits, int32_t num_docs, uint8_t *out,
                          hipStream_t stream);

}  // namespace pinot
