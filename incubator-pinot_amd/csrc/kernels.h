// Kernel argument blocks and launch entry points (implemented in kernels.hip).
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

constexpr int kMaxProgramColumns = 16;
constexpr int kMaxProgramInstr = 48;
constexpr int kMaxStack = 8;
constexpr int kMaxAggs = 8;
constexpr int kMaxGroupCols = 8;
constexpr int kBlock = 256;

struct DevColumn {
  const uint8_t *fwd;  // packed forward index (BE, MSB-first)
  int32_t bits;
  int32_t card;
};

enum FilterOp : int32_t {
  OP_LEAF_RANGE = 0,   // dictId in [a, b)            (flags & 1: negate)
  OP_LEAF_LUT = 1,     // bit dictId of luts[a ..]     (flags & 1: negate)
  OP_LEAF_BITSET = 2,  // precomputed bitset slot a
  OP_AND = 3,          // pop a, push AND
  OP_OR = 4,           // pop a, push OR
  OP_ALL = 5,          // push all-ones (match all)
  OP_NONE = 6          // push zero (empty)
};

struct FilterInstr {
  int32_t op;
  int32_t col;  // index into FilterProgram::cols
  int32_t a;
  int32_t b;
  int32_t flags;
};

struct FilterProgram {
  int32_t n_instr;
  int32_t n_cols;
  FilterInstr ins[kMaxProgramInstr];
  DevColumn cols[kMaxProgramColumns];
  const uint32_t *luts;     // concatenated dictId-membership bitmaps
  const uint64_t *bitsets;  // slot s at bitsets + s * bitset_stride
  int64_t bitset_stride;    // words per slot
};

// Filter scan: evaluates the program for every 64-doc word, writes the final bitset
// (may be null) and adds the number of matching docs into *count.
void launch_filter_scan(const FilterProgram &prog, int64_t nwords, int32_t num_docs, uint64_t *out_bitset,
                        unsigned long long *count, hipStream_t stream);

// Sorted-index leaf: ranges (inclusive [start, end], sorted, disjoint) -> bitset.
void launch_ranges_to_bitset(const int32_t *ranges, int32_t nranges, int64_t nwords, int32_t num_docs,
                             uint64_t *out, hipStream_t stream);

// Roaring container descriptor, built on the host at segment registration.
struct RoaringContainer {
  uint64_t payload_offset;  // byte offset into the inverted-index payload
  uint32_t cardinality;
  uint16_t key;             // high 16 bits of the docIds
  uint16_t type;            // 0 array, 1 bitmap, 2 run (runs: cardinality = run count)
};

// Bitmap-inverted-index leaf: OR of the containers of `ids` (exclusive: flip the result).
void launch_roaring_expand(const uint8_t *payload, const RoaringContainer *containers, const int32_t *dir,
                           const int32_t *ids, int32_t nids, int exclusive, int64_t nwords, int32_t num_docs,
                           uint64_t *out, hipStream_t stream);

enum AggKind : int32_t {
  AGG_SUM_I32 = 0,   // int64 sum of an int32 dictionary
  AGG_SUM_I64 = 1,   // double sum of an int64 dictionary
  AGG_SUM_F64 = 2,   // double sum of a double dictionary
  AGG_MINMAX = 3,    // min / max dictId
  AGG_HLL = 4,       // registers via per-dictId (register << 8 | rank) LUT
  AGG_NOP = 5
};

struct AggSpecDev {
  int32_t kind;
  int32_t col;            // index into AggProgram::cols
  const void *dict;       // int32 / int64 / double dictionary
  const uint16_t *hll_lut;
};

struct AggPartial {          // one per workgroup per aggregation
  long long sum_i64;
  double sum_f64;
  int32_t min_id;
  int32_t max_id;
};

struct AggProgram {
  int32_t n_aggs;
  int32_t n_cols;
  AggSpecDev aggs[kMaxAggs];
  DevColumn cols[kMaxProgramColumns];
};

// Aggregation over docs selected by bitset (null = all docs). Writes `grid` partials per agg
// (partials[agg * grid + block]) and HLL registers (hll_regs[agg * 256 + j], atomicMax).
int launch_aggregate(const AggProgram &prog, const uint64_t *bitset, int64_t nwords, int32_t num_docs,
                     AggPartial *partials, uint32_t *hll_regs, hipStream_t stream);
int aggregate_grid(int64_t nwords);

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
// First matching doc per key (atomicMin), for the num.groups.limit first-appearance rule.
void launch_first_doc(const GroupByProgram &prog, const uint64_t *bitset, int64_t nwords, int32_t num_docs,
                      uint32_t *first_doc, hipStream_t stream);

void launch_reduce_partials(const AggPartial *in, int grid, int n_aggs, AggPartial *out, hipStream_t stream);
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
