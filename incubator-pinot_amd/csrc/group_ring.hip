// Ring-partitioned group-by (the large-key-space plan, config 4): no histogram pass, fixed-capacity regions.
//
//   k_group_ring         one block of 12 waves per CU over a contiguous range of chunks. Waves 0..7 (decoders, two per
//                        SIMD) read each 1024-doc quarter lane-owns-quarter (lane l: docs 16l .. 16l + 15), evaluate the
//                        segment's top-level conjunction of scan leaves on it (or take GB_FILTER's words for other
//                        filter shapes), decode the group key and aggregated dictIds into u64 records (local key |
//                        dictId fields) and append each to its partition's LDS bucket of 16 entries (two halves of 8):
//                        one LDS add claims an entry, so a decoder never issues an HBM store (its vmcnt holds its own
//                        loads only). Waves 8..11 (flushers, one per SIMD) move every completed half to the block's
//                        region of that partition as one aligned 64-B piece, between block barriers: region
//                        (p, block) holds records [0, n) in claim order, so no histogram, scan or cursor leaves the CU.
//   k_ring_reduce        one block per partition of K <= 1024 consecutive keys: the partition's records from every
//                        block's region folded into LDS accumulators (count packed beside the first affine dictId
//                        SUM, int64 / double sums, ordered min / max, HLL registers as 4-bit nibbles with the rare
//                        rank > 15 kept in an exception list), then written to the dense arrays with plain stores.
//
// Restates DictionaryBasedGroupKeyGenerator.generateKeysForBlock (raw key = mixed radix over the group columns'
// dictIds, PC/query/aggregation/groupby/DictionaryBasedGroupKeyGenerator.java:195-302) and DefaultGroupByExecutor
// .process / aggregateGroupBySV (PC/query/aggregation/groupby/DefaultGroupByExecutor.java:70-168); the quarter-form
// filter restates ScanBasedFilterOperator over the dictionary predicate evaluators (fused_common.h). Regions are sized
// for every doc of the busiest block matching with uniform keys; a partition whose records exceed its region (skewed
// keys) sets a status bit and the host answers the query on the counted plan instead (executor.cpp).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "fused_common.h"
#include "group_lq.h"
#include "group_ring.h"

namespace pinot {

// Records per region: the busiest block's docs spread over the partitions by key share, + 12.5 % + 64, a multiple of
// 16 (128-B aligned regions), never above the allocation.
__host__ __device__ uint32_t ring_region_records(uint64_t max_block_docs, int64_t K, int64_t G, uint32_t cap) {
  const uint64_t mean = (max_block_docs * (uint64_t)K + (uint64_t)G - 1) / (uint64_t)G;
  uint64_t c = mean + mean / 8 + 64;
  c = (c + 15) & ~15ull;
  return (uint32_t)(c < cap ? c : cap);
}

namespace {
using namespace dev;

constexpr int kRingBlock = 768;                             // one block of 12 waves per CU (the buckets take the LDS)
constexpr int kRingWaves = kRingBlock / 64;
constexpr int kRingFlushWaves = 4;                           // waves 8..11: the flush phases (one per SIMD)
constexpr int kRingDecWaves = kRingWaves - kRingFlushWaves;  // waves 0..7: filter, decode, insert (two per SIMD)
constexpr int kRingRoundRecs = 8;                            // records per decoder lane between two flush phases
constexpr int kRingBucket = 16;                              // entries per partition bucket (two 64-B halves)
// Bucket stride in entries: 144 B = 36 dwords, so the flushers' 16-B reads of consecutive partitions start on distinct
// banks (a 128-B stride puts every lane of a ds_read_b128 group on the same four banks) and an insert's 8-B write lands
// on a bank set by its partition, not only by its slot.
constexpr int kRingBucketStride = 18;
constexpr int kRecPShift = 53;                               // bucket entries carry their partition in bits [53, 63)
constexpr int kRingBackBits = 12;                            // hist: front count (20 bits) | back count << 20
static_assert(16 % kRingRoundRecs == 0, "whole rounds per pass");

// stream-lib MurmurHash.hashLong + HyperLogLog (register << 8 | rank): hll.cpp's murmur_hash_long / hll_register_rank
__device__ __forceinline__ uint32_t murmur_hash_long_g(long long data) {
  constexpr uint32_t kM = 0x5bd1e995u;
  const unsigned long long d = (unsigned long long)data;
  uint32_t h = 0;
  uint32_t k = (uint32_t)d * kM;
  k ^= k >> 24;
  h ^= k * kM;
  k = (uint32_t)(d >> 32) * kM;
  k ^= k >> 24;
  h *= kM;
  h ^= k * kM;
  h ^= h >> 13;
  h *= kM;
  h ^= h >> 15;
  return h;
}

// murmur_hash_long_g of a value in [0, 2^32): the high word's block multiplies h by kM once more
__device__ __forceinline__ uint32_t murmur_hash_lo32_g(uint32_t lo) {
  constexpr uint32_t kM = 0x5bd1e995u, kMM = kM * kM;
  uint32_t k = lo * kM;
  k ^= k >> 24;
  uint32_t h = k * kMM;
  h ^= h >> 13;
  h *= kM;
  h ^= h >> 15;
  return h;
}

__device__ __forceinline__ uint32_t hll_register_rank_g(uint32_t h) {
  return ((h >> 24) << 8) | (uint32_t)(__builtin_clz((h << 8) | 129u) + 1);
}

// The record field of an HLL aggregation whose (register, rank) the scatter computes (RingArgs.hll): the value
// base + step * dictId (< 2^32) of an affine dictionary hashed as stream-lib does, kept as register << 5 | rank (13 bits)
__device__ __forceinline__ uint32_t hll_field_g(uint32_t id, uint32_t base, uint32_t step) {
  const uint32_t h = murmur_hash_lo32_g(base + step * id);
  return ((h >> 24) << 5) | (uint32_t)(__builtin_clz((h << 8) | 129u) + 1);
}

// A record on its way out of the block (a flush, the final partial flush, a bucket-overflow write): its HLL field's
// dictId replaced by hll_field_g of it. The flusher waves do this between their barriers, so the hash costs the
// decoders nothing (they wait at barriers far less than the flushers, round 5).
__device__ __forceinline__ unsigned long long ring_hll_out(const RingArgs &a, unsigned long long r) {
  const unsigned long long m = ((1ull << a.hll_bits) - 1ull) << a.hll_shift;
  const uint32_t id = (uint32_t)((r & m) >> a.hll_shift);
  return (r & ~m) | ((unsigned long long)hll_field_g(id, a.hll_base, a.hll_step) << a.hll_shift);
}

struct RingLds {
  unsigned long long *bkt;  // [P][16] bucket entries: record | partition << 53
  uint32_t *ctr;            // [P]: entries in the bucket (bits 0-15; claims beyond 16 overflowed) | head (0 / 8) << 16
  uint32_t *back;           // [P]: records written from the region's end (bucket overflow)
  uint32_t *list;           // [flusher waves][kRingListPerWave]: the flush phase's listed halves
};

__device__ __forceinline__ RingLds ring_lds(uint8_t *lds, int P) {
  RingLds r;
  r.bkt = reinterpret_cast<unsigned long long *>(lds);
  r.ctr = reinterpret_cast<uint32_t *>(r.bkt + (size_t)P * kRingBucketStride);
  r.back = r.ctr + P;
  r.list = r.back + P;
  return r;
}

__device__ __forceinline__ uint32_t rec_part(unsigned long long r) { return (uint32_t)(r >> kRecPShift) & 1023u; }

// Record i of a region array of RB-byte records (RB = 6: the low 48 bits, as three 16-bit stores).
template <int RB>
__device__ __forceinline__ void store_rec(uint8_t *base, size_t i, unsigned long long v) {
  if constexpr (RB == 8) {
    reinterpret_cast<unsigned long long *>(base)[i] = v;
  } else {
    uint16_t *d = reinterpret_cast<uint16_t *>(base + i * 6);
    d[0] = (uint16_t)v;
    d[1] = (uint16_t)(v >> 16);
    d[2] = (uint16_t)(v >> 32);
  }
}

// Insert phase: record j of each of the lane's kRingRoundRecs records (J0 ..) claims the next entry of its partition's
// bucket (one LDS add returns the claim index and the head) and is written at (head + claim) mod 16. No flush runs
// during an insert phase (block barriers on both sides), so a claim below 16 always finds its entry free; a claim of
// 16 or more (a bucket that received more than 9 records in one round; rare) goes to the back of its region instead.
template <int RB, bool HLL, int J0>
__device__ __forceinline__ void ring_insert(const RingArgs &a, const RingLds &L, uint32_t act,
                                            const unsigned long long (&rec)[16], uint8_t *region0,
                                            uint32_t C) {
  uint32_t old[kRingRoundRecs], p[kRingRoundRecs];
#pragma unroll
  for (int j = 0; j < kRingRoundRecs; j++) {
    const bool on = (act >> (J0 + j)) & 1u;
    p[j] = on ? rec_part(rec[J0 + j]) : 0u;  // branch-free: an inactive record adds 0 to partition 0's counter
    old[j] = atomicAdd(L.ctr + p[j], on ? 1u : 0u);
  }
  uint32_t over = 0;
#pragma unroll
  for (int j = 0; j < kRingRoundRecs; j++) {
    const bool on = (act >> (J0 + j)) & 1u;
    const uint32_t s = old[j] & 0xFFFFu, h = old[j] >> 16;
    if (on && s < (uint32_t)kRingBucket)
      L.bkt[p[j] * kRingBucketStride + ((h + s) & (kRingBucket - 1))] = rec[J0 + j];
    over |= (on && s >= (uint32_t)kRingBucket) ? (1u << j) : 0u;
  }
  if (__any(over != 0)) {  // uniform, rare
#pragma unroll
    for (int j = 0; j < kRingRoundRecs; j++)
      if ((over >> j) & 1u) {
        const uint32_t k = atomicAdd(L.back + p[j], 1u);
        if (k < C) {
          unsigned long long r = rec[J0 + j] & ((1ull << kRecPShift) - 1ull);
          if constexpr (HLL) r = ring_hll_out(a, r);
          store_rec<RB>(region0, ((size_t)p[j] * a.nblk + 1) * C - 1 - k, r);
        }
      }
  }
}

// A flushed 16-B piece of a region: a plain store, so L2 merges a region's two 64-B halves into one line before it
// writes the line back (measured 2 % faster than non-temporal stores, r05p).
// RB = 6: two 8-B entries (x, y | z, w; the record in the low 48 bits of each) packed into 12 B. (sizeof(u32x3a) is 16:
// never index an array of them, address 12-B units in bytes.)
typedef uint32_t u32x3a __attribute__((ext_vector_type(3), aligned(4)));
template <int RB>
__device__ __forceinline__ void ring_store(u32x4 v, uint8_t *dst) {
  if constexpr (RB == 8) {
    *reinterpret_cast<u32x4 *>(dst) = v;
  } else {
    u32x3a z;
    z.x = v.x;
    z.y = (v.y & 0xFFFFu) | (v.z << 16);
    z.z = (v.z >> 16) | (v.w << 16);
    *reinterpret_cast<u32x3a *>(dst) = z;
  }
}

// Flush phase (flusher waves only, between two block barriers): every bucket holding 8 or more entries moves its
// oldest half (entries head .. head + 7: one aligned 64-B piece of LDS) to the front of its region at the partition's
// front cursor (64-B aligned: regions start 128-B aligned and the front advances by 8 records), then the head moves
// to the other half. Lane l of flusher wave fw owns partitions fw * 64 + l + 256 k and keeps their front cursors; it
// lists the complete halves of two of its partitions at a time in the wave's LDS list (a ballot gives each its slot),
// then every store instruction writes 16 listed halves with four lanes each, all 64 lanes active: the scatter's stores
// share the CU's vector-memory path with the decoders' loads, so fewer store instructions per flushed byte let the
// loads issue sooner (k_group_ring 5.59 -> 5.09 ms against one lane storing each of its halves, r05s).
constexpr int kRingListPerWave = 64 * 2 * 2;  // 2 partitions per lane per batch, <= 2 halves each
template <int RB, bool HLL, int KP>
__device__ __forceinline__ void ring_flush_phase(const RingArgs &a, const RingLds &L, uint8_t *region0,
                                                 uint32_t C, int fw, int lane, uint32_t (&front)[KP],
                                                 uint32_t &status) {
  uint32_t *list = L.list + fw * kRingListPerWave;
  const u32x4 m = {0xFFFFFFFFu, 0x001FFFFFu, 0xFFFFFFFFu, 0x001FFFFFu};  // strip the partition bits
  const int sub = lane & 3;
#pragma unroll
  for (int k0 = 0; k0 < KP; k0 += 2) {
    uint32_t c[2];
#pragma unroll
    for (int kk = 0; kk < 2; kk++) {
      const int p = fw * 64 + lane + 64 * kRingFlushWaves * (k0 + kk);
      c[kk] = (k0 + kk < KP && p < a.P) ? L.ctr[p] : 0u;
    }
    uint32_t base = 0;
#pragma unroll
    for (int kk = 0; kk < 2; kk++) {
      const int k = k0 + kk;
      if (k >= KP) break;
      const int p = fw * 64 + lane + 64 * kRingFlushWaves * k;
      uint32_t n = min(c[kk] & 0xFFFFu, (uint32_t)kRingBucket), h = c[kk] >> 16;
#pragma unroll
      for (int j = 0; j < 2; j++) {
        const bool full = n >= 8u;
        const unsigned long long bal = __ballot(full);
        if (full) {
          const uint32_t pos = base + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
          const bool ok = front[k] + 8u <= C;
          if (!ok) status |= 1u;  // region full: the query falls back to the counted plan
          // entry: front (20 bits) | head half (1) | partition (10) | stored (1)
          list[pos] = (front[k] & 0xFFFFFu) | ((h >> 3) << 20) | ((uint32_t)p << 21) | (ok ? 0x80000000u : 0u);
          front[k] += 8u;
          h ^= 8u;
          n -= 8u;
        }
        base += (uint32_t)__popcll(bal);
      }
      if ((c[kk] & 0xFFFFu) >= 8u) L.ctr[p] = (h << 16) | n;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (uint32_t i = (uint32_t)(lane >> 2); i < base; i += 16) {
      const uint32_t ent = list[i];
      const uint32_t p = (ent >> 21) & 1023u, fr = ent & 0xFFFFFu, hh = ((ent >> 20) & 1u) * 8u;
      const u32x4 x = reinterpret_cast<const u32x4 *>(L.bkt + p * kRingBucketStride + hh)[sub];
      if (ent >> 31) {
        u32x4 y = x & m;
        if constexpr (HLL) {
          const unsigned long long r0 = ring_hll_out(a, ((unsigned long long)y.y << 32) | y.x),
                                   r1 = ring_hll_out(a, ((unsigned long long)y.w << 32) | y.z);
          y.x = (uint32_t)r0;
          y.y = (uint32_t)(r0 >> 32);
          y.z = (uint32_t)r1;
          y.w = (uint32_t)(r1 >> 32);
        }
        ring_store<RB>(y, region0 + ((size_t)p * a.nblk * C + fr) * RB + sub * (2 * RB));
      }
    }
    __builtin_amdgcn_wave_barrier();  // the list is rewritten by the next batch
  }
}


// Segment of global chunk c (the chunk windows of the segments, concatenated in order): uniform scalar scan forward
// from g0, a segment at or before c's (a wave's chunks ascend, so the scan usually stops at once).
__device__ __forceinline__ int ring_segment(const RingArgs &a, int64_t c, int g0 = 0) {
  int g = g0;
  while (g + 1 < a.nsegs && load_const(a.cstart + g + 1) <= c) g++;
  return g;
}

// Lane l of quarter q takes docs 1024q + 16l .. +15: bits 16(l & 3) .. of the chunk word 16q + l/4.
__device__ __forceinline__ uint32_t quarter_bits(uint64_t word, int q, int lane) {
  const int src = 16 * q + (lane >> 2);
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)word, src, 64);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(word >> 32), src, 64);
  return (((lane & 2) ? hi : lo) >> (16 * (lane & 1))) & 0xFFFFu;
}

// Column slots of the ring decoder: [0, kRingGroupCols) group columns, then kRingAggCols aggregated columns (the
// distinct accumulators' fields); bits 0 = unused slot.
struct RingColsDev {
  const uint8_t *fwd[kRingGroupCols + kRingAggCols];
  const int32_t *remap[kRingGroupCols];
  uint32_t stride[kRingGroupCols];
  int bits[kRingGroupCols + kRingAggCols], fsh[kRingGroupCols + kRingAggCols];
};

__device__ __forceinline__ RingColsDev ring_cols(const RingArgs &a, const GroupSegment &sg) {
  RingColsDev k;
#pragma unroll
  for (int c = 0; c < kRingGroupCols + kRingAggCols; c++) {
    k.fwd[c] = nullptr;
    k.bits[c] = 0;
    k.fsh[c] = 0;
  }
#pragma unroll
  for (int c = 0; c < kRingGroupCols; c++) {
    k.remap[c] = nullptr;
    k.stride[c] = 0;
    if (c < a.n_gcols) {
      const GroupColDev gc = load_const(a.gcols + sg.first_gcol + c);
      k.fwd[c] = gc.fwd;
      k.remap[c] = gc.remap;
      k.stride[c] = (uint32_t)gc.stride;
      k.bits[c] = gc.bits;
    }
  }
#pragma unroll
  for (int c = 0; c < kRingAggCols; c++)
    if (a.n_gcols + c < a.nc && a.pf_agg[a.n_gcols + c] >= 0) {
      const GroupAggDev ag = load_const(a.aggs + sg.first_agg + a.pf_agg[a.n_gcols + c]);
      k.fwd[kRingGroupCols + c] = ag.fwd;
      k.bits[kRingGroupCols + c] = ag.bits;
      k.fsh[kRingGroupCols + c] = ag.field_shift;
    }
  return k;
}

// Values J0 .. JE - 1 of a lane's quarter (group_lq.h decode_quarter_apply over a sub-range).
template <int B, int J, int JE, typename F>
__device__ __forceinline__ void ring_quarter_apply(const uint32_t (&D)[(B + 1) / 2 + 1], F &f) {
  constexpr int q = J * B, k = q >> 5, o = q & 31;
  constexpr uint32_t mask = (uint32_t)((1ull << B) - 1ull);
  if constexpr (o + B <= 32) f.template put<J>((D[k] >> (32 - o - B)) & mask);
  else f.template put<J>(__builtin_amdgcn_alignbit(D[k], D[k + 1], 64 - o - B) & mask);
  if constexpr (J + 1 < JE) ring_quarter_apply<B, J + 1, JE>(D, f);
}

// Lane-owns-quarter decode that hands values J0 .. JE - 1 of the lane's 16 to f.put<J>(v) as they are extracted (no
// 16-value array: the decoders' registers go to the raw dwords of the columns in flight); only the dwords those values
// span are byte-swapped. The raw dwords pass through an empty volatile asm first, so the compiler cannot hoist the byte
// swaps of every width of the switch above it.
template <int B, int J0, int JE, typename F>
__device__ __forceinline__ void ring_decode_b(const uint32_t (&Rin)[12], int64_t qi, F &f) {
  constexpr int N = (B + 1) / 2 + (B & 1);
  // the dwords the values span (odd widths: + the 16-bit shift of odd quarters), as sources of the last alignbit too
  constexpr int LO = (J0 * B) >> 5, HI = ((JE * B + 15) >> 5) + 2 < N ? ((JE * B + 15) >> 5) + 2 : N;
  uint32_t D[(B + 1) / 2 + 1];
#pragma unroll
  for (int i = 0; i < (B + 1) / 2 + 1; i++) D[i] = 0;
#pragma unroll
  for (int i = LO; i < HI; i++) {
    uint32_t r = Rin[i];
    asm volatile("" : "+v"(r));
    D[i] = bswap32(r);
  }
  if constexpr (B & 1) {
    if (qi & 1) {
#pragma unroll
      for (int i = LO; i + 1 < HI; i++) D[i] = __builtin_amdgcn_alignbit(D[i], D[i + 1], 16);
    }
  }
  ring_quarter_apply<B, J0, JE>(D, f);
}

template <int J0, int JE, typename F>
__device__ __forceinline__ void ring_decode(const uint32_t (&R)[12], int bits, int64_t qi, F &f) {
#define PINOT_RD(B) ring_decode_b<B, J0, JE>(R, qi, f)
  switch (bits) {  // widths up to kGroupLwMaxBits (plan_ring checks)
    case 1: PINOT_RD(1); break;   case 2: PINOT_RD(2); break;   case 3: PINOT_RD(3); break;   case 4: PINOT_RD(4); break;
    case 5: PINOT_RD(5); break;   case 6: PINOT_RD(6); break;   case 7: PINOT_RD(7); break;   case 8: PINOT_RD(8); break;
    case 9: PINOT_RD(9); break;   case 10: PINOT_RD(10); break; case 11: PINOT_RD(11); break; case 12: PINOT_RD(12); break;
    case 13: PINOT_RD(13); break; case 14: PINOT_RD(14); break; case 15: PINOT_RD(15); break; case 16: PINOT_RD(16); break;
    case 17: PINOT_RD(17); break; case 18: PINOT_RD(18); break; case 19: PINOT_RD(19); break; case 20: PINOT_RD(20); break;
    default: break;
  }
#undef PINOT_RD
}

struct RingKeyFold {  // key += global id * stride (DictionaryBasedGroupKeyGenerator's mixed radix)
  uint32_t (&key)[16];
  const int32_t *remap;
  uint32_t stride;
  template <int J>
  __device__ __forceinline__ void put(uint32_t id) {
    key[J] += (remap ? (uint32_t)gload<int32_t>(remap + id) : id) * stride;
  }
};

struct RingFieldFold {  // record |= dictId << field shift
  unsigned long long (&rec)[16];
  int shift;
  template <int J>
  __device__ __forceinline__ void put(uint32_t id) {
    rec[J] |= (unsigned long long)id << shift;
  }
};


// The fields of a quarter-form scan leaf (FusedStep) the decoders keep in scalar registers.
struct RingLeaf {
  const uint8_t *fwd;
  const uint32_t *table;
  uint64_t lut64;
  uint32_t lo, span;
  int32_t bits, kind, negate;
};

__device__ __forceinline__ RingLeaf ring_leaf(const FusedStep *p) {
  RingLeaf l;
  const FusedStep st = load_const(p);
  l.fwd = st.fwd;
  l.table = static_cast<const uint32_t *>(st.table);
  l.lut64 = st.lut64;
  l.lo = st.lo;
  l.span = st.span;
  l.bits = st.bits;
  l.kind = st.kind;
  l.negate = st.negate;
  return l;
}

struct RingLeafFold {  // bit J of m = the leaf's predicate on value J (FusedStep, fused_common.h leaf_half)
  const RingLeaf &st;
  uint32_t &m;
  template <int J>
  __device__ __forceinline__ void put(uint32_t id) {
    uint32_t x;
    if (st.kind == FK_LEAF_RANGE) x = id - st.lo < st.span ? 1u : 0u;
    else if (st.kind == FK_LEAF_LUT64) x = (uint32_t)(st.lut64 >> (id & 63u)) & 1u;
    else x = (gload<uint32_t>(st.table + (id >> 5)) >> (id & 31u)) & 1u;
    m |= x << J;
  }
};

// A decoder wave's matching docs of segment g into numDocsScanned's per-segment counter.
__device__ __forceinline__ void ring_add_matched(const RingArgs &a, int g, uint32_t n, int lane) {
  const unsigned long long t = wave_sum((unsigned long long)n);
  if (lane == 0 && t) atomicAdd(a.matched + g, t);
}

// What the decoders keep of a segment's descriptor (GroupSegment): ch0 = its first chunk minus its first global chunk.
struct RingSeg {
  const uint64_t *pre;
  int64_t nwords, ch0;
  int32_t num_docs, n_leaves;
};

// A lane's raw dwords of a column's quarter (group_lq.h load_raw_lq) as three unconditional loads: conditional
// loads let the register allocator reuse a pending load's destination on the other path, and every later write of that
// register then waits for all outstanding loads (vmcnt(0) between the columns' loads). The bytes past the quarter's
// ceil(B / 2) + 1 dwords stay inside the forward index's padding and hit lines the wave reads anyway.
__device__ __forceinline__ void ring_load_raw(const uint8_t *fwd, int bits, int64_t qi, uint32_t (&R)[12]) {
  // 11 dwords: the most a quarter of <= 20 bits spans (a dead 12th dword would be a pending load's destination the
  // allocator hands out again, and that write waits for every load)
  const uint32_t *p = reinterpret_cast<const uint32_t *>(fwd) + ((qi * bits) >> 1);
  const u32x4a x0 = gload<u32x4a>(p), x1 = gload<u32x4a>(p + 4);
  const u32x3a x2 = gload<u32x3a>(p + 8);
  R[0] = x0.x; R[1] = x0.y; R[2] = x0.z; R[3] = x0.w;
  R[4] = x1.x; R[5] = x1.y; R[6] = x1.z; R[7] = x1.w;
  R[8] = x2.x; R[9] = x2.y; R[10] = x2.z; R[11] = 0;
}

// A decoder wave's quarters: load(t) requests pass t's quarter (its filter word and the raw dwords of its filter leaves,
// group and aggregated columns: issued, not waited for), decode() turns the requested quarter into 16 records per lane
// (act: the docs passing the filter). The segment descriptors follow the requested quarter; a quarter past the block's
// range (or a chunk with no candidate doc) requests nothing and decodes to no record.
template <int NF, bool WORDS>
struct RingDecoder {
  int64_t c0, nq, g_end;  // g_end: the first global chunk past segment g
  int wave, g;
  RingSeg sg;
  RingColsDev k;
  RingLeaf st[NF > 0 ? NF : 1];
  uint32_t seg_matched;  // this lane's matching docs of segment g
  // the requested quarter
  bool live;
  int64_t qi;
  uint32_t word_bits;    // the lane's 16 candidate docs (pre / filter words, tail)
  uint32_t F[NF > 0 ? NF : 1][12];
  uint32_t RA[kRingGroupCols][12], RB[kRingAggCols][12];
  // the decoded quarter (act_next / skip_next: the requested quarter's filter between its two decode halves)
  uint32_t act, act_next;
  bool skip_next;
  unsigned long long rec[16];

  __device__ __forceinline__ void init(const RingArgs &a, int64_t c0_, int64_t nq_, int wave_, int lane) {
    c0 = c0_;
    nq = nq_;
    wave = wave_;
    g = -1;
    g_end = 0;
    seg_matched = 0;
    live = false;
    act = act_next = 0;
    skip_next = true;
#pragma unroll
    for (int j = 0; j < 16; j++) rec[j] = 0;
  }

  __device__ __forceinline__ void load(const RingArgs &a, int64_t t) {
    const int64_t qg = t * kRingDecWaves + wave;
    live = qg < nq;
    if (!live) return;  // uniform
    const int64_t c = c0 + (qg >> 2);
    const int q = (int)(qg & 3);
    const int lane = threadIdx.x & 63;
    if (g < 0 || c >= g_end) {  // uniform: the descriptors change with the segment only
      const int gn = ring_segment(a, c, g < 0 ? 0 : g);
      g_end = gn + 1 < a.nsegs ? load_const(a.cstart + gn + 1) : INT64_MAX;
      if (!WORDS && g >= 0) ring_add_matched(a, g, seg_matched, lane);
      seg_matched = 0;
      g = gn;
      const GroupSegment gs = load_const(a.segs + g);
      sg.pre = gs.pre;
      sg.nwords = gs.nwords;
      sg.num_docs = gs.num_docs;
      sg.n_leaves = gs.n_leaves;
      sg.ch0 = gs.ch_begin - load_const(a.cstart + g);
      k = ring_cols(a, gs);
#pragma unroll
      for (int i = 0; i < NF; i++)
        if (i < sg.n_leaves) st[i] = ring_leaf(a.leaves + gs.first_leaf + i);
    }
    const int64_t ch = sg.ch0 + c;
    const int64_t w = ch * 64 + 16 * q + (lane >> 2);  // the chunk word holding this lane's 16 docs
    uint64_t word;
    if constexpr (WORDS) {
      word = w < sg.nwords ? gload<uint64_t>(a.filter + (size_t)g * a.filter_stride + w) : 0ull;
    } else {
      word = w < sg.nwords ? (sg.pre ? gload<uint64_t>(sg.pre + w) : ~0ull) & tail_mask(w, sg.nwords, sg.num_docs) : 0ull;
    }
    word_bits = (uint32_t)(word >> (16 * (lane & 3))) & 0xFFFFu;
    qi = ch * 256 + 64 * q + lane;
#pragma unroll
    for (int i = 0; i < NF; i++)
      if (i < sg.n_leaves) ring_load_raw(st[i].fwd, st[i].bits, qi, F[i]);
#pragma unroll
    for (int cc = 0; cc < kRingGroupCols; cc++)
      if (k.bits[cc]) ring_load_raw(k.fwd[cc], k.bits[cc], qi, RA[cc]);
#pragma unroll
    for (int cc = 0; cc < kRingAggCols; cc++)
      if (k.bits[kRingGroupCols + cc]) ring_load_raw(k.fwd[kRingGroupCols + cc], k.bits[kRingGroupCols + cc], qi, RB[cc]);
  }

  // Records J0 .. JE - 1 of the requested quarter (keys, then the aggregated fields).
  template <int J0, int JE>
  __device__ __forceinline__ void decode_records(const RingArgs &a) {
    uint32_t key[16];
#pragma unroll
    for (int j = J0; j < JE; j++) key[j] = 0;
#pragma unroll
    for (int cc = 0; cc < kRingGroupCols; cc++) {
      if (!k.bits[cc]) continue;
      RingKeyFold f{key, k.remap[cc], k.stride[cc]};
      ring_decode<J0, JE>(RA[cc], k.bits[cc], qi, f);
    }
    const uint32_t lmask = (1u << a.shift) - 1u;
#pragma unroll
    for (int j = J0; j < JE; j++)
      rec[j] = (unsigned long long)(key[j] & lmask) | ((unsigned long long)(key[j] >> a.shift) << kRecPShift);
#pragma unroll
    for (int cc = 0; cc < kRingAggCols; cc++) {
      if (!k.bits[kRingGroupCols + cc]) continue;
      RingFieldFold f{rec, k.fsh[kRingGroupCols + cc]};
      ring_decode<J0, JE>(RB[cc], k.bits[kRingGroupCols + cc], qi, f);
    }
  }

  // First half of the requested quarter's decode (while the flushers empty round 0's buckets): its filter (every doc)
  // into act_next and records 0 .. 7, whose round-0 entries of the current pass are already in the buckets.
  __device__ __forceinline__ void decode_front(const RingArgs &a) {
    act_next = live ? word_bits : 0u;
    skip_next = !__any(act_next != 0);  // uniform: nothing to insert
    if (skip_next) {
      act_next = 0;
      return;
    }
    if constexpr (NF > 0) {
#pragma unroll
      for (int i = 0; i < NF; i++)
        if (i < sg.n_leaves) {
          uint32_t m = 0;
          RingLeafFold f{st[i], m};
          ring_decode<0, 16>(F[i], st[i].bits, qi, f);
          act_next &= (st[i].negate ? ~m : m) & 0xFFFFu;
        }
    }
    if constexpr (!WORDS) seg_matched += __popc(act_next);
    decode_records<0, kRingRoundRecs>(a);
  }

  // Second half (while the flushers empty round 1's buckets): records 8 .. 15; the quarter becomes the current one.
  __device__ __forceinline__ void decode_back(const RingArgs &a) {
    act = act_next;
    if (skip_next) return;
    if constexpr (kRingRoundRecs < 16) decode_records<kRingRoundRecs, 16>(a);
  }

  __device__ __forceinline__ void finish(const RingArgs &a, int lane) {
    if (!WORDS && g >= 0) ring_add_matched(a, g, seg_matched, lane);
  }
};

// WORDS: the filter words GB_FILTER wrote; else the segment's top-level conjunction of <= NF scan leaves evaluated here
// on each quarter (lane-owns-quarter reads, like the group columns), AND-ed with the `pre` words if any.
//
// The block walks its quarters in passes: in pass t decoder wave w takes quarter 4 c0 + 8 t + w of the block's range
// (none past its end: that wave inserts nothing). A pass inserts the wave's 16 records per lane in two rounds of
// [insert phase | barrier | flush phase | barrier]; during the first flush phase the decoders evaluate the filter of the
// next pass's quarter (its raw dwords requested a pass earlier) and decode its records 0 .. 7 (the slots round 0 just
// emptied), during the second its records 8 .. 15, then request the quarter after it: the decode's VALU work fills
// both flush phases. Every wave executes the same barriers.
template <int NF, bool WORDS, int RB, bool HLL>
__global__ __launch_bounds__(kRingBlock) void k_group_ring(RingArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: chunk indices and descriptors in SGPRs
  const int b = blockIdx.x;
  const RingLds L = ring_lds(lds, a.P);
  for (int i = tid; i < a.P; i += kRingBlock) {
    L.ctr[i] = 0;
    L.back[i] = 0;
  }
  __syncthreads();
  const uint32_t C = a.cap;
  if (b == 0 && tid == 0) *a.region = C;
  uint8_t *region0 = a.records + (size_t)b * C * RB;  // region (p, b): records ((p * nblk + b) * C ...) of RB bytes
  uint32_t status = 0;
  const int64_t c0 = a.total_chunks * b / a.nblk, c1 = a.total_chunks * (b + 1) / a.nblk;
  const int64_t nq = (c1 - c0) * 4;  // the block's quarters
  const int64_t npass = (nq + kRingDecWaves - 1) / kRingDecWaves;
  constexpr int KP = (kRingMaxPartitions + 64 * kRingFlushWaves - 1) / (64 * kRingFlushWaves);
  if (wave >= kRingDecWaves) {  // flusher
    const int fw = wave - kRingDecWaves;
    uint32_t front[KP];
#pragma unroll
    for (int k = 0; k < KP; k++) front[k] = 0;
    for (int64_t t = 0; t < npass; t++)
#pragma unroll 1
      for (int r = 0; r < 16 / kRingRoundRecs; r++) {
        __syncthreads();  // inserts of the round done
        ring_flush_phase<RB, HLL, KP>(a, L, region0, C, fw, lane, front, status);
        __syncthreads();  // flushes done (and the decoders' next quarter decoded)
      }
    // the partial buckets (< 8 entries) to their fronts, then each region's counts
#pragma unroll
    for (int k = 0; k < KP; k++) {
      const int p = fw * 64 + lane + 64 * kRingFlushWaves * k;
      if (p >= a.P) continue;
      const uint32_t c = L.ctr[p], n = min(c & 0xFFFFu, (uint32_t)kRingBucket), h = c >> 16, nb = L.back[p];
      for (uint32_t i = 0; i < n; i++)
        if (front[k] + i < C)
        {
          unsigned long long r = L.bkt[p * kRingBucketStride + ((h + i) & (kRingBucket - 1))] & ((1ull << kRecPShift) - 1ull);
          if constexpr (HLL) r = ring_hll_out(a, r);
          store_rec<RB>(region0, (size_t)p * a.nblk * C + front[k] + i, r);
        }
      const uint32_t f = front[k] + n;
      if (f + nb > C || f >= (1u << (32 - kRingBackBits)) || nb >= (1u << kRingBackBits)) status |= 1u;
      a.hist[(size_t)p * a.nblk + b] = min(f, (1u << (32 - kRingBackBits)) - 1u) | (min(nb, (1u << kRingBackBits) - 1u) << (32 - kRingBackBits));
    }
  } else {  // decoder
    RingDecoder<NF, WORDS> d;
    d.init(a, c0, nq, wave, lane);
    d.load(a, 0);  // pass 0's raw dwords
    d.decode_front(a);
    d.decode_back(a);
    d.load(a, 1);  // in flight during pass 0's rounds
    for (int64_t t = 0; t < npass; t++) {
      ring_insert<RB, HLL, 0>(a, L, d.act, d.rec, region0, C);
      if constexpr (kRingRoundRecs < 16) {
        __syncthreads();  // inserts of round 0 done
        // the next pass's quarter: filter and records 0 .. 7 decoded meanwhile the flushers empty round 0's buckets
        d.decode_front(a);
        __syncthreads();  // flush done
        ring_insert<RB, HLL, kRingRoundRecs>(a, L, d.act, d.rec, region0, C);
      }
      __syncthreads();  // inserts of round 1 done
      // records 8 .. 15 of the next pass's quarter decoded meanwhile the flushers empty round 1's buckets, then the
      // quarter after it requested
      if constexpr (kRingRoundRecs == 16) d.decode_front(a);
      d.decode_back(a);
      d.load(a, t + 2);
      __syncthreads();  // flush done
    }
    d.finish(a, lane);
  }
  if (status) atomicOr(a.status, status);
}

// ----------------------------------------------------------------------------------------------------- reduce
constexpr int kRingReduceBlock = 1024;
constexpr int kRingReduceUnroll = 4;   // 16-B / 12-B loads (two records each) per lane and step
constexpr int kRingExceptions = 512;   // HLL ranks > 15 per partition (nibble registers saturate at 15)

__device__ __forceinline__ unsigned long long ordered_bits_g(double d) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(d);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}

__device__ __forceinline__ double dict_value_g(const void *dict, int value_kind, uint32_t id) {
  switch (value_kind) {
    case 0: return (double)static_cast<const int32_t *>(dict)[id];
    case 1: return (double)static_cast<const long long *>(dict)[id];
    default: return static_cast<const double *>(dict)[id];
  }
}

// GATHER = false: every aggregation is a COUNT, an affine-dictionary SUM / AVG or an affine-dictionary HLL (the host
// checks), so the fold issues no memory loads and the records' prefetched loads are waited for exactly.
template <int N, bool GATHER>
__device__ __forceinline__ void ring_fold(const RingReduceArgs &a, uint8_t *lds, uint32_t *cnt, uint32_t *exc_n,
                                          uint32_t *exc, const unsigned long long (&rec)[N], const bool (&ok)[N],
                                          int pk, int sbits, bool lo32, uint32_t &status) {
  const uint32_t kmask = (1u << a.shift) - 1u;
  uint32_t k[N];
#pragma unroll
  for (int u = 0; u < N; u++) k[u] = (uint32_t)rec[u] & kmask;
  if (pk < 0) {
#pragma unroll
    for (int u = 0; u < N; u++)
      if (ok[u]) atomicAdd(cnt + k[u], 1u);
  }
  for (int g = 0; g < a.n_aggs; g++) {
    const GroupAggDev &ag = a.aggs[g];
    if (ag.acc_kind == 5) continue;
    // a slot outside the streamed range holds whatever the region's memory held (an earlier query's records): its
    // dictId indexes nothing, so the gathers below read entry 0 for it
    uint32_t id[N];
#pragma unroll
    for (int u = 0; u < N; u++) {
      id[u] = (uint32_t)((rec[u] >> ag.field_shift) & ((1ull << ag.bits) - 1ull));
      if constexpr (GATHER) id[u] = ok[u] ? id[u] : 0u;
    }
    uint8_t *acc = lds + ag.lds_off;
    if (ag.acc_kind == 0) {
      unsigned long long v[N];  // affine: Σ dictId here, Σ value = base * count + step * Σ dictId at the end
#pragma unroll
      for (int u = 0; u < N; u++)
        v[u] = (!GATHER || ag.affine) ? (unsigned long long)id[u]
                                      : (unsigned long long)(long long)gload<int32_t>(static_cast<const int32_t *>(ag.dict) + id[u]);
      if (g == pk) {
#pragma unroll
        for (int u = 0; u < N; u++) v[u] += 1ull << sbits;
      }
#pragma unroll
      for (int u = 0; u < N; u++)
        if (ok[u]) atomicAdd(reinterpret_cast<unsigned long long *>(acc) + k[u], v[u]);
    } else if (ag.acc_kind == 4) {  // 4-bit registers: max by CAS on the containing dword
      uint32_t h[N];  // register << 8 | rank
      if ((a.hll_pre >> g) & 1) {  // the scatter's field: register << 5 | rank
#pragma unroll
        for (int u = 0; u < N; u++) h[u] = ((id[u] >> 5) << 8) | (id[u] & 31u);
      } else {
#pragma unroll
        for (int u = 0; u < N; u++)
          h[u] = (GATHER && !ag.affine) ? (uint32_t)gload<uint16_t>(ag.hll_lut + id[u])
                 : lo32 ? hll_register_rank_g(murmur_hash_lo32_g((uint32_t)ag.affine_base + (uint32_t)ag.affine_step * id[u]))
                        : hll_register_rank_g(murmur_hash_long_g(ag.affine_base + ag.affine_step * (long long)id[u]));
      }
      uint32_t *word[N], old[N], rk[N];
      int sh[N];
      uint32_t over = 0;  // records whose rank exceeds the nibble: the exception list (rare)
#pragma unroll
      for (int u = 0; u < N; u++) {
        const uint32_t idx = k[u] * 256 + (h[u] >> 8), rank = h[u] & 0xFFu;
        word[u] = reinterpret_cast<uint32_t *>(acc) + (idx >> 3);
        sh[u] = (int)(idx & 7) * 4;
        rk[u] = ok[u] ? min(rank, 15u) : 0u;
        over |= (ok[u] && rank > 15u) ? (1u << u) : 0u;
        old[u] = *word[u];
      }
      if (__any(over != 0)) {  // uniform, rare: out of the register reads' way (no branch or wait between them)
#pragma unroll
        for (int u = 0; u < N; u++)
          if ((over >> u) & 1u) {
            const uint32_t e = atomicAdd(exc_n, 1u);
            if (e < (uint32_t)kRingExceptions) exc[e] = (k[u] << 13) | ((h[u] >> 8) << 5) | (h[u] & 0xFFu);
            else status |= 4u;
          }
      }
#pragma unroll
      for (int u = 0; u < N; u++) {
        if (((old[u] >> sh[u]) & 15u) >= rk[u]) continue;
        uint32_t seen = atomicCAS(word[u], old[u], (old[u] & ~(15u << sh[u])) | (rk[u] << sh[u]));
        while (seen != old[u]) {
          old[u] = seen;
          if (((old[u] >> sh[u]) & 15u) >= rk[u]) break;
          seen = atomicCAS(word[u], old[u], (old[u] & ~(15u << sh[u])) | (rk[u] << sh[u]));
        }
      }
    } else if constexpr (GATHER) {
      double v[N];
#pragma unroll
      for (int u = 0; u < N; u++) v[u] = ok[u] ? dict_value_g(ag.dict, ag.value_kind, id[u]) : 0.0;
#pragma unroll
      for (int u = 0; u < N; u++) {
        if (!ok[u]) continue;
        if (ag.acc_kind == 1) atomicAdd(reinterpret_cast<double *>(acc) + k[u], v[u]);
        else if (ag.acc_kind == 2) atomicMin(reinterpret_cast<unsigned long long *>(acc) + k[u], ordered_bits_g(v[u]));
        else atomicMax(reinterpret_cast<unsigned long long *>(acc) + k[u], ordered_bits_g(v[u]));
      }
    }
  }
}

// A 16-B (RB = 8) or 12-B (RB = 6) unit of two consecutive records.
template <int RB>
using RingUnit = typename std::conditional<RB == 8, u32x4, u32x3a>::type;

template <int RB, int U, bool GATHER>
__device__ __forceinline__ void ring_fold_units(const RingReduceArgs &a, uint8_t *lds, uint32_t *cnt, uint32_t *exc_n,
                                                uint32_t *exc, const RingUnit<RB> (&v)[U], const uint32_t (&n)[U], int pk,
                                                int sbits, bool lo32, uint32_t &status) {
  unsigned long long rec[2 * U];
  bool ok[2 * U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    // the loaded set passes through an empty asm here, in straight-line code: the compiler waits for exactly these
    // loads (the other set's stay in flight); a first use inside the fold's runtime loops would wait for every load
    RingUnit<RB> x = v[u];
    asm volatile("" : "+v"(x));
    if constexpr (RB == 8) {
      rec[2 * u] = ((unsigned long long)x.y << 32) | x.x;
      rec[2 * u + 1] = ((unsigned long long)x.w << 32) | x.z;
    } else {
      rec[2 * u] = ((unsigned long long)(x.y & 0xFFFFu) << 32) | x.x;
      rec[2 * u + 1] = ((unsigned long long)x.z << 16) | (x.y >> 16);
    }
    ok[2 * u] = n[u] & 1u;
    ok[2 * u + 1] = (n[u] >> 1) & 1u;
  }
  ring_fold<2 * U, GATHER>(a, lds, cnt, exc_n, exc, rec, ok, pk, sbits, lo32, status);
}

constexpr int kRingReduceWaves = kRingReduceBlock / 64;

// A reduce wave's position in its regions' record ranges: region v, part (0: its front [0, F), 1: its back
// [C - B, C)), next 16-B unit i of the units [i, u1) covering the range [s0, s0 + n) (a unit = records 2i, 2i + 1).
struct RingStream {
  int v, part;
  uint32_t i, u1, s0, n;
};

// Loads the wave's next kRingReduceUnroll units per lane (64 lanes x 16 B consecutive per load), moving on to the
// wave's next non-empty range when this one is done (wave w: regions w, w + 16, ..., each front then back); v >= nblk
// once the stream is exhausted (loads then stay in bounds and count no record). cnt[u]: bit 0 / 1 = record 2i / 2i + 1
// of the unit is in the range.
template <int RB>
__device__ __forceinline__ bool ring_stream_next(const RingReduceArgs &a, const uint32_t *hrow, uint32_t C,
                                                 const uint8_t *base, RingStream &rs, int lane,
                                                 RingUnit<RB> (&v)[kRingReduceUnroll], uint32_t (&cnt)[kRingReduceUnroll]) {
  while (rs.i >= rs.u1) {  // uniform
    if (rs.part == 0) {
      rs.part = 1;
    } else {
      rs.part = 0;
      rs.v += kRingReduceWaves;
      if (rs.v >= a.nblk) break;
    }
    const uint32_t h = (uint32_t)__builtin_amdgcn_readfirstlane((int)hrow[rs.v]);
    const uint32_t f = min(h & ((1u << (32 - kRingBackBits)) - 1u), C), bk = min(h >> (32 - kRingBackBits), C - f);
    rs.s0 = rs.part ? C - bk : 0u;
    rs.n = rs.part ? bk : f;
    rs.i = rs.s0 >> 1;
    rs.u1 = (rs.s0 + rs.n + 1) >> 1;
  }
  const bool live = rs.v < a.nblk;
  // byte addressing: a 3-vector's sizeof is 16, so unit i of the 12-B units is at 12 i, not at src + i
  const uint8_t *src = base + (size_t)(live ? rs.v : 0) * C * RB;
#pragma unroll
  for (int u = 0; u < kRingReduceUnroll; u++) {
    const uint32_t idx = rs.i + (uint32_t)(u * 64 + lane);
    const bool ok = live && idx < rs.u1;
    const uint32_t r0 = 2 * idx;
    cnt[u] = ok ? ((r0 >= rs.s0 && r0 < rs.s0 + rs.n) ? 1u : 0u) | ((r0 + 1 >= rs.s0 && r0 + 1 < rs.s0 + rs.n) ? 2u : 0u)
                : 0u;
    v[u] = __builtin_nontemporal_load(  // unconditional (a branch would cost the counted wait)
        reinterpret_cast<const RingUnit<RB> *>(src + (size_t)(ok ? idx : 0u) * (2 * RB)));
  }
  rs.i += 64 * kRingReduceUnroll;
  return live;
}

template <bool GATHER, int RB>
__global__ __launch_bounds__(kRingReduceBlock) void k_ring_reduce(RingReduceArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x;
  const int p = blockIdx.x;
  const int K = 1 << a.shift;
  uint32_t *cnt = reinterpret_cast<uint32_t *>(lds + a.cnt_off);
  uint32_t *hrow = reinterpret_cast<uint32_t *>(lds + a.hist_off);
  uint32_t *exc_n = reinterpret_cast<uint32_t *>(lds + a.exc_off);
  uint32_t *exc = exc_n + 4;
  for (int i = tid; i < a.lds_zero_bytes / 4; i += kRingReduceBlock) reinterpret_cast<uint32_t *>(lds)[i] = 0;
  __syncthreads();
  for (int g = 0; g < a.n_aggs; g++)
    if (a.aggs[g].acc_kind == 2) {
      unsigned long long *m = reinterpret_cast<unsigned long long *>(lds + a.aggs[g].lds_off);
      for (int i = tid; i < K; i += kRingReduceBlock) m[i] = ~0ull;
    }
  __shared__ uint32_t s_n, s_C, s_over;
  if (tid == 0) {
    s_n = 0;
    s_C = *a.region;
    s_over = *a.status & 1u;
  }
  __syncthreads();
  // a region overflowed: its counts name slots never written this query (the host answers on the counted plan)
  if (s_over) return;
  {
    uint32_t part = 0;
    for (int i = tid; i < a.nblk; i += kRingReduceBlock) {
      const uint32_t h = a.hist[(size_t)p * a.nblk + i];  // front | back << 20
      hrow[i] = h;
      part += (h & ((1u << (32 - kRingBackBits)) - 1u)) + (h >> (32 - kRingBackBits));
    }
    atomicAdd(&s_n, part);
  }
  __syncthreads();
  const uint32_t C = s_C, n = s_n;
  // count folded into the first affine dictId SUM: (1 << sbits) + dictId per record, when both fields fit 64 bits
  const int cbits = n ? 32 - __builtin_clz(n) : 1;
  int pk = -1, sbits = 0;
  for (int g = 0; g < a.n_aggs; g++)
    if (pk < 0 && a.aggs[g].acc_kind == 0 && a.aggs[g].affine && a.aggs[g].bits + 2 * cbits <= 64) {
      pk = g;
      sbits = a.aggs[g].bits + cbits;
    }
  // affine HLL values all in [0, 2^32): the 32-bit form of the hash (every HLL aggregation of the query)
  bool lo32 = true;
  for (int g = 0; g < a.n_aggs; g++)
    if (a.aggs[g].acc_kind == 4) {
      const GroupAggDev &ag = a.aggs[g];
      const long long top = ag.affine_base + ag.affine_step * (long long)((1ull << ag.bits) - 1ull);
      lo32 = lo32 && ag.affine && ag.affine_base >= 0 && ag.affine_step >= 0 && ag.bits < 32 && top < (1ll << 32);
    }
  uint32_t status = 0;
  const uint8_t *base = a.records + (size_t)p * a.nblk * C * RB;
  // wave w streams record ranges w, w + 16, ... (each region's front and back): 16-B loads (two records) per lane,
  // kRingReduceUnroll loads per lane and step, the next step's loads issued before this step's records are folded
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int U = kRingReduceUnroll;
  RingStream rs{};
  rs.v = wave - kRingReduceWaves;
  rs.part = 1;  // the first advance moves to region `wave`, front part
  rs.i = 0;
  rs.u1 = 0;
  // two register sets, unrolled by two (no copies: a copy of a set still in flight would wait for its loads)
  RingUnit<RB> va[U], vb[U];
  uint32_t na[U], nb[U];
  bool live_a = ring_stream_next<RB>(a, hrow, C, base, rs, lane, va, na);
  while (live_a) {  // uniform; every load unconditional (an exhausted stream loads unit 0 with no record counted)
    const bool live_b = ring_stream_next<RB>(a, hrow, C, base, rs, lane, vb, nb);
    ring_fold_units<RB, U, GATHER>(a, lds, cnt, exc_n, exc, va, na, pk, sbits, lo32, status);
    if (!live_b) break;
    live_a = ring_stream_next<RB>(a, hrow, C, base, rs, lane, va, na);
    ring_fold_units<RB, U, GATHER>(a, lds, cnt, exc_n, exc, vb, nb, pk, sbits, lo32, status);
  }
  __syncthreads();
  const long long kbase = (long long)p * K;
  const long long nkeys = a.G - kbase < (long long)K ? a.G - kbase : (long long)K;
  for (int i = tid; i < nkeys; i += kRingReduceBlock) {
    uint32_t c = 0;
    if (pk >= 0) c = (uint32_t)(reinterpret_cast<const unsigned long long *>(lds + a.aggs[pk].lds_off)[i] >> sbits);
    else c = cnt[i];
    a.counts[kbase + i] = c;
  }
  const uint32_t ne = min(*exc_n, (uint32_t)kRingExceptions);
  for (int g = 0; g < a.n_aggs; g++) {
    const GroupAggDev &ag = a.aggs[g];
    if (ag.acc_kind == 5) continue;
    const uint8_t *acc = lds + ag.lds_off;
    if (ag.acc_kind == 4) {  // nibbles [K][128 B] -> u8 [G][256], 16 registers per thread (+ the exceptions)
      u32x4 *out = reinterpret_cast<u32x4 *>(static_cast<uint8_t *>(ag.acc) + kbase * 256);
      unsigned long long *sums = reinterpret_cast<unsigned long long *>(static_cast<uint8_t *>(ag.acc) + a.G * 256);
      for (long long t = tid; t < nkeys * 16; t += kRingReduceBlock) {  // a key's 16 threads: 16 consecutive lanes
        const unsigned long long x = reinterpret_cast<const unsigned long long *>(acc)[t];
        uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 16; j++) {
          uint32_t v = (uint32_t)(x >> (4 * j)) & 15u;
          if (v == 15u && ne) {
            const uint32_t key = (uint32_t)(t >> 4), reg = (uint32_t)(t & 15) * 16 + j;
            for (uint32_t e = 0; e < ne; e++) {
              const uint32_t ex = exc[e];
              if ((ex >> 13) == key && ((ex >> 5) & 0xFFu) == reg) v = max(v, ex & 31u);
            }
          }
          w[j >> 2] |= v << (8 * (j & 3));
        }
        u32x4 o;
        o.x = w[0];
        o.y = w[1];
        o.z = w[2];
        o.w = w[3];
        out[t] = o;
        if (a.hll_sums) {  // HyperLogLog.cardinality's exact fixed-point sum and zero count (k_group_final kind 9)
          unsigned long long sv = 0;
          uint32_t z = 0;
#pragma unroll
          for (int j = 0; j < 16; j++) {
            const uint32_t v = (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            sv += 1ull << (32 - v);
            z += v == 0u;
          }
#pragma unroll
          for (int o2 = 8; o2 > 0; o2 >>= 1) {
            sv += __shfl_xor(sv, o2, 16);
            z += __shfl_xor(z, o2, 16);
          }
          if ((t & 15) == 0) sums[kbase + (t >> 4)] = sv | ((unsigned long long)z << 48);
        }
      }
    } else {
      unsigned long long *out = static_cast<unsigned long long *>(ag.acc);
      for (int i = tid; i < nkeys; i += kRingReduceBlock) {
        unsigned long long v = reinterpret_cast<const unsigned long long *>(acc)[i];
        if (ag.acc_kind == 0 && ag.affine) {
          uint32_t c = 0;
          if (pk >= 0) {
            c = (uint32_t)(reinterpret_cast<const unsigned long long *>(lds + a.aggs[pk].lds_off)[i] >> sbits);
            if (g == pk) v &= (1ull << sbits) - 1ull;
          } else {
            c = cnt[i];
          }
          v = (unsigned long long)ag.affine_base * c + (unsigned long long)ag.affine_step * v;  // exact mod 2^64
        }
        out[kbase + i] = v;
      }
    }
  }
  if (status) atomicOr(a.status, status);
}

}  // namespace

size_t ring_lds_bytes(int P) {
  return (size_t)P * (kRingBucketStride * 8 + 4 + 4) + (size_t)kRingFlushWaves * kRingListPerWave * 4 + 16;
}

void launch_group_ring(const RingArgs &a, hipStream_t stream) {
  if (a.nblk <= 0 || a.total_chunks <= 0) return;
  const size_t lds = ring_lds_bytes(a.P);
  const dim3 grid((unsigned)a.nblk), block(kRingBlock);
  // instances: the filter form (GB_FILTER words / 0-2 quarter-form leaves) x record bytes x the flushers' HLL field
#define PINOT_RING(NF, W)                                                                                   \
  do {                                                                                                      \
    if (a.rec_bytes == 6) {                                                                                 \
      if (a.hll) hipLaunchKernelGGL((k_group_ring<NF, W, 6, true>), grid, block, lds, stream, a);           \
      else hipLaunchKernelGGL((k_group_ring<NF, W, 6, false>), grid, block, lds, stream, a);                \
    } else {                                                                                                \
      if (a.hll) hipLaunchKernelGGL((k_group_ring<NF, W, 8, true>), grid, block, lds, stream, a);           \
      else hipLaunchKernelGGL((k_group_ring<NF, W, 8, false>), grid, block, lds, stream, a);                \
    }                                                                                                       \
  } while (0)
  if (a.nf < 0) PINOT_RING(0, true);
  else if (a.nf == 0) PINOT_RING(0, false);
  else if (a.nf == 1) PINOT_RING(1, false);
  else PINOT_RING(2, false);
#undef PINOT_RING
}

void launch_ring_reduce(const RingReduceArgs &a, hipStream_t stream) {
  if (a.P <= 0) return;
  bool gather = false;  // any aggregation reading its dictionary / HLL LUT in the fold
  for (int g = 0; g < a.n_aggs; g++) {
    const int k = a.aggs[g].acc_kind;
    gather = gather || k == 1 || k == 2 || k == 3 || ((k == 0 || k == 4) && !a.aggs[g].affine);
  }
  const dim3 grid((unsigned)a.P), block(kRingReduceBlock);
  const size_t lds = (size_t)a.lds_bytes;
  if (a.rec_bytes == 6) {
    if (gather) hipLaunchKernelGGL((k_ring_reduce<true, 6>), grid, block, lds, stream, a);
    else hipLaunchKernelGGL((k_ring_reduce<false, 6>), grid, block, lds, stream, a);
  } else {
    if (gather) hipLaunchKernelGGL((k_ring_reduce<true, 8>), grid, block, lds, stream, a);
    else hipLaunchKernelGGL((k_ring_reduce<false, 8>), grid, block, lds, stream, a);
  }
}

int ring_reduce_exceptions() { return kRingExceptions; }

}  // namespace pinot
