// Ring-partitioned group-by (the large-key-space plan, config 4): no histogram pass, fixed-capacity regions.
//
//   k_group_query<GB_FILTER>  (fused_group.hip) the filter program once: filter words per segment + the matching docs
//                        of every ring block (region sizing), no group column read.
//   k_group_ring         one block per CU, every wave a loader: per 1024-doc quarter each lane decodes its 16 docs'
//                        group key and aggregated dictIds (lane-owns-quarter reads, the next quarter's loads in
//                        flight while this one is sunk) into u64 records (local key | dictId fields | partition) and
//                        appends them to its partition's LDS ring of 16 slots (two halves of 8). The lane whose
//                        write completes a half moves it to the block's region of that partition as one aligned 64-B
//                        piece: region (p, block) holds records [0, n) in claim order, so every flush lands on its own
//                        64-B sector and no histogram, scan or cursor leaves the CU.
//   k_ring_reduce        one block per partition of K <= 1024 consecutive keys: the partition's records from every
//                        block's region folded into LDS accumulators (count packed beside the first affine dictId
//                        SUM, int64 / double sums, ordered min / max, HLL registers as 4-bit nibbles with the rare
//                        rank > 15 kept in an exception list), then written to the dense arrays with plain stores.
//
// Restates DictionaryBasedGroupKeyGenerator.generateKeysForBlock (raw key = mixed radix over the group columns'
// dictIds, PC/query/aggregation/groupby/DictionaryBasedGroupKeyGenerator.java:195-302) and DefaultGroupByExecutor
// .process / aggregateGroupBySV (PC/query/aggregation/groupby/DefaultGroupByExecutor.java:70-168). Region sizes come
// from the filter's per-block match counts; a partition whose records exceed its region (skewed keys) sets a status
// bit and the host answers the query on the counted plan instead (executor.cpp).
#include <hip/hip_runtime.h>

#include "fused_common.h"
#include "group_lq.h"

namespace pinot {

// Records per region: the busiest block's matching docs spread over the partitions by key share, + 12.5 % + 64,
// a multiple of 16 (128-B aligned regions), never above the allocation.
__host__ __device__ uint32_t ring_region_records(uint64_t max_block_docs, int64_t K, int64_t G, uint32_t cap) {
  const uint64_t mean = (max_block_docs * (uint64_t)K + (uint64_t)G - 1) / (uint64_t)G;
  uint64_t c = mean + mean / 8 + 64;
  c = (c + 15) & ~15ull;
  return (uint32_t)(c < cap ? c : cap);
}

namespace {
using namespace dev;

constexpr int kRingBlock = 512;  // 8 waves: the 16-record sink and the next quarter's raw loads need the registers
constexpr int kRingWaves = kRingBlock / 64;
constexpr int kRecPShift = 53;  // records carry their partition in bits [53, 64)

struct RingLds {
  unsigned long long *ring;  // [P][16]
  unsigned long long *meta;  // [P]: claims (bits 0-31) | half 0 laps flushed (32-47) | half 1 laps flushed (48-63)
  uint32_t *wr;              // [P][2]: records written per half (mod 8 = 7 on the completing write)
  uint32_t *flist;           // [waves][64]: this round's flushes (partition << 18 | half-lap)
};

__device__ __forceinline__ RingLds ring_lds(uint8_t *lds, int P) {
  RingLds r;
  r.ring = reinterpret_cast<unsigned long long *>(lds);
  r.meta = r.ring + (size_t)P * 16;
  r.wr = reinterpret_cast<uint32_t *>(r.meta + P);
  r.flist = r.wr + 2 * P;
  return r;
}

__device__ __forceinline__ uint32_t rec_part(unsigned long long r) { return (uint32_t)(r >> kRecPShift); }

// Move the listed completed halves out: every lane that completed one lists (partition, half-lap) at its rank among
// this round's flushing lanes, then the wave stores eight halves per instruction (8 lanes x 8 B each). The laps-flushed
// bump follows the ring reads in this wave's LDS order, so a writer of the next lap (which waits for the bump) never
// overwrites a slot before it has been read.
template <int DBG>
__device__ __forceinline__ void ring_flush(const RingArgs &a, const RingLds &L, uint32_t *fl, uint32_t comp,
                                           const uint32_t (&pos)[16], const unsigned long long (&rec)[16],
                                           unsigned long long *region0, uint32_t C, int lane) {
  while (true) {
    const uint64_t fm = __ballot(comp != 0);
    if (!fm) break;  // uniform
    if (comp) {
      const int j = __builtin_ctz(comp);
      uint32_t pj = 0, mj = 0;
#pragma unroll
      for (int t = 0; t < 16; t++)
        if (t == j) {
          pj = rec_part(rec[t]);
          mj = pos[t] >> 3;
        }
      const int f = __builtin_amdgcn_mbcnt_hi((uint32_t)(fm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u));
      fl[f] = (pj << 18) | mj;
      comp &= comp - 1u;
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);  // list writes before the list reads (one wave's LDS order)
    const int nf = __popcll(fm);
    for (int f0 = 0; f0 < nf; f0 += 8) {  // uniform
      const int f = f0 + (lane >> 3), r = lane & 7;
      if (f < nf) {
        const uint32_t e = fl[f];
        const uint32_t p = e >> 18, m = e & 0x3FFFFu, h = m & 1u;
        const unsigned long long v = L.ring[p * 16 + h * 8 + r];
        if (DBG == 0 || a.debug != 2) __builtin_nontemporal_store(v, region0 + ((size_t)p * a.nblk) * C + (size_t)m * 8 + r);
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        if (r == 0) __hip_atomic_fetch_add(L.meta + p, 1ull << (32 + 16 * h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
  }
}

// Sink of a lane's 16 records (act: bit j = record j is live), in two batches of 8 claims. DBG = 1: the instrumented
// instance (debug.ring modes and the wait counters), never the production one.
template <int DBG>
__device__ __forceinline__ void ring_sink(const RingArgs &a, const RingLds &L, uint32_t *fl, uint32_t act,
                                          const unsigned long long (&rec)[16], unsigned long long *region0, uint32_t C,
                                          int lane, uint32_t &over, uint32_t &waits, uint32_t &sleeps) {
  uint32_t pos[16];
  uint32_t todo = 0, pend = 0;
  // claims: one 64-bit LDS add returns the claim index and both halves' flushed-lap counts
#pragma unroll
  for (int j0 = 0; j0 < 16; j0 += 8) {
    unsigned long long old[8];
#pragma unroll
    for (int j = 0; j < 8; j++)
      old[j] = ((act >> (j0 + j)) & 1u) ? __hip_atomic_fetch_add(L.meta + rec_part(rec[j0 + j]), 1ull, __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_WORKGROUP)
                                        : 0ull;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      pos[j0 + j] = (uint32_t)old[j];
      if (!((act >> (j0 + j)) & 1u)) continue;
      if (pos[j0 + j] >= C) {  // region full: the query falls back to the counted plan
        over |= 1u;
        continue;
      }
      const uint32_t h = (pos[j0 + j] >> 3) & 1u, lap = (pos[j0 + j] >> 4) & 0xFFFFu;
      const uint32_t flh = (uint32_t)(old[j] >> (32 + 16 * h)) & 0xFFFFu;
      if (flh == lap) todo |= 1u << (j0 + j);
      else pend |= 1u << (j0 + j);
    }
  }
  if (DBG && a.debug == 3) return;  // claims only
  if (DBG && __any(pend != 0)) waits++;
  // records whose slot still holds the previous lap (its half not yet moved out) wait for the bump and go in a later
  // round; every wave moves out what it completed before it waits, so the half it waits for always drains
  uint32_t spins = 0;
  while (true) {
    uint32_t comp = 0;
#pragma unroll
    for (int j = 0; j < 16; j++)
      if ((todo >> j) & 1u) L.ring[rec_part(rec[j]) * 16 + (pos[j] & 15u)] = rec[j] & ((1ull << kRecPShift) - 1ull);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
#pragma unroll
    for (int j = 0; j < 16; j++)
      if ((todo >> j) & 1u) {
        const uint32_t w = __hip_atomic_fetch_add(L.wr + rec_part(rec[j]) * 2 + ((pos[j] >> 3) & 1u), 1u,
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        comp |= ((w & 7u) == 7u) ? (1u << j) : 0u;
      }
    ring_flush<DBG>(a, L, fl, comp, pos, rec, region0, C, lane);
    if (!__any(pend != 0)) break;  // uniform
    if (++spins > (1u << 22)) {  // bounded: a protocol fault ends the launch with a status, never a hang
      over |= 2u;
      break;
    }
    __builtin_amdgcn_s_sleep(2);
    if (DBG) sleeps++;
    todo = 0;
    for (uint32_t x = pend; x; x &= x - 1u) {
      const int j = __builtin_ctz(x);
      uint32_t pj = 0, psj = 0;
#pragma unroll
      for (int t = 0; t < 16; t++)
        if (t == j) {
          pj = rec_part(rec[t]);
          psj = pos[t];
        }
      const unsigned long long m = __hip_atomic_load(L.meta + pj, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const uint32_t h = (psj >> 3) & 1u, lap = (psj >> 4) & 0xFFFFu;
      if (((uint32_t)(m >> (32 + 16 * h)) & 0xFFFFu) == lap) todo |= 1u << j;
    }
    pend &= ~todo;
  }
}

// Segment of global chunk c (the chunk windows of the segments, concatenated in order): uniform scalar scan forward
// from g0, a segment at or before c's (a wave's chunks ascend, so the scan usually stops at once).
__device__ __forceinline__ int ring_segment(const RingArgs &a, int64_t c, int g0 = 0) {
  int g = g0;
  while (g + 1 < a.nsegs && load_const(a.cstart + g + 1) <= c) g++;
  return g;
}

struct RingCursor {
  int64_t c;      // current chunk (global index), >= end: done
  int64_t cn;     // next chunk of this wave
  uint64_t wc;    // this lane's filter word of chunk c
  uint64_t wn;    // ... of chunk cn (prefetched)
  int q;          // quarter of c
  uint32_t m;     // this lane's 16 filter bits of quarter q
  int gn;         // segment of chunk cn (a wave's chunks ascend)
};

__device__ __forceinline__ uint64_t ring_word(const RingArgs &a, int64_t c, int64_t end, int lane, int &gs) {
  if (c >= end) return 0ull;
  const int g = gs = ring_segment(a, c, gs);
  const GroupSegment sg = load_const(a.segs + g);
  const int64_t ch = sg.ch_begin + (c - load_const(a.cstart + g));
  const int64_t w = ch * 64 + lane;
  return w < sg.nwords ? gload<uint64_t>(a.filter + (size_t)g * a.filter_stride + w) : 0ull;
}

// Lane l of quarter q takes docs 1024q + 16l .. +15: bits 16(l & 3) .. of the chunk word 16q + l/4.
__device__ __forceinline__ uint32_t quarter_bits(uint64_t word, int q, int lane) {
  const int src = 16 * q + (lane >> 2);
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)word, src, 64);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(word >> 32), src, 64);
  return (((lane & 2) ? hi : lo) >> (16 * (lane & 1))) & 0xFFFFu;
}

// Next quarter with a matching doc (possibly in a later chunk of this wave).
__device__ __forceinline__ void ring_advance(const RingArgs &a, RingCursor &cu, int64_t end, int lane) {
  cu.q++;
  while (true) {
    if (cu.q == 4) {
      cu.c = cu.cn;
      cu.wc = cu.wn;
      cu.cn += kRingWaves;
      cu.wn = ring_word(a, cu.cn, end, lane, cu.gn);
      cu.q = 0;
      if (cu.c >= end) return;
      if (!__any(cu.wc != 0)) {  // uniform: nothing in this chunk
        cu.q = 4;
        continue;
      }
    }
    cu.m = quarter_bits(cu.wc, cu.q, lane);
    if (__any(cu.m != 0)) return;
    cu.q++;
  }
}

struct RingColsDev {
  const uint8_t *fwd[kGroupPfCols];
  const int32_t *remap[kGroupPfCols];
  uint32_t stride[kGroupPfCols];
  int bits[kGroupPfCols], fsh[kGroupPfCols];  // bits 0 = unused slot; fsh -1 = a group column (key fold)
};

__device__ __forceinline__ RingColsDev ring_cols(const RingArgs &a, int g) {
  const GroupSegment sg = load_const(a.segs + g);
  RingColsDev k;
#pragma unroll
  for (int c = 0; c < kGroupPfCols; c++) {
    k.fwd[c] = nullptr;
    k.remap[c] = nullptr;
    k.stride[c] = 0;
    k.bits[c] = 0;
    k.fsh[c] = -1;
    if (c < a.nc) {
      if (c < a.n_gcols) {
        const GroupColDev gc = load_const(a.gcols + sg.first_gcol + c);
        k.fwd[c] = gc.fwd;
        k.remap[c] = gc.remap;
        k.stride[c] = (uint32_t)gc.stride;
        k.bits[c] = gc.bits;
      } else {
        const int ai = c == 1 ? a.pf_agg[1] : c == 2 ? a.pf_agg[2] : a.pf_agg[3];
        const GroupAggDev ag = load_const(a.aggs + sg.first_agg + ai);
        k.fwd[c] = ag.fwd;
        k.bits[c] = ag.bits;
        k.fsh[c] = ag.field_shift;
      }
    }
  }
  return k;
}

__device__ __forceinline__ int64_t ring_qi(const RingArgs &a, const RingCursor &cu, int lane, int &g) {
  g = ring_segment(a, cu.c, g);
  const GroupSegment sg = load_const(a.segs + g);
  const int64_t ch = sg.ch_begin + (cu.c - load_const(a.cstart + g));
  return ch * 256 + 64 * cu.q + lane;
}

template <int DBG>
__global__ __launch_bounds__(kRingBlock) void k_group_ring(RingArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x;
  const RingLds L = ring_lds(lds, a.P);
  for (int i = tid; i < a.P; i += kRingBlock) {
    L.meta[i] = 0;
    L.wr[2 * i] = 0;
    L.wr[2 * i + 1] = 0;
  }
  // region size: the busiest block's matching docs (every block computes the same value)
  __shared__ uint32_t s_max;
  if (tid == 0) s_max = 0;
  __syncthreads();
  {
    uint32_t mx = 0;
    for (int i = tid; i < a.nblk; i += kRingBlock) mx = max(mx, a.blk_matched[i]);
    atomicMax(&s_max, mx);
  }
  __syncthreads();
  const uint32_t C = ring_region_records(s_max, int64_t(1) << a.shift, a.G, a.cap);
  if (b == 0 && tid == 0) *a.region = C;
  unsigned long long *region0 = a.records + (size_t)b * C;  // region (p, b) at ((p * nblk + b) * C)
  uint32_t *fl = L.flist + wave * 64;
  const int64_t c0 = a.total_chunks * b / a.nblk, c1 = a.total_chunks * (b + 1) / a.nblk;
  uint32_t over = 0, waits = 0, sleeps = 0;
  RingCursor cu;
  cu.cn = c0 + wave;
  cu.gn = 0;
  cu.wn = ring_word(a, cu.cn, c1, lane, cu.gn);
  cu.q = 3;
  cu.c = -1;
  ring_advance(a, cu, c1, lane);
  uint32_t R[kGroupPfCols][12];
  int g = 0;
  RingColsDev k{};
  int64_t qi = 0;
  if (cu.c < c1) {
    qi = ring_qi(a, cu, lane, g);
    k = ring_cols(a, g);
#pragma unroll
    for (int c = 0; c < kGroupPfCols; c++)
      if (k.bits[c]) load_raw_lq(k.fwd[c], k.bits[c], qi, R[c]);
  }
  const uint32_t lmask = (1u << a.shift) - 1u;
  while (cu.c < c1) {
    // decode this quarter: group key (mixed radix over global ids), then the record's fields
    uint32_t key[16];
#pragma unroll
    for (int j = 0; j < 16; j++) key[j] = 0;
#pragma unroll
    for (int c = 0; c < kGroupPfCols; c++) {
      if (!k.bits[c] || k.fsh[c] >= 0) continue;
      const int32_t *remap = k.remap[c];
      const uint32_t stride = k.stride[c];
      decode_raw_lq(R[c], k.bits[c], qi, [&](const uint32_t (&id)[16]) {
        if (remap) {
#pragma unroll
          for (int j = 0; j < 16; j++) key[j] += (uint32_t)gload<int32_t>(remap + id[j]) * stride;
        } else {
#pragma unroll
          for (int j = 0; j < 16; j++) key[j] += id[j] * stride;
        }
      });
    }
    unsigned long long rec[16];
#pragma unroll
    for (int j = 0; j < 16; j++)
      rec[j] = (unsigned long long)(key[j] & lmask) | ((unsigned long long)(key[j] >> a.shift) << kRecPShift);
#pragma unroll
    for (int c = 0; c < kGroupPfCols; c++) {
      if (!k.bits[c] || k.fsh[c] < 0) continue;
      const int fsh = k.fsh[c];
      decode_raw_lq(R[c], k.bits[c], qi, [&](const uint32_t (&id)[16]) {
#pragma unroll
        for (int j = 0; j < 16; j++) rec[j] |= (unsigned long long)id[j] << fsh;
      });
    }
    const uint32_t act = cu.m;
    // the next quarter's loads go out before this one is sunk (the sink issues LDS work and 64-B stores only)
    ring_advance(a, cu, c1, lane);
    if (cu.c < c1) {
      const int gp = g;
      qi = ring_qi(a, cu, lane, g);
      if (g != gp) k = ring_cols(a, g);  // uniform: the column descriptors change with the segment only
#pragma unroll
      for (int c = 0; c < kGroupPfCols; c++)
        if (k.bits[c]) load_raw_lq(k.fwd[c], k.bits[c], qi, R[c]);
    }
    if (DBG && a.debug == 1) {  // decode only: keep the records alive without the sink
      unsigned long long x = 0;
#pragma unroll
      for (int j = 0; j < 16; j++) x ^= ((act >> j) & 1u) ? rec[j] : 0ull;
      if (x == 0x0123456789ABCDEFull) over |= 8u;
      continue;
    }
    ring_sink<DBG>(a, L, fl, act, rec, region0, C, lane, over, waits, sleeps);
  }
  if (DBG && lane == 0 && waits) atomicAdd(a.status + 2, waits);
  if (DBG && lane == 0 && sleeps) atomicAdd(a.status + 3, sleeps);
  __syncthreads();
  // every complete half is out; the partial last half of each partition and the region's record count remain
  for (int p = tid; p < a.P; p += kRingBlock) {
    const uint32_t n = (uint32_t)L.meta[p];
    a.hist[(size_t)p * a.nblk + b] = n;
    if (n > C) {
      over = 1;
      continue;
    }
    const uint32_t kk = n & 7u, h = (n >> 3) & 1u, m = n >> 3;
    for (uint32_t r = 0; r < kk; r++)
      region0[((size_t)p * a.nblk) * C + (size_t)m * 8 + r] = L.ring[p * 16 + h * 8 + r];
  }
  if (over) atomicOr(a.status, over);
}

// ----------------------------------------------------------------------------------------------------- reduce
constexpr int kRingReduceBlock = 1024;
constexpr int kRingReduceRegions = 2;  // regions read per step (8 records in flight per thread)
constexpr int kRingReduceUnroll = 4;   // records per thread and region per step
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

__device__ __forceinline__ uint32_t hll_register_rank_g(uint32_t h) {
  return ((h >> 24) << 8) | (uint32_t)(__builtin_clz((h << 8) | 129u) + 1);
}

template <int N>
__device__ __forceinline__ void ring_fold(const RingReduceArgs &a, uint8_t *lds, uint32_t *cnt, uint32_t *exc_n,
                                          uint32_t *exc, const unsigned long long (&rec)[N], const bool (&ok)[N],
                                          int pk, int sbits, uint32_t &status) {
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
    uint32_t id[N];
#pragma unroll
    for (int u = 0; u < N; u++) id[u] = (uint32_t)((rec[u] >> ag.field_shift) & ((1ull << ag.bits) - 1ull));
    uint8_t *acc = lds + ag.lds_off;
    if (ag.acc_kind == 0) {
      unsigned long long v[N];  // affine: Σ dictId here, Σ value = base * count + step * Σ dictId at the end
#pragma unroll
      for (int u = 0; u < N; u++)
        v[u] = ag.affine ? (unsigned long long)id[u] : (unsigned long long)(long long)gload<int32_t>(static_cast<const int32_t *>(ag.dict) + id[u]);
      if (g == pk) {
#pragma unroll
        for (int u = 0; u < N; u++) v[u] += 1ull << sbits;
      }
#pragma unroll
      for (int u = 0; u < N; u++)
        if (ok[u]) atomicAdd(reinterpret_cast<unsigned long long *>(acc) + k[u], v[u]);
    } else if (ag.acc_kind == 4) {  // 4-bit registers: max by CAS on the containing dword
      uint32_t h[N];
#pragma unroll
      for (int u = 0; u < N; u++)
        h[u] = ag.affine ? hll_register_rank_g(murmur_hash_long_g(ag.affine_base + ag.affine_step * (long long)id[u]))
                         : (uint32_t)gload<uint16_t>(ag.hll_lut + id[u]);
      uint32_t *word[N], old[N], rk[N];
      int sh[N];
#pragma unroll
      for (int u = 0; u < N; u++) {
        const uint32_t idx = k[u] * 256 + (h[u] >> 8), rank = h[u] & 0xFFu;
        word[u] = reinterpret_cast<uint32_t *>(acc) + (idx >> 3);
        sh[u] = (int)(idx & 7) * 4;
        rk[u] = ok[u] ? min(rank, 15u) : 0u;
        if (ok[u] && rank > 15u) {
          const uint32_t e = atomicAdd(exc_n, 1u);
          if (e < (uint32_t)kRingExceptions) exc[e] = (k[u] << 13) | ((h[u] >> 8) << 5) | rank;
          else status |= 4u;
        }
        old[u] = *word[u];
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
    } else {
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
  __shared__ uint32_t s_n, s_C;
  if (tid == 0) {
    s_n = 0;
    s_C = *a.region;
  }
  __syncthreads();
  {
    uint32_t part = 0;
    for (int i = tid; i < a.nblk; i += kRingReduceBlock) {
      const uint32_t h = a.hist[(size_t)p * a.nblk + i];
      hrow[i] = h;
      part += h;
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
  uint32_t status = 0;
  const unsigned long long *base = a.records + (size_t)p * a.nblk * C;
  constexpr int RB = kRingReduceRegions, U = kRingReduceUnroll, N = RB * U;
  for (int b0 = 0; b0 < a.nblk; b0 += RB) {
    uint32_t hmax = 0;
#pragma unroll
    for (int r = 0; r < RB; r++) hmax = max(hmax, b0 + r < a.nblk ? hrow[b0 + r] : 0u);
    hmax = min(hmax, C);
    for (uint32_t r0 = 0; r0 < hmax; r0 += (uint32_t)U * kRingReduceBlock) {
      unsigned long long rec[N];
      bool ok[N];
#pragma unroll
      for (int r = 0; r < RB; r++)
#pragma unroll
        for (int u = 0; u < U; u++) {
          const int bb = b0 + r;
          const uint32_t i = r0 + (uint32_t)(u * kRingReduceBlock + tid);
          const bool v = bb < a.nblk && i < min(hrow[bb < a.nblk ? bb : 0], C);
          ok[r * U + u] = v;
          rec[r * U + u] = v ? __builtin_nontemporal_load(base + (size_t)bb * C + i) : 0ull;
        }
      ring_fold<N>(a, lds, cnt, exc_n, exc, rec, ok, pk, sbits, status);
    }
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
      for (long long t = tid; t < nkeys * 16; t += kRingReduceBlock) {
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

size_t ring_lds_bytes(int P) { return (size_t)P * (16 * 8 + 8 + 8) + (size_t)kRingWaves * 64 * 4; }

void launch_group_ring(const RingArgs &a, hipStream_t stream) {
  if (a.nblk <= 0 || a.total_chunks <= 0) return;
  if (a.debug) hipLaunchKernelGGL(k_group_ring<1>, dim3((unsigned)a.nblk), dim3(kRingBlock), ring_lds_bytes(a.P), stream, a);
  else hipLaunchKernelGGL(k_group_ring<0>, dim3((unsigned)a.nblk), dim3(kRingBlock), ring_lds_bytes(a.P), stream, a);
}

void launch_ring_reduce(const RingReduceArgs &a, hipStream_t stream) {
  if (a.P <= 0) return;
  hipLaunchKernelGGL(k_ring_reduce, dim3((unsigned)a.P), dim3(kRingReduceBlock), (size_t)a.lds_bytes, stream, a);
}

int ring_reduce_exceptions() { return kRingExceptions; }

}  // namespace pinot
