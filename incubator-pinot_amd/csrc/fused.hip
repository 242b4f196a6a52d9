// K1 + K5 fused: ONE launch per aggregation-only query over every segment resident on the GPU.
//
// Per 4096-doc chunk (64 words of 64 docs, one lane per word) a wave
//   1. starts from the segment's `pre` bitset (index leaves / OR subtrees) or all docs,
//   2. for each scan leaf of the top-level conjunction: stages the chunk of the column in LDS with
//      coalesced 1-KiB global_load_lds_dwordx4 pieces, decodes the lane's 64 dictIds (two halves of 32,
//      unrolled per bit width, selected by a 32-way switch) and ANDs the predicate bits into the mask
//      that stays in registers (no bitset round trip through HBM),
//   3. stops touching the chunk as soon as the wave's mask is empty (skips every remaining column),
//   4. folds the aggregated columns over the matching docs: COUNT, Σ dictId (arithmetic-progression
//      dictionaries), Σ int32 dictionary values, min/max dictId (sorted dictionaries), HLL registers.
// Block partials go to HBM; the last block to arrive reduces them in a fixed order into host-mapped memory.
//
// Restates: PinotDataBitSet.readInt (PC/io/util/PinotDataBitSet.java:79-100), SVScanDocIdIterator
// (PC/operator/dociditerators/SVScanDocIdIterator.java:85-159), AndBlockDocIdSet (:144-227),
// AggregationOperator.getNextBlock (PC/operator/query/AggregationOperator.java:56-82) and the
// Count/Sum/Min/Max/Avg/DistinctCountHLL aggregate() loops.
#include <hip/hip_runtime.h>

#include "device.h"
#include "kernels.h"

namespace pinot {
namespace {
using namespace dev;

// Runtime bit width, compile-time extraction: a wave stages the chunk of the step's column in LDS
// (ceil(B/2) coalesced 1-KiB DMA pieces), then each lane decodes its 64 values as two halves of 32.
// Half h of the lane's super-word is the B dwords at byte 8*B*lane + 4*B*h; a 32-way switch over B
// (PINOT_WIDTH_SWITCH) selects a step instance whose shifts are constants.
template <int B, int J>
__device__ __forceinline__ void decode_half_step(const uint32_t (&D)[B], uint32_t (&v)[32]) {
  constexpr int p = J * B, k = p >> 5, o = p & 31;
  constexpr uint32_t mask = (uint32_t)((1ull << B) - 1ull);
  if constexpr (o + B <= 32) v[J] = (D[k] >> (32 - o - B)) & mask;
  else v[J] = __builtin_amdgcn_alignbit(D[k], D[k + 1], 64 - o - B) & mask;
  if constexpr (J + 1 < 32) decode_half_step<B, J + 1>(D, v);
}

template <int B>
__device__ __forceinline__ void decode_half(const uint8_t *p, uint32_t (&v)[32]) {
  uint32_t D[B];
  if constexpr (B % 2 == 0) {
#pragma unroll
    for (int i = 0; i < B / 2; i++) {
      const u32x2 x = *reinterpret_cast<const u32x2 *>(p + 8 * i);
      D[2 * i] = bswap32(x.x);
      D[2 * i + 1] = bswap32(x.y);
    }
  } else {
#pragma unroll
    for (int i = 0; i < B; i++) D[i] = bswap32(*reinterpret_cast<const uint32_t *>(p + 4 * i));
  }
  decode_half_step<B, 0>(D, v);
}

// Stages chunk `ch` (64 words = 4096 docs, 512*B contiguous bytes) of a packed column into the wave's LDS.
// nt: non-temporal cache policy (aux = 2) for the once-read column streams.
__device__ __forceinline__ void stage_chunk_rt(const uint8_t *__restrict__ fwd, int bits, int64_t ch, uint8_t *lds_wave,
                                               int lane, bool nt = false) {
  const uint8_t *src = fwd + (size_t)ch * (size_t)(512 * bits) + lane * 16;
  const int pieces = (bits + 1) >> 1;
  if (nt) {
    for (int i = 0; i < pieces; i++)
      __builtin_amdgcn_global_load_lds((glob_void_t *)(src + i * 1024), (lds_void_t *)(lds_wave + i * 1024), 16, 0, 2);
  } else {
    for (int i = 0; i < pieces; i++)
      __builtin_amdgcn_global_load_lds((glob_void_t *)(src + i * 1024), (lds_void_t *)(lds_wave + i * 1024), 16, 0, 0);
  }
}

// Predicate bits of 32 decoded dictIds, bit j = value j, shifted in from j = 31 down.
// RANGE: (v - lo) < span as the borrow of a subtract, shifted in by one v_addc: 3 VALU ops per value
// (the compiler's own form is compare + cndmask + shift/or, 4.5).
#define PINOT_RANGE_STEP(x) \
  "v_sub_u32 %1, " x ", %6\n\tv_sub_co_u32 %1, vcc, %1, %7\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc\n\t"
__device__ __forceinline__ uint32_t range_bits(const uint32_t (&v)[32], uint32_t lo, uint32_t span) {
  uint32_t m = 0;
#pragma unroll
  for (int j = 31; j >= 3; j -= 4) {
    uint32_t t;
    asm(PINOT_RANGE_STEP("%2") PINOT_RANGE_STEP("%3") PINOT_RANGE_STEP("%4") PINOT_RANGE_STEP("%5")
        : "+v"(m), "=&v"(t)
        : "v"(v[j]), "v"(v[j - 1]), "v"(v[j - 2]), "v"(v[j - 3]), "v"(lo), "v"(span)
        : "vcc");
  }
  return m;
}
#undef PINOT_RANGE_STEP

template <bool G>
__device__ __forceinline__ uint32_t leaf_half(const FusedStep &st, const uint32_t (&v)[32]) {
  uint32_t m = 0;
  if (st.kind == FK_LEAF_RANGE) {
    m = range_bits(v, st.lo, st.span);
  } else if (!G || st.kind == FK_LEAF_LUT64) {
    if ((st.lut64 >> 32) == 0) {  // cardinality <= 32: one 32-bit LUT word, v_bfe_u32 per value
      const uint32_t lut = (uint32_t)st.lut64;
#pragma unroll
      for (int j = 31; j >= 0; j--) m = (m << 1) + __builtin_amdgcn_ubfe(lut, v[j], 1);
    } else {
#pragma unroll
      for (int j = 31; j >= 0; j--) m = (m << 1) + ((uint32_t)(st.lut64 >> v[j]) & 1u);
    }
  } else {
    const uint32_t *__restrict__ lut = static_cast<const uint32_t *>(st.table);
#pragma unroll
    for (int j = 31; j >= 0; j--) m = (m << 1) + __builtin_amdgcn_ubfe(lut[v[j] >> 5], v[j] & 31, 1);
  }
  return m;
}

constexpr int kFusedWaves = kBlock / 64;

// HLL registers of the block (G programs only; atomicMax per matching doc). Everything else a block
// reduces lives in registers until the flush, which reuses the (then idle) staging LDS as BlockRed, so a
// streaming-only program (G = false) has no static LDS at all: 4 blocks x 4 waves x 10 KiB stages fill
// the CU's 160 KiB at b = 20.
typedef uint32_t HllRegs[256];

struct BlockRed {
  uint32_t last;  // this block arrived last: it reduces every block's partials
  uint32_t pad;
  unsigned long long cnt[kFusedWaves];
  unsigned long long sum[kFusedWaves][kMaxFusedFolds];
  uint32_t mn[kFusedWaves][kMaxFusedFolds], mx[kFusedWaves][kMaxFusedFolds];
};

// Per-lane fold accumulators, held in registers for the whole kernel (the fold loop is unrolled over
// kMaxFusedFolds so fold f indexes them at compile time). LDS is touched only once, at the flush: an
// LDS atomic inside the chunk loop would make the compiler wait (vmcnt) for the in-flight LDS-DMA.
struct FoldAcc {
  unsigned long long sum[kMaxFusedFolds];
  uint32_t mn[kMaxFusedFolds], mx[kMaxFusedFolds];
};

// Bit j of the match mask as an opaque 0/1 value: keeps the compiler from turning the per-value
// masking into 32 lane-mask selects (which it hoists into SGPR pairs and then spills).
__device__ __forceinline__ uint32_t mbit(uint32_t mh, int j) {
  uint32_t r;
  asm("v_bfe_u32 %0, %1, %2, 1" : "=v"(r) : "v"(mh), "i"(j));
  return r;
}

// Fold partials of one chunk (both halves) for one aggregated column.
struct FoldPart {
  unsigned long long sum = 0;
  uint32_t mn = 0xFFFFFFFFu, mx = 0;
};

template <int B, bool G>
__device__ __forceinline__ void fold_half(const FusedStep &st, uint32_t mh, const uint32_t (&v)[32], FoldPart &r,
                                          HllRegs *hll) {
  if (st.ops & FOLD_IDSUM) {
    if constexpr (B <= 24) {  // v * bit + t as a 24-bit multiply-add; 32 values of <= 24 bits sum below 2^29
      uint32_t t = 0;
#pragma unroll
      for (int j = 0; j < 32; j++) t += __umul24(v[j], mbit(mh, j));
      r.sum += t;
    } else {
#pragma unroll
      for (int j = 0; j < 32; j++) r.sum += (unsigned long long)(v[j] & (0u - mbit(mh, j)));
    }
  }
  if (G && (st.ops & FOLD_DICT32)) {
    const int32_t *__restrict__ dict = static_cast<const int32_t *>(st.table);
    long long s = 0;
#pragma unroll
    for (int j = 0; j < 32; j++) s += (long long)(dict[v[j]] & (int32_t)(0u - mbit(mh, j)));
    r.sum += (unsigned long long)s;
  }
  if (st.ops & FOLD_MINMAX) {  // max over v & m, min over v | ~m (m = all-ones when the doc matches)
#pragma unroll
    for (int j = 0; j < 32; j++) {
      const uint32_t b = mbit(mh, j);
      r.mn = min(r.mn, v[j] | (b - 1u));
      r.mx = max(r.mx, v[j] & (0u - b));
    }
  }
  if (G && (st.ops & FOLD_HLL)) {
    uint32_t *regs = hll[st.hll_set];
#pragma unroll
    for (int j = 0; j < 32; j++)
      if ((mh >> j) & 1u) {
        const uint32_t e = st.hll_lut[v[j]];
        atomicMax(&regs[e >> 8], e & 0xFFu);
      }
  }
}

// One step of a chunk at compile-time width B: decode the lane's two halves from LDS and apply.
template <int B, bool G>
__device__ __forceinline__ void leaf_step(const FusedStep &st, const uint8_t *p, uint64_t &mask) {
  uint32_t v[32];
  decode_half<B>(p, v);
  const uint32_t m0 = leaf_half<G>(st, v);
  decode_half<B>(p + 4 * B, v);
  const uint32_t m1 = leaf_half<G>(st, v);
  const uint64_t m = ((uint64_t)m1 << 32) | m0;
  mask &= st.negate ? ~m : m;
}

template <int B, bool G>
__device__ __forceinline__ void fold_step(const FusedStep &st, const uint8_t *p, uint64_t mask, FoldPart &r,
                                          HllRegs *hll) {
  uint32_t v[32];
  decode_half<B>(p, v);
  fold_half<B, G>(st, (uint32_t)mask, v, r, hll);
  decode_half<B>(p + 4 * B, v);
  fold_half<B, G>(st, (uint32_t)(mask >> 32), v, r, hll);
}

#define PINOT_WIDTH_SWITCH(bits, CALL)                                                                         \
  switch (bits) {                                                                                              \
    case 1: CALL(1); break;   case 2: CALL(2); break;   case 3: CALL(3); break;   case 4: CALL(4); break;     \
    case 5: CALL(5); break;   case 6: CALL(6); break;   case 7: CALL(7); break;   case 8: CALL(8); break;     \
    case 9: CALL(9); break;   case 10: CALL(10); break; case 11: CALL(11); break; case 12: CALL(12); break;   \
    case 13: CALL(13); break; case 14: CALL(14); break; case 15: CALL(15); break; case 16: CALL(16); break;   \
    case 17: CALL(17); break; case 18: CALL(18); break; case 19: CALL(19); break; case 20: CALL(20); break;   \
    case 21: CALL(21); break; case 22: CALL(22); break; case 23: CALL(23); break; case 24: CALL(24); break;   \
    case 25: CALL(25); break; case 26: CALL(26); break; case 27: CALL(27); break; case 28: CALL(28); break;   \
    case 29: CALL(29); break; case 30: CALL(30); break; case 31: CALL(31); break; case 32: CALL(32); break;   \
    default: break;                                                                                            \
  }

template <bool G>
__device__ __forceinline__ void leaf_rt(const FusedStep &st, const uint8_t *p, uint64_t &mask) {
#define PINOT_LEAF(B) leaf_step<B, G>(st, p, mask)
  PINOT_WIDTH_SWITCH(st.bits, PINOT_LEAF)
#undef PINOT_LEAF
}

template <bool G>
__device__ __forceinline__ void fold_rt(const FusedStep &st, const uint8_t *p, uint64_t mask, FoldPart &r,
                                        HllRegs *hll) {
#define PINOT_FOLD(B) fold_step<B, G>(st, p, mask, r, hll)
  PINOT_WIDTH_SWITCH(st.bits, PINOT_FOLD)
#undef PINOT_FOLD
}

// The per-query program (segments, steps) is read-only for the whole launch: reading it through the
// constant address space makes the compiler use scalar loads (s_load, lgkmcnt), so fetching a step
// descriptor never waits on the vector-memory counter that tracks the in-flight LDS-DMA stages.
typedef const __attribute__((address_space(4))) uint32_t cword_t;

template <typename T>
__device__ __forceinline__ T load_const(const T *p) {
  static_assert(sizeof(T) % 4 == 0, "dword-sized descriptor");
  T r;
  const cword_t *q = (const cword_t *)p;
  uint32_t *d = reinterpret_cast<uint32_t *>(&r);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); i++) d[i] = q[i];
  return r;
}

// Block-wide setup / teardown shared by both kernel shapes.
__device__ __forceinline__ void init_acc(FoldAcc &A) {
#pragma unroll
  for (int f = 0; f < kMaxFusedFolds; f++) {
    A.sum[f] = 0;
    A.mn[f] = 0xFFFFFFFFu;
    A.mx[f] = 0;
  }
}

__device__ __forceinline__ void init_hll(HllRegs *hll, int tid) {
  for (int i = tid; i < kMaxHll * 256; i += kBlock) (&hll[0][0])[i] = 0;
  __syncthreads();
}

// Block partials: wave reductions (shuffles) -> BlockRed in the idle staging LDS -> thread 0 adds the
// block's totals into the per-segment accumulators with memory-side integer atomics (u64 add, u32
// min/max: exact and order-independent, so the result is deterministic). The last block to arrive copies
// the accumulators and HLL registers into host-mapped memory and resets them to their identities for
// the next launch (replaces a reduce launch, a memset and a D2H copy). No __threadfence: an agent-scope
// fence writes back and invalidates the XCD's whole L2 under every still-streaming block; atomics
// execute at the memory side, vmcnt(0) waits for their acknowledgement before the arrival atomic, and
// the last block reads with agent-scope (L2-bypassing) loads.
__device__ __forceinline__ void flush_block(const FusedArgs &a, uint8_t *stage_lds, HllRegs *hll, const FoldAcc &A,
                                            unsigned long long cnt, int g, int tid, int lane, int wave) {
  const int nfolds = (a.nslots - 1) / 2;
  __syncthreads();  // every wave is done with its stage: reuse it
  BlockRed &R = *reinterpret_cast<BlockRed *>(stage_lds);
  cnt = wave_sum(cnt);
  if (lane == 0) R.cnt[wave] = cnt;
#pragma unroll
  for (int f = 0; f < kMaxFusedFolds; f++) {
    if (f >= nfolds) break;
    const unsigned long long s = wave_sum(A.sum[f]);
    uint32_t lo = A.mn[f], hi = A.mx[f];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      lo = min(lo, (uint32_t)__shfl_xor((int)lo, o, 64));
      hi = max(hi, (uint32_t)__shfl_xor((int)hi, o, 64));
    }
    if (lane == 0) {
      R.sum[wave][f] = s;
      R.mn[wave][f] = lo;
      R.mx[wave][f] = hi;
    }
  }
  __syncthreads();
  unsigned long long *acc = a.acc + (int64_t)g * a.res_stride;
  if (tid == 0) {
    unsigned long long c = 0;
    for (int w = 0; w < kFusedWaves; w++) c += R.cnt[w];
    if (c) atomicAdd(acc, c);
    for (int f = 0; f < nfolds; f++) {
      unsigned long long s = 0;
      uint32_t lo = 0xFFFFFFFFu, hi = 0;
      for (int w = 0; w < kFusedWaves; w++) {
        s += R.sum[w][f];
        lo = min(lo, R.mn[w][f]);
        hi = max(hi, R.mx[w][f]);
      }
      if (s) atomicAdd(acc + 1 + 2 * f, s);
      uint32_t *mm = reinterpret_cast<uint32_t *>(acc + 2 + 2 * f);  // little-endian: [0] = min, [1] = max
      if (lo != 0xFFFFFFFFu) atomicMin(mm, lo);
      if (hi) atomicMax(mm + 1, hi);
    }
  }
  if (hll)
    for (int h = 0; h < a.n_hll; h++)
      for (int i = tid; i < 256; i += kBlock) {
        const uint32_t r = hll[h][i];
        if (r) atomicMax(&a.hll_out[h * 256 + i], r);
      }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const uint32_t nblk = (uint32_t)(a.nsegs * a.bps);
  if (tid == 0) R.last = atomicAdd(a.done, 1u) == nblk - 1 ? 1u : 0u;
  __syncthreads();
  if (!R.last) return;
  const int n = a.nsegs * a.res_stride;
  for (int i = tid; i < n; i += kBlock) {
    const int sl = i % a.res_stride;
    a.result[i] = __hip_atomic_load(a.acc + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    a.acc[i] = slot_init((sl == 0 || (sl & 1)) ? SLOT_SUM_U64 : SLOT_MINMAX);
  }
  uint32_t *res_hll = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(a.result) + a.result_hll_off);
  for (int i = tid; i < a.n_hll * 256; i += kBlock) {
    res_hll[i] = __hip_atomic_load(&a.hll_out[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    a.hll_out[i] = 0;
  }
  if (tid == 0) *a.done = 0;
}

// ---------------------------------------------------------------- index leaves evaluated in registers
// The lane's 64-doc word w of a sorted-index leaf (SortedInvertedIndexBasedFilterOperator: matching
// dictIds -> merged inclusive doc ranges) and of a bitmap-index leaf (BitmapBasedFilterOperator: OR of the
// dictIds' roaring bitmaps, flipped when exclusive), computed on the fly from the ranges / roaring
// containers — no dense bitset is materialised. A 4096-doc chunk lies inside one 65536-doc roaring key,
// so the container search is wave-uniform.
__device__ __forceinline__ uint64_t bits_between(int lo_bit, int hi_bit) {  // inclusive, 0 <= lo <= hi <= 63
  const uint64_t upper = hi_bit == 63 ? ~0ull : ((1ull << (hi_bit + 1)) - 1ull);
  return upper & (~0ull << lo_bit);
}

__device__ __forceinline__ uint64_t ranges_word(const int32_t *__restrict__ r, int n, int64_t w) {
  const int64_t lo = w * 64, hi = lo + 63;
  int l = 0, h = n;
  while (l < h) {  // first range ending at or after lo
    const int m = (l + h) >> 1;
    if (r[2 * m + 1] < lo) l = m + 1;
    else h = m;
  }
  uint64_t x = 0;
  for (int i = l; i < n && r[2 * i] <= hi; i++) {
    const int64_t s = max((int64_t)r[2 * i], lo), e = min((int64_t)r[2 * i + 1], hi);
    x |= bits_between((int)(s - lo), (int)(e - lo));
  }
  return x;
}

__device__ __forceinline__ uint32_t ld16(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }

__device__ __forceinline__ uint64_t roaring_word(const FusedStep &st, int64_t w) {
  const uint8_t *payload = st.fwd;
  const RoaringContainer *conts = static_cast<const RoaringContainer *>(st.aux0);
  const int32_t *dir = static_cast<const int32_t *>(st.aux1);
  const int32_t *ids = static_cast<const int32_t *>(st.table);
  const uint32_t key = (uint32_t)(w >> 10);            // 1024 words per roaring key
  const uint32_t first = (uint32_t)(w & 1023) * 64;    // the word's first low-16 doc
  uint64_t x = 0;
  for (int i = 0; i < (int)st.lo; i++) {
    const int id = ids[i];
    int l = dir[id], r = dir[id + 1];
    const int end = r;
    while (l < r) {
      const int m = (l + r) >> 1;
      if (conts[m].key < key) l = m + 1;
      else r = m;
    }
    if (l >= end || conts[l].key != key) continue;
    const RoaringContainer c = conts[l];
    const uint8_t *p = payload + c.payload_offset;
    if (c.type == 1) {  // bitmap container: 1024 LE u64 words
      const uint8_t *q = p + (first >> 3);
      x |= (uint64_t)ld16(q) | ((uint64_t)ld16(q + 2) << 16) | ((uint64_t)ld16(q + 4) << 32) |
           ((uint64_t)ld16(q + 6) << 48);
    } else if (c.type == 0) {  // sorted u16 array
      int a = 0, b = (int)c.cardinality;
      while (a < b) {
        const int m = (a + b) >> 1;
        if (ld16(p + 2 * m) < first) a = m + 1;
        else b = m;
      }
      for (; a < (int)c.cardinality; a++) {
        const uint32_t v = ld16(p + 2 * a);
        if (v >= first + 64) break;
        x |= 1ull << (v - first);
      }
    } else {  // run container: (start, length - 1) pairs
      for (uint32_t k = 0; k < c.cardinality; k++) {
        const uint32_t s0 = ld16(p + 4 * k), e0 = s0 + ld16(p + 4 * k + 2);
        if (s0 >= first + 64) break;
        if (e0 < first) continue;
        x |= bits_between((int)(max(s0, first) - first), (int)(min(e0, first + 63) - first));
      }
    }
  }
  return st.negate ? ~x : x;
}

// One leaf's 64-bit word for this lane (scan leaves decode the staged chunk).
template <bool G, typename Src>
__device__ __forceinline__ uint64_t leaf_word(const FusedStep &st, int i, int64_t w, int lane, Src &src) {
  if (G && st.kind == FK_LEAF_RANGES) return ranges_word(static_cast<const int32_t *>(st.table), (int)st.lo, w);
  if (G && st.kind == FK_LEAF_ROARING) return roaring_word(st, w);
  uint64_t x = ~0ull;
  leaf_rt<G>(st, src(i, st) + lane * (8 * st.bits), x);
  return x;
}

// The filter program of a chunk: terms AND-ed into `mask` (early exit once the wave's mask is empty).
template <bool G, typename Src>
__device__ __forceinline__ uint64_t eval_filter(const FusedStep *__restrict__ steps, int n_leaves, uint64_t mask,
                                                int64_t w, int64_t nwords, int32_t num_docs, int lane, Src &&src) {
  uint64_t term = ~0ull;
  bool pending = false;
  for (int i = 0; i < n_leaves; i++) {
    const FusedStep st = load_const(steps + i);
    if (st.join == JOIN_NEW) {
      if (pending) mask &= term;
      pending = false;
      if (!__any(mask != 0)) return 0;  // wave-uniform: nothing left in this chunk, skip its other columns
    }
    uint64_t x = leaf_word<G>(st, i, w, lane, src);
    x = w < nwords ? x & tail_mask(w, nwords, num_docs) : 0ull;
    if (st.join == JOIN_NEW) term = x;
    else if (st.join == JOIN_OR) term |= x;
    else term &= x;
    pending = true;
  }
  return pending ? (mask & term) : mask;
}

// One chunk of the segment program: the filter program, then the folds over the surviving docs.
// `src(i, st)` returns the LDS address of step i's staged chunk (staging it first in the stepwise kernel). Returns the chunk's matching doc count.
template <bool G, typename Src>
__device__ __forceinline__ unsigned long long eval_chunk(const FusedStep *__restrict__ steps, int n_leaves,
                                                         int n_folds, uint64_t mask, FoldAcc &A, HllRegs *hll,
                                                         int64_t w, int64_t nwords, int32_t num_docs, int lane,
                                                         Src &&src) {
  mask = eval_filter<G>(steps, n_leaves, mask, w, nwords, num_docs, lane, src);
  const unsigned long long cnt = __popcll(mask);
  for (int i = 0; i < n_folds; i++) {
    if (!__any(mask != 0)) break;
    const FusedStep st = load_const(steps + n_leaves + i);  // st.fold == i (host order)
    FoldPart r;
    fold_rt<G>(st, src(n_leaves + i, st) + lane * (8 * st.bits), mask, r, hll);
#pragma unroll
    for (int f = 0; f < kMaxFusedFolds; f++)  // uniform select of the register accumulator
      if (f == i) {
        A.sum[f] += r.sum;
        A.mn[f] = min(A.mn[f], r.mn);
        A.mx[f] = max(A.mx[f], r.mx);
      }
  }
  return cnt;
}

__device__ __forceinline__ uint64_t chunk_word(const uint64_t *pre, int64_t nwords, int32_t num_docs, int64_t ch,
                                               int lane) {
  const int64_t w = ch * 64 + lane;
  if (w >= nwords) return 0;
  return (pre ? pre[w] : ~0ull) & tail_mask(w, nwords, num_docs);
}

// Stepwise shape: per chunk, each step's column is staged into the wave's single LDS stage and
// decoded before the next step is fetched (a step is fetched only while the chunk still has matches).
// G = false: streaming-only program (RANGE / 64-entry LUT leaves, Σ dictId and min/max folds), register-light;
// G = true: also memory-LUT leaves, dictionary-value sums and HLL (per-value gathers).
template <bool G>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(G ? 2 : 4))) void k_scan_query(FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t stage_lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  HllRegs *hll = nullptr;
  if constexpr (G) {
    __shared__ HllRegs hll_lds[kMaxHll];
    hll = hll_lds;
    init_hll(hll, tid);
  }
  const int g = blockIdx.x / a.bps, b = blockIdx.x % a.bps;
  const FusedSegment sg = load_const(a.segs + g);
  const FusedStep *steps = a.steps + sg.first_step;
  uint8_t *lds_wave = stage_lds + wave * a.stage_bytes;
  unsigned long long cnt = 0;
  FoldAcc A;
  init_acc(A);
  const int64_t nchunks = min((sg.nwords + 63) >> 6, sg.ch_end);
  for (int64_t ch = sg.ch_begin + (int64_t)b * kFusedWaves + wave; ch < nchunks; ch += (int64_t)a.bps * kFusedWaves) {
    cnt += eval_chunk<G>(steps, sg.n_leaves, sg.n_folds, chunk_word(sg.pre, sg.nwords, sg.num_docs, ch, lane), A, hll,
                         ch * 64 + lane, sg.nwords, sg.num_docs, lane,
                         [&](int, const FusedStep &st) -> const uint8_t * {
                           stage_chunk_rt(st.fwd, st.bits, ch, lds_wave, lane);
                           wait_stage();
                           return lds_wave;
                         });
  }
  flush_block(a, stage_lds, hll, A, cnt, g, tid, lane, wave);
}

// Pipelined shape: a chunk's every column is staged at once into one of the wave's two LDS slots, and
// the NEXT chunk of the wave is in flight (global_load_lds DMA) while this one is decoded. A slot is
//   [ 512 B: the `pre` words of the chunk after next | step 0 pieces | step 1 pieces | ... ]
// so the candidate mask of a chunk is known one iteration before its columns are fetched, and a chunk
// without candidate docs (sorted / bitmap index leaves, OR subtrees) costs 512 B instead of its columns.
// Only the leaf early exit inside a chunk saves decode work but not bytes. Every global access in the
// loop is an LDS-DMA, so the one `s_waitcnt vmcnt(0)` per iteration waits for exactly the chunk staged
// one iteration earlier. The host picks this shape when a slot fits (<= kMaxPipeSlotBytes).
__device__ __forceinline__ void stage_pre(const uint64_t *__restrict__ pre, int64_t ch, uint8_t *dst, int lane) {
  if (lane < 32)  // 32 lanes x 16 B = the chunk's 64 bitset words
    __builtin_amdgcn_global_load_lds((glob_void_t *)(pre + ch * 64 + lane * 2), (lds_void_t *)dst, 16, 0, 0);
}

__device__ __forceinline__ uint64_t pre_mask(const FusedSegment &sg, const uint8_t *slot, int64_t ch, int lane) {
  const int64_t w = ch * 64 + lane;
  if (w >= sg.nwords) return 0;
  const uint64_t p = sg.pre ? reinterpret_cast<const uint64_t *>(slot)[lane] : ~0ull;
  return p & tail_mask(w, sg.nwords, sg.num_docs);
}

template <bool G>
__global__ __launch_bounds__(kBlock) void k_scan_query_pipe(FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t stage_lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  HllRegs *hll = nullptr;
  if constexpr (G) {
    __shared__ HllRegs hll_lds[kMaxHll];
    hll = hll_lds;
    init_hll(hll, tid);
  }
  const int g = blockIdx.x / a.bps, b = blockIdx.x % a.bps;
  const FusedSegment sg = load_const(a.segs + g);
  const FusedStep *steps = a.steps + sg.first_step;
  const int nsteps = sg.n_leaves + sg.n_folds;
  uint8_t *const slots = stage_lds + (size_t)wave * 2 * a.stage_bytes;
  const int64_t nchunks = min((sg.nwords + 63) >> 6, sg.ch_end);
  const int64_t stride = (int64_t)a.bps * kFusedWaves;
  auto slot = [&](int p) { return slots + p * a.stage_bytes; };
  auto stage_cols = [&](int64_t c, uint8_t *dst) {
    for (int i = 0; i < nsteps; i++) {
      const FusedStep st = load_const(steps + i);
      stage_chunk_rt(st.fwd, st.bits, c, dst + st.stage_off, lane, a.nt != 0);
    }
  };
  unsigned long long cnt = 0;
  FoldAcc A;
  init_acc(A);
  int64_t ch = sg.ch_begin + (int64_t)b * kFusedWaves + wave;
  // prologue: pre words of ch (slot 0 area, waited for), of ch + stride (slot 1 area, read at iteration 0)
  if (sg.pre && ch < nchunks) stage_pre(sg.pre, ch, slot(0), lane);
  wait_stage();
  uint64_t m0 = ch < nchunks ? pre_mask(sg, slot(0), ch, lane) : 0;
  if (sg.pre && ch + stride < nchunks) stage_pre(sg.pre, ch + stride, slot(1), lane);
  bool live0 = __any(m0 != 0);
  if (live0) stage_cols(ch, slot(0));
  int par = 0;
  for (; ch < nchunks; ch += stride) {
    wait_stage();  // columns of ch and pre words of ch + stride, both issued one iteration ago
    uint8_t *cur = slot(par), *nxt = slot(par ^ 1);
    const uint64_t m1 = ch + stride < nchunks ? pre_mask(sg, nxt, ch + stride, lane) : 0;
    const bool live1 = __any(m1 != 0);
    if (live1) stage_cols(ch + stride, nxt);
    // cur's pre area (pre words of ch, read one iteration ago) is free again
    if (sg.pre && ch + 2 * stride < nchunks) stage_pre(sg.pre, ch + 2 * stride, cur, lane);
    if (live0)
      cnt += eval_chunk<G>(steps, sg.n_leaves, sg.n_folds, m0, A, hll, ch * 64 + lane, sg.nwords, sg.num_docs, lane,
                           [&](int, const FusedStep &st) -> const uint8_t * { return cur + st.stage_off; });
    m0 = m1;
    live0 = live1;
    par ^= 1;
  }
  wait_stage();
  flush_block(a, stage_lds, hll, A, cnt, g, tid, lane, wave);
}

// ======================================================================== fused group-by
// k_group_query: the filter of k_scan_query (stepwise leaves over LDS-staged chunks) followed, per
// 64-doc word of the chunk, by one-doc-per-lane key / dictId reads straight from the packed streams
// (a wave's 64 lanes read the 8*b contiguous bytes of the word: coalesced) and a sink (GroupMode).
// Restates DictionaryBasedGroupKeyGenerator.getGroupKey / processSingleValue (raw key = fold of
// key * card_j + dictId_j; PC/query/aggregation/groupby/DictionaryBasedGroupKeyGenerator.java:195-302)
// and DefaultGroupByExecutor.process (PC/query/aggregation/groupby/DefaultGroupByExecutor.java:70-168).
constexpr int kGroupBlock = 1024;                // 16 waves: the per-doc reads are latency-bound
constexpr int kGroupWaves = kGroupBlock / 64;
constexpr int kGroupUnroll = 8;                  // words whose reads are in flight together

__device__ __forceinline__ uint32_t decode_doc(const uint8_t *__restrict__ fwd, int bits, int64_t doc) {
  const uint64_t bitpos = (uint64_t)doc * (uint32_t)bits;
  const uint32_t *p = reinterpret_cast<const uint32_t *>(fwd) + (bitpos >> 5);
  const uint64_t x = ((uint64_t)bswap32(p[0]) << 32) | bswap32(p[1]);
  return (uint32_t)((x << (bitpos & 31)) >> (64 - bits));
}

__device__ __forceinline__ unsigned long long ordered_bits(double d) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(d);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}

__device__ __forceinline__ double dict_value(const void *dict, int value_kind, uint32_t id) {
  switch (value_kind) {
    case 0: return (double)static_cast<const int32_t *>(dict)[id];
    case 1: return (double)static_cast<const long long *>(dict)[id];
    default: return static_cast<const double *>(dict)[id];
  }
}

// HLL registers are bytes in HBM ([G][256] u8): max via CAS on the containing dword (low contention).
__device__ __forceinline__ void hll_max_u8(uint8_t *regs, long long idx, uint32_t rank) {
  uint32_t *word = reinterpret_cast<uint32_t *>(regs + (idx & ~3ll));
  const int sh = (int)(idx & 3) * 8;
  uint32_t old = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while (((old >> sh) & 0xFFu) < rank) {
    const uint32_t nv = (old & ~(0xFFu << sh)) | (rank << sh);
    const uint32_t seen = atomicCAS(word, old, nv);
    if (seen == old) break;
    old = seen;
  }
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

// One aggregated value into accumulator `acc` at index k (global or LDS address space by pointer).
template <bool LDS>
__device__ __forceinline__ void agg_update(const GroupAggDev &ag, void *acc, long long k, uint32_t id) {
  switch (ag.acc_kind) {
    case 0:
      atomicAdd(static_cast<unsigned long long *>(acc) + k,
                (unsigned long long)(long long)static_cast<const int32_t *>(ag.dict)[id]);
      break;
    case 1:
      atomicAdd(static_cast<double *>(acc) + k, dict_value(ag.dict, ag.value_kind, id));
      break;
    case 2:
      atomicMin(static_cast<unsigned long long *>(acc) + k, ordered_bits(dict_value(ag.dict, ag.value_kind, id)));
      break;
    case 3:
      atomicMax(static_cast<unsigned long long *>(acc) + k, ordered_bits(dict_value(ag.dict, ag.value_kind, id)));
      break;
    case 4: {
      const uint32_t e = ag.hll_lut[id];
      if constexpr (LDS) atomicMax(static_cast<uint32_t *>(acc) + k * 256 + (e >> 8), e & 0xFFu);
      else hll_max_u8(static_cast<uint8_t *>(acc), k * 256 + (e >> 8), e & 0xFFu);
      break;
    }
    default:
      break;
  }
}

__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {  // splitmix64 finaliser
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return x;
}

__device__ __forceinline__ long long hash_insert(const GroupArgs &a, unsigned long long fp) {
  const unsigned long long m = (unsigned long long)a.hcap - 1ull;
  unsigned long long slot = fp & m;
  for (long long probe = 0; probe < a.hcap; probe++) {
    unsigned long long cur = __hip_atomic_load(a.htable + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == 0) cur = atomicCAS(a.htable + slot, 0ull, fp);
    if (cur == 0 || cur == fp) return (long long)slot;
    slot = (slot + 1) & m;
  }
  return 0;  // unreachable: hcap >= 2 x docs
}

__device__ __forceinline__ long long hash_find(const GroupArgs &a, unsigned long long fp) {
  const unsigned long long m = (unsigned long long)a.hcap - 1ull;
  unsigned long long slot = fp & m;
  for (long long probe = 0; probe < a.hcap; probe++) {
    const unsigned long long cur = __hip_atomic_load(a.htable + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == fp) return (long long)slot;
    if (cur == 0) return -1;
    slot = (slot + 1) & m;
  }
  return -1;
}

__device__ __forceinline__ uint32_t tuple_id(const GroupArgs &a, int seg, int j, int64_t doc) {
  const GroupSegment s = load_const(a.segs + seg);
  const GroupColDev gc = load_const(a.gcols + s.first_gcol + j);
  const uint32_t id = decode_doc(gc.fwd, gc.bits, doc);
  return gc.remap ? (uint32_t)gc.remap[id] : id;
}

// Does doc of segment `sg` (this block's) carry the same global-id tuple as the representative `rep`?
__device__ __forceinline__ bool same_tuple(const GroupArgs &a, const GroupSegment &sg, int64_t doc, unsigned long long rep) {
  const int seg = (int)(rep >> 32);
  const int64_t rdoc = (int64_t)(rep & 0xFFFFFFFFull);
  const int mine = blockIdx.x / a.bps;
  for (int j = 0; j < a.n_gcols; j++)
    if (tuple_id(a, mine, j, doc) != tuple_id(a, seg, j, rdoc)) return false;
  return true;
}

template <int MODE>
__device__ __forceinline__ void group_chunk(const GroupArgs &a, const GroupSegment &sg, int64_t ch, uint64_t mask,
                                            int lane, uint8_t *acc_lds, uint32_t *plds) {
  for (int w0 = 0; w0 < 64; w0 += kGroupUnroll) {
    uint64_t mw[kGroupUnroll];
    bool any = false;
#pragma unroll
    for (int u = 0; u < kGroupUnroll; u++) {
      mw[u] = readlane64(mask, w0 + u);
      any = any || mw[u] != 0;
    }
    if (!any) continue;  // uniform
    int64_t doc[kGroupUnroll];
    unsigned long long key[kGroupUnroll];
    bool act[kGroupUnroll];
#pragma unroll
    for (int u = 0; u < kGroupUnroll; u++) {
      doc[u] = ((ch << 6) + w0 + u) * 64 + lane;
      key[u] = 0;
      act[u] = (mw[u] >> lane) & 1ull;
    }
    if (a.hashed) {
#pragma unroll
      for (int u = 0; u < kGroupUnroll; u++) key[u] = a.hseed;
    }
    for (int j = 0; j < a.n_gcols; j++) {
      const GroupColDev gc = load_const(a.gcols + sg.first_gcol + j);
      uint32_t id[kGroupUnroll];
#pragma unroll
      for (int u = 0; u < kGroupUnroll; u++) id[u] = decode_doc(gc.fwd, gc.bits, doc[u]);  // all docs: loads batch
#pragma unroll
      for (int u = 0; u < kGroupUnroll; u++) {
        const uint32_t gid = gc.remap ? (uint32_t)gc.remap[id[u]] : id[u];
        if (a.hashed) key[u] = mix64(key[u] ^ ((unsigned long long)gid + 0x9E3779B97F4A7C15ull * (unsigned long long)(j + 1)));
        else key[u] += (unsigned long long)gid * (unsigned long long)gc.stride;
      }
    }
    if (a.hashed) {
#pragma unroll
      for (int u = 0; u < kGroupUnroll; u++)
        if (act[u]) {
          const unsigned long long fp = key[u] | 1ull;  // 0 marks an empty slot
          if constexpr (MODE == GB_VERIFY) {
            const long long slot = hash_find(a, fp);
            if (slot < 0 || !same_tuple(a, sg, doc[u], __hip_atomic_load(a.reps + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)))
              atomicOr(a.verify_err, 1u);
            act[u] = false;
          } else {
            const long long slot = hash_insert(a, fp);
            atomicMin(a.reps + slot, ((unsigned long long)(blockIdx.x / a.bps) << 32) | (unsigned long long)doc[u]);
            key[u] = (unsigned long long)slot;
          }
        }
    }
    if (a.admitted) {
#pragma unroll
      for (int u = 0; u < kGroupUnroll; u++)
        act[u] = act[u] && ((a.admitted[key[u] >> 5] >> (key[u] & 31)) & 1u);
    }
    if constexpr (MODE == GB_VERIFY) {
      continue;
    } else if constexpr (MODE == GB_COUNT) {
#pragma unroll
      for (int u = 0; u < kGroupUnroll; u++)
        if (act[u]) atomicAdd(&plds[key[u] >> a.shift], 1u);
    } else if constexpr (MODE == GB_EMIT) {
      const int rshift = a.shift + a.split;  // two-level: records go to coarse run key >> (shift + split)
      unsigned long long rec[kGroupUnroll];
#pragma unroll
      for (int u = 0; u < kGroupUnroll; u++) rec[u] = key[u] & ((1ull << rshift) - 1ull);
      for (int g = 0; g < a.n_aggs; g++) {
        const GroupAggDev ag = load_const(a.aggs + sg.first_agg + g);
        if (ag.acc_kind == 5) continue;
#pragma unroll
        for (int u = 0; u < kGroupUnroll; u++)
          rec[u] |= (unsigned long long)decode_doc(ag.fwd, ag.bits, doc[u]) << ag.field_shift;
      }
      if (a.reserved2 == 0) {
        // all cursor claims first (inactive lanes add 0: no divergent branch around the LDS atomics, one
        // lgkmcnt wait), then the stores; the runs' lines combine in L2
        uint32_t pos[kGroupUnroll];
#pragma unroll
        for (int u = 0; u < kGroupUnroll; u++) pos[u] = atomicAdd(&plds[key[u] >> rshift], act[u] ? 1u : 0u);
#pragma unroll
        for (int u = 0; u < kGroupUnroll; u++)
          if (act[u]) a.emit[pos[u]] = rec[u];
      }
#pragma unroll
      for (int u = 0; u < kGroupUnroll; u++)
        if (act[u]) {
          if (a.reserved2 == 1) {  // debug.emit=1 (timing only, wrong results): sequential stores
            a.emit[doc[u]] = rec[u];
          } else if (a.reserved2 == 2) {  // debug.emit=2: LDS cursor only
            atomicAdd(&plds[key[u] >> a.shift], 1u);
          }
        }
    } else {
      unsigned long long *cnt_g = a.counts;
      uint32_t *cnt_l = reinterpret_cast<uint32_t *>(acc_lds);
#pragma unroll
      for (int u = 0; u < kGroupUnroll; u++)
        if (act[u]) {
          if constexpr (MODE == GB_LDS) atomicAdd(cnt_l + key[u], 1u);
          else atomicAdd(cnt_g + key[u], 1ull);
        }
      for (int g = 0; g < a.n_aggs; g++) {
        const GroupAggDev ag = load_const(a.aggs + sg.first_agg + g);
        if (ag.acc_kind == 5) continue;
        uint32_t id[kGroupUnroll];
#pragma unroll
        for (int u = 0; u < kGroupUnroll; u++) id[u] = decode_doc(ag.fwd, ag.bits, doc[u]);
        void *acc = MODE == GB_LDS ? (void *)(acc_lds + ag.lds_off) : ag.acc;
#pragma unroll
        for (int u = 0; u < kGroupUnroll; u++)
          if (act[u]) agg_update<MODE == GB_LDS>(ag, acc, (long long)key[u], id[u]);
      }
    }
  }
}

// GB_COUNT / GB_EMIT with every needed column prefetched: one global-memory round trip per kGroupPfUnroll
// words instead of one per column (the per-doc reads are latency-bound).
constexpr int kGroupPfUnroll = 4;

template <int MODE>
__device__ __forceinline__ void group_chunk_pf(const GroupArgs &a, const GroupSegment &sg, int64_t ch, uint64_t mask,
                                               int lane, uint32_t *plds) {
  constexpr int C = kGroupPfCols, U = kGroupPfUnroll;
  const int nc = MODE == GB_COUNT ? a.n_gcols : a.pf_nc;
  const uint8_t *fwd[C];
  const int32_t *remap[C];
  unsigned long long stride[C];
  int bits[C], fshift[C];
#pragma unroll
  for (int c = 0; c < C; c++) {
    fwd[c] = nullptr;
    remap[c] = nullptr;
    stride[c] = 0;
    bits[c] = 1;
    fshift[c] = 0;
    if (c < a.n_gcols) {
      const GroupColDev gc = load_const(a.gcols + sg.first_gcol + c);
      fwd[c] = gc.fwd;
      remap[c] = gc.remap;
      stride[c] = (unsigned long long)gc.stride;
      bits[c] = gc.bits;
    } else if (c < nc) {
      const GroupAggDev ag = load_const(a.aggs + sg.first_agg + a.pf_agg[c]);
      fwd[c] = ag.fwd;
      bits[c] = ag.bits;
      fshift[c] = ag.field_shift;
    }
  }
  const int rshift = a.shift + a.split;
  for (int w0 = 0; w0 < 64; w0 += U) {
    uint64_t mw[U];
    bool any = false;
#pragma unroll
    for (int u = 0; u < U; u++) {
      mw[u] = readlane64(mask, w0 + u);
      any = any || mw[u] != 0;
    }
    if (!any) continue;  // uniform
    int64_t doc[U];
    bool act[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      doc[u] = ((ch << 6) + w0 + u) * 64 + lane;
      act[u] = (mw[u] >> lane) & 1ull;
    }
    uint32_t lo[C][U], hi[C][U];
#pragma unroll
    for (int c = 0; c < C; c++)
      if (c < nc) {
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint32_t *p = reinterpret_cast<const uint32_t *>(fwd[c]) + (((uint64_t)doc[u] * (uint32_t)bits[c]) >> 5);
          lo[c][u] = p[0];
          hi[c][u] = p[1];
        }
      }
    unsigned long long key[U], rec[U];
#pragma unroll
    for (int u = 0; u < U; u++) key[u] = rec[u] = 0;
#pragma unroll
    for (int c = 0; c < C; c++)
      if (c < nc) {
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint64_t bitpos = (uint64_t)doc[u] * (uint32_t)bits[c];
          const uint64_t x = ((uint64_t)bswap32(lo[c][u]) << 32) | bswap32(hi[c][u]);
          const uint32_t id = (uint32_t)((x << (bitpos & 31)) >> (64 - bits[c]));
          if (c < a.n_gcols) key[u] += (unsigned long long)(remap[c] ? (uint32_t)remap[c][id] : id) * stride[c];
          else rec[u] |= (unsigned long long)id << fshift[c];
        }
      }
    if (a.admitted) {
#pragma unroll
      for (int u = 0; u < U; u++) act[u] = act[u] && ((a.admitted[key[u] >> 5] >> (key[u] & 31)) & 1u);
    }
    if constexpr (MODE == GB_COUNT) {
#pragma unroll
      for (int u = 0; u < U; u++)
        if (act[u]) atomicAdd(&plds[key[u] >> a.shift], 1u);
    } else {
      uint32_t pos[U];
#pragma unroll
      for (int u = 0; u < U; u++) pos[u] = atomicAdd(&plds[key[u] >> rshift], act[u] ? 1u : 0u);
#pragma unroll
      for (int u = 0; u < U; u++)
        if (act[u]) {
          const unsigned long long r = rec[u] | (key[u] & ((1ull << rshift) - 1ull));
          if (a.nt_store) __builtin_nontemporal_store(r, a.emit + pos[u]);
          else a.emit[pos[u]] = r;
        }
    }
  }
}

// LDS accumulator identities (GB_LDS): counts 0, sums 0, min all-ones, max 0, HLL 0.
__device__ __forceinline__ void init_group_lds(const GroupArgs &a, const GroupSegment &sg, uint8_t *acc_lds, int tid) {
  uint32_t *w = reinterpret_cast<uint32_t *>(acc_lds);
  for (int i = tid; i < a.lds_acc_bytes / 4; i += kGroupBlock) w[i] = 0;
  __syncthreads();
  for (int g = 0; g < a.n_aggs; g++) {
    const GroupAggDev ag = load_const(a.aggs + sg.first_agg + g);
    if (ag.acc_kind == 2) {
      unsigned long long *m = reinterpret_cast<unsigned long long *>(acc_lds + ag.lds_off);
      for (long long i = tid; i < a.G; i += kGroupBlock) m[i] = ~0ull;
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void flush_group_lds(const GroupArgs &a, const GroupSegment &sg, uint8_t *acc_lds, int tid) {
  __syncthreads();
  const uint32_t *cnt = reinterpret_cast<const uint32_t *>(acc_lds);
  for (long long k = tid; k < a.G; k += kGroupBlock) {
    const uint32_t c = cnt[k];
    if (!c) continue;
    atomicAdd(a.counts + k, (unsigned long long)c);
    for (int g = 0; g < a.n_aggs; g++) {
      const GroupAggDev ag = load_const(a.aggs + sg.first_agg + g);
      const uint8_t *src = acc_lds + ag.lds_off;
      switch (ag.acc_kind) {
        case 0:
          atomicAdd(static_cast<unsigned long long *>(ag.acc) + k, reinterpret_cast<const unsigned long long *>(src)[k]);
          break;
        case 1:
          atomicAdd(static_cast<double *>(ag.acc) + k, reinterpret_cast<const double *>(src)[k]);
          break;
        case 2:
          atomicMin(static_cast<unsigned long long *>(ag.acc) + k, reinterpret_cast<const unsigned long long *>(src)[k]);
          break;
        case 3:
          atomicMax(static_cast<unsigned long long *>(ag.acc) + k, reinterpret_cast<const unsigned long long *>(src)[k]);
          break;
        case 4:
          for (int r = 0; r < 256; r++) {
            const uint32_t v = reinterpret_cast<const uint32_t *>(src)[k * 256 + r];
            if (v) hll_max_u8(static_cast<uint8_t *>(ag.acc), k * 256 + r, v);
          }
          break;
        default:
          break;
      }
    }
  }
}

template <int MODE, bool PF = false>
__global__ __launch_bounds__(kGroupBlock) void k_group_query(GroupArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = blockIdx.x / a.bps, b = blockIdx.x % a.bps;
  const int nblk = a.nsegs * a.bps;
  const GroupSegment sg = load_const(a.segs + g);
  const FusedStep *leaves = a.leaves + sg.first_leaf;
  uint8_t *stage = lds + wave * a.stage_bytes;
  uint8_t *acc_lds = lds + (size_t)kGroupWaves * a.stage_bytes;
  uint32_t *plds = reinterpret_cast<uint32_t *>(acc_lds);
  if constexpr (MODE == GB_LDS) init_group_lds(a, sg, acc_lds, tid);
  if constexpr (MODE == GB_COUNT) {
    for (int p = tid; p < a.P; p += kGroupBlock) plds[p] = 0;
    __syncthreads();
  }
  if constexpr (MODE == GB_EMIT) {
    if (a.split == 0) {
      for (int p = tid; p < a.P; p += kGroupBlock) plds[p] = a.offsets[(size_t)p * nblk + blockIdx.x];
    } else {  // coarse run (q, block) starts where run q starts + this block's share of q's earlier blocks
      const int F = 1 << a.split, Q = (a.P + F - 1) >> a.split;
      for (int q = tid; q < Q; q += kGroupBlock) {
        uint32_t c = a.pstart[q * F];
        for (int p = q * F; p < min(a.P, (q + 1) * F); p++) c += a.offsets[(size_t)p * nblk + blockIdx.x] - a.pstart[p];
        plds[q] = c;
      }
    }
    __syncthreads();
  }
  const int64_t nchunks = min((sg.nwords + 63) >> 6, sg.ch_end);
  unsigned long long matched = 0;
  for (int64_t ch = sg.ch_begin + (int64_t)b * kGroupWaves + wave; ch < nchunks; ch += (int64_t)a.bps * kGroupWaves) {
    uint64_t mask = chunk_word(sg.pre, sg.nwords, sg.num_docs, ch, lane);
    mask = eval_filter<true>(leaves, sg.n_leaves, mask, ch * 64 + lane, sg.nwords, sg.num_docs, lane,
                             [&](int, const FusedStep &st) -> const uint8_t * {
                               stage_chunk_rt(st.fwd, st.bits, ch, stage, lane);
                               wait_stage();
                               return stage;
                             });
    matched += __popcll(mask);
    if (__any(mask != 0)) {
      if constexpr (PF) group_chunk_pf<MODE>(a, sg, ch, mask, lane, plds);
      else group_chunk<MODE>(a, sg, ch, mask, lane, acc_lds, plds);
    }
  }
  matched = wave_sum(matched);  // the EMIT pass re-reads what the COUNT pass already counted
  if (MODE != GB_EMIT && MODE != GB_VERIFY && lane == 0 && matched) atomicAdd(a.matched + g, matched);
  if constexpr (MODE == GB_LDS) flush_group_lds(a, sg, acc_lds, tid);
  if constexpr (MODE == GB_COUNT) {
    __syncthreads();
    for (int p = tid; p < a.P; p += kGroupBlock) a.hist[(size_t)p * nblk + blockIdx.x] = plds[p];
  }
}

}  // namespace

int scan_query_blocks_per_cu(int stage_bytes, bool gathers, bool pipelined) {
  static int cache[2][2][20] = {{{0}}};
  const int k = (stage_bytes + 1023) / 1024;
  const bool cacheable = k >= 1 && k < 20;
  if (cacheable && cache[pipelined][gathers][k] > 0) return cache[pipelined][gathers][k];
  const size_t lds = (size_t)kFusedWaves * stage_bytes * (pipelined ? 2 : 1);
  int n = 0;
  hipError_t err;
  if (pipelined)
    err = gathers ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_scan_query_pipe<true>, kBlock, lds)
                  : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_scan_query_pipe<false>, kBlock, lds);
  else
    err = gathers ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_scan_query<true>, kBlock, lds)
                  : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_scan_query<false>, kBlock, lds);
  if (err != hipSuccess || n < 1) n = 1;
  if (cacheable) cache[pipelined][gathers][k] = n;
  return n;
}

void launch_scan_query(const FusedArgs &a, bool gathers, bool pipelined, hipStream_t stream) {
  if (a.nsegs <= 0 || a.bps <= 0) return;
  const dim3 grid((unsigned)(a.nsegs * a.bps)), block(kBlock);
  const size_t lds = (size_t)kFusedWaves * a.stage_bytes * (pipelined ? 2 : 1);
  if (pipelined) {
    if (gathers) hipLaunchKernelGGL(k_scan_query_pipe<true>, grid, block, lds, stream, a);
    else hipLaunchKernelGGL(k_scan_query_pipe<false>, grid, block, lds, stream, a);
  } else {
    if (gathers) hipLaunchKernelGGL(k_scan_query<true>, grid, block, lds, stream, a);
    else hipLaunchKernelGGL(k_scan_query<false>, grid, block, lds, stream, a);
  }
}


size_t group_query_lds_bytes(const GroupArgs &a) {
  size_t acc = 0;
  if (a.mode == GB_LDS) acc = (size_t)a.lds_acc_bytes;
  if (a.mode == GB_COUNT || a.mode == GB_EMIT) acc = (size_t)a.P * 4;
  return (size_t)kGroupWaves * a.stage_bytes + acc;
}

int group_query_blocks_per_cu(const GroupArgs &a) {
  int n = 0;
  const size_t lds = group_query_lds_bytes(a);
  hipError_t err = hipErrorInvalidValue;
  switch (a.mode) {
    case GB_GLOBAL: err = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_group_query<GB_GLOBAL>, kGroupBlock, lds); break;
    case GB_LDS: err = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_group_query<GB_LDS>, kGroupBlock, lds); break;
    case GB_COUNT: err = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_group_query<GB_COUNT>, kGroupBlock, lds); break;
    default: err = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_group_query<GB_EMIT>, kGroupBlock, lds); break;
  }
  return (err != hipSuccess || n < 1) ? 1 : n;
}

void launch_group_query(const GroupArgs &a, hipStream_t stream) {
  if (a.nsegs <= 0 || a.bps <= 0) return;
  const dim3 grid((unsigned)(a.nsegs * a.bps)), block(kGroupBlock);
  const size_t lds = group_query_lds_bytes(a);
  switch (a.mode) {
    case GB_GLOBAL: hipLaunchKernelGGL(k_group_query<GB_GLOBAL>, grid, block, lds, stream, a); break;
    case GB_LDS: hipLaunchKernelGGL(k_group_query<GB_LDS>, grid, block, lds, stream, a); break;
    case GB_COUNT: hipLaunchKernelGGL(k_group_query<GB_COUNT>, grid, block, lds, stream, a); break;  // 2 columns: no gain
    case GB_EMIT:
      if (a.pf_nc > 0) hipLaunchKernelGGL((k_group_query<GB_EMIT, true>), grid, block, lds, stream, a);
      else hipLaunchKernelGGL(k_group_query<GB_EMIT>, grid, block, lds, stream, a);
      break;
    default: hipLaunchKernelGGL(k_group_query<GB_VERIFY>, grid, block, lds, stream, a); break;
  }
}

namespace {
__global__ void k_hash_tuples(GroupArgs a, const long long *__restrict__ slots, long long n, int32_t *ids) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const unsigned long long rep = a.reps[slots[i]];
    const int seg = (int)(rep >> 32);
    const int64_t doc = (int64_t)(rep & 0xFFFFFFFFull);
    for (int j = 0; j < a.n_gcols; j++) ids[i * a.n_gcols + j] = (int32_t)tuple_id(a, seg, j, doc);
  }
}
}  // namespace

void launch_hash_tuples(const GroupArgs &a, const long long *slots, long long n, int32_t *ids, hipStream_t stream) {
  if (n <= 0) return;
  const int grid = (int)std::min<long long>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_hash_tuples, dim3(grid), dim3(256), 0, stream, a, slots, n, ids);
}

}  // namespace pinot
