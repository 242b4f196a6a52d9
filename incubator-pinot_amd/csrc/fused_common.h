// Device building blocks shared by the fused query kernels (fused.hip: aggregation; fused_group.hip: group-by):
// LDS-DMA chunk staging, per-width MSB-first big-endian decode (PinotDataBitSet.readInt,
// PC/io/util/PinotDataBitSet.java:79-100), predicate leaves evaluated into 64-bit register masks, and the
// in-register sorted / bitmap index leaves (SortedInvertedIndexBasedFilterOperator, BitmapBasedFilterOperator).
#pragma once
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

// Half of a lane's super-word at byte `off` of a staged chunk (pieces kPieceStride apart: a byte offset o of the
// packed chunk lives at o + kPiecePad * (o >> 10); 8-byte reads never straddle a piece).
__device__ __forceinline__ const uint8_t *staged_at(const uint8_t *stage, uint32_t o) {
  return stage + o + kPiecePad * (o >> 10);
}

template <int B>
__device__ __forceinline__ void decode_half(const uint8_t *stage, uint32_t off, uint32_t (&v)[32]) {
  uint32_t D[B];
  if constexpr (B % 2 == 0) {
#pragma unroll
    for (int i = 0; i < B / 2; i++) {
      const u32x2 x = *reinterpret_cast<const u32x2 *>(staged_at(stage, off + 8 * i));
      D[2 * i] = bswap32(x.x);
      D[2 * i + 1] = bswap32(x.y);
    }
  } else {
#pragma unroll
    for (int i = 0; i < B; i++) D[i] = bswap32(*reinterpret_cast<const uint32_t *>(staged_at(stage, off + 4 * i)));
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
      __builtin_amdgcn_global_load_lds((glob_void_t *)(src + i * 1024), (lds_void_t *)(lds_wave + i * kPieceStride), 16, 0, 2);
  } else {
    for (int i = 0; i < pieces; i++)
      __builtin_amdgcn_global_load_lds((glob_void_t *)(src + i * 1024), (lds_void_t *)(lds_wave + i * kPieceStride), 16, 0, 0);
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


// One step of a chunk at compile-time width B: decode the lane's two halves from LDS and apply.
template <int B, bool G>
__device__ __forceinline__ void leaf_step(const FusedStep &st, const uint8_t *stage, uint32_t off, uint64_t &mask) {
  uint32_t v[32];
  decode_half<B>(stage, off, v);
  const uint32_t m0 = leaf_half<G>(st, v);
  decode_half<B>(stage, off + 4 * B, v);
  const uint32_t m1 = leaf_half<G>(st, v);
  const uint64_t m = ((uint64_t)m1 << 32) | m0;
  mask &= st.negate ? ~m : m;
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

// Widths above MAXB never reach the kernel (the host builds such leaves into the `pre` bitset).
#define PINOT_WIDTH_SWITCH_12(bits, CALL)                                                                      \
  switch (bits) {                                                                                              \
    case 1: CALL(1); break;   case 2: CALL(2); break;   case 3: CALL(3); break;   case 4: CALL(4); break;     \
    case 5: CALL(5); break;   case 6: CALL(6); break;   case 7: CALL(7); break;   case 8: CALL(8); break;     \
    case 9: CALL(9); break;   case 10: CALL(10); break; case 11: CALL(11); break; case 12: CALL(12); break;   \
    default: break;                                                                                            \
  }

template <bool G, int MAXB = 32>
__device__ __forceinline__ void leaf_rt(const FusedStep &st, const uint8_t *stage, uint32_t off, uint64_t &mask) {
#define PINOT_LEAF(B) leaf_step<B, G>(st, stage, off, mask)
  if constexpr (MAXB <= 12) {
    PINOT_WIDTH_SWITCH_12(st.bits, PINOT_LEAF)
  } else {
    PINOT_WIDTH_SWITCH(st.bits, PINOT_LEAF)
  }
#undef PINOT_LEAF
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

// The 64 docs [first, first + 64) (low 16 bits) of one roaring container, as a word.
__device__ __forceinline__ uint64_t container_word(const uint8_t *payload, const RoaringContainer &c, uint32_t first) {
  const uint8_t *p = payload + c.payload_offset;
  uint64_t x = 0;
  if (c.type == 1) {  // bitmap container: 1024 LE u64 words
    const uint8_t *q = p + (first >> 3);
    x = (uint64_t)ld16(q) | ((uint64_t)ld16(q + 2) << 16) | ((uint64_t)ld16(q + 4) << 32) | ((uint64_t)ld16(q + 6) << 48);
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
  return x;
}

__device__ __forceinline__ uint64_t roaring_word(const FusedStep &st, int64_t w) {
  const uint8_t *payload = st.fwd;
  const RoaringContainer *conts = static_cast<const RoaringContainer *>(st.aux0);
  // a chunk's 64 words lie in one 1024-word roaring key: the key, each id's container search and the container header
  // are wave-uniform (scalar loads); only the word inside the container is per lane
  const uint32_t key = (uint32_t)__builtin_amdgcn_readfirstlane((int)(w >> 10));
  const uint32_t first = (uint32_t)(w & 1023) * 64;    // the word's first low-16 doc
  uint64_t x = 0;
  if (st.ops) {  // many dictIds: their containers listed per key (aux1 = key directory, table = container indices)
    const int32_t *kdir = static_cast<const int32_t *>(st.aux1);
    const int32_t *list = static_cast<const int32_t *>(st.table);
    if (key < st.lo) {
      const int l1 = load_const(kdir + key + 1);
      for (int l = load_const(kdir + key); l < l1; l++) x |= container_word(payload, load_const(conts + load_const(list + l)), first);
    }
    return st.negate ? ~x : x;
  }
  const int32_t *dir = static_cast<const int32_t *>(st.aux1);
  const int32_t *ids = static_cast<const int32_t *>(st.table);
  for (int i = 0; i < (int)st.lo; i++) {
    const int id = load_const(ids + i);
    int l = load_const(dir + id), r = load_const(dir + id + 1);
    const int end = r;
    while (l < r) {
      const int m = (l + r) >> 1;
      if (load_const(conts + m).key < key) l = m + 1;
      else r = m;
    }
    if (l >= end) continue;
    const RoaringContainer c = load_const(conts + l);
    if (c.key != key) continue;
    x |= container_word(payload, c, first);
  }
  return st.negate ? ~x : x;
}

// One leaf's 64-bit word for this lane (scan leaves decode the staged chunk).
template <bool G, int MAXB, typename Src>
__device__ __forceinline__ uint64_t leaf_word(const FusedStep &st, int i, int64_t w, int lane, Src &src) {
  if (G && st.kind == FK_LEAF_RANGES) return ranges_word(static_cast<const int32_t *>(st.table), (int)st.lo, w);
  if (G && st.kind == FK_LEAF_ROARING) return roaring_word(st, w);
  uint64_t x = ~0ull;
  leaf_rt<G, MAXB>(st, src(i, st), (uint32_t)(lane * (8 * st.bits)), x);
  return x;
}

// The filter program of a chunk: terms AND-ed into `mask` (early exit once the wave's mask is empty). A term is an
// AND / OR tree in postfix over a register stack (STACK entries s0.. below the running term; the planner starts each node's term
// with its deepest child, so only bushy trees push): nested subtrees of the filter (FilterOperatorUtils.java:74-122
// builds them with AndFilterOperator / OrFilterOperator) stay in registers.
template <bool G, int MAXB = 32, int STACK = kMaxFusedStackGroup, typename Src>
__device__ __forceinline__ uint64_t eval_filter(const FusedStep *__restrict__ steps, int n_leaves, uint64_t mask,
                                                int64_t w, int64_t nwords, int32_t num_docs, int lane, Src &&src) {
  uint64_t term = ~0ull, s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  bool pending = false;
  for (int i = 0; i < n_leaves; i++) {
    const FusedStep st = load_const(steps + i);
    if (st.kind == FK_OP) {  // uniform: the nested term closes into the entry below it
      term = st.join == JOIN_OR ? (s0 | term) : (s0 & term);
      s0 = s1;
      s1 = s2;
      if constexpr (STACK >= 4) s2 = s3;
      continue;
    }
    if (st.join == JOIN_NEW) {
      if (pending) mask &= term;
      pending = false;
      if (!__any(mask != 0)) return 0;  // wave-uniform: nothing left in this chunk, skip its other columns
    }
    uint64_t x = leaf_word<G, MAXB>(st, i, w, lane, src);
    x = w < nwords ? x & tail_mask(w, nwords, num_docs) : 0ull;
    if (st.join == JOIN_NEW) term = x;
    else if (st.join == JOIN_OR) term |= x;
    else if (st.join == JOIN_AND) term &= x;
    else {  // JOIN_PUSH
      if constexpr (STACK >= 4) s3 = s2;
      s2 = s1;
      s1 = s0;
      s0 = term;
      term = x;
    }
    pending = true;
  }
  return pending ? (mask & term) : mask;
}

__device__ __forceinline__ uint64_t chunk_word(const uint64_t *pre, int64_t nwords, int32_t num_docs, int64_t ch,
                                               int lane) {
  const int64_t w = ch * 64 + lane;
  if (w >= nwords) return 0;
  return (pre ? pre[w] : ~0ull) & tail_mask(w, nwords, num_docs);
}

}  // namespace
}  // namespace pinot
