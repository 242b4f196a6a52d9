// Fused group-by (K6 + K7 over the K1 filter): ONE launch per group-by query over every segment on the GPU.
// Restates DictionaryBasedGroupKeyGenerator (PC/query/aggregation/groupby/DictionaryBasedGroupKeyGenerator.java:195-302)
// and DefaultGroupByExecutor.process (PC/query/aggregation/groupby/DefaultGroupByExecutor.java:70-168) over the
// filter program of fused_common.h (PC = pinot-core/src/main/java/org/apache/pinot/core).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "fused_common.h"
#include "group_lq.h"

namespace pinot {
namespace {
using namespace dev;

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

// Lane of the f-th (0-based) set bit of a 64-bit lane mask (f < popcount(m)).
__device__ __forceinline__ int select_bit(uint64_t m, int f) {
  int pos = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const uint64_t low = m & ((1ull << w) - 1ull);
    const int c = __popcll(low);
    if (f >= c) {
      f -= c;
      m >>= w;
      pos += w;
    } else {
      m = low;
    }
  }
  return pos;
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
    case 0:  // LDS + affine dictionary: Σ dictId here, Σ value = base * count + step * Σ dictId at the flush
      atomicAdd(static_cast<unsigned long long *>(acc) + k,
                LDS && ag.affine ? (unsigned long long)id
                                 : (unsigned long long)(long long)static_cast<const int32_t *>(ag.dict)[id]);
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
    if (MODE != GB_FIRST && sg.admitted) {
#pragma unroll
      for (int u = 0; u < kGroupUnroll; u++)
        act[u] = act[u] && ((sg.admitted[key[u] >> 5] >> (key[u] & 31)) & 1u);
    }
    if constexpr (MODE == GB_VERIFY) {
      continue;
    } else if constexpr (MODE == GB_FIRST) {
      uint32_t *fd = a.first_doc + (size_t)(blockIdx.x / a.bps) * (size_t)a.G;
#pragma unroll
      for (int u = 0; u < kGroupUnroll; u++)  // values only decrease: a stale (larger) read still takes the atomic
        if (act[u] && fd[key[u]] > (uint32_t)doc[u]) atomicMin(fd + key[u], (uint32_t)doc[u]);
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
      // all cursor claims first (inactive lanes add 0: no divergent branch around the LDS atomics, one lgkmcnt
      // wait), then the stores; the runs' lines combine in L2
      uint32_t pos[kGroupUnroll];
#pragma unroll
      for (int u = 0; u < kGroupUnroll; u++) pos[u] = atomicAdd(&plds[key[u] >> rshift], act[u] ? 1u : 0u);
#pragma unroll
      for (int u = 0; u < kGroupUnroll; u++)
        if (act[u]) a.emit[pos[u]] = rec[u];
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

// The sink of U docs per lane (act: the doc passes filter and admission; key: its raw key; rec: its aggregated
// fields, local key bits still clear).
template <int MODE, int U>
__device__ __forceinline__ void group_sink(const GroupArgs &a, uint32_t *plds, const bool (&act)[U],
                                           const unsigned long long (&key)[U], const unsigned long long (&rec)[U],
                                           int lane) {
  const int rshift = a.shift + a.split;
  if constexpr (MODE == GB_COUNT) {
#pragma unroll
    for (int u = 0; u < U; u++)
      if (act[u]) atomicAdd(&plds[key[u] >> a.shift], 1u);
  } else if constexpr (MODE == GB_EMIT2) {
    // LDS [cursor P][count P][written P][bucket P x kBucketRecs]. Per batch of U words: every record claims a
    // slot (count), writes it and bumps `written`; the record that completes a bucket (written ==
    // kBucketRecs - 1) flushes it: the wave moves its flushers' buckets out eight lanes per bucket (one coalesced
    // 64-B piece each) to the block's next run positions, then reopens them. A record that finds its bucket full
    // (only when one batch brings more than kBucketRecs records of a partition) goes straight to its run slot.
    uint32_t *cur = plds, *cnt = plds + a.P, *wrt = plds + 2 * a.P;
    unsigned long long *bkt = reinterpret_cast<unsigned long long *>(plds + ((3 * a.P + 3) & ~3));
    uint32_t p[U], pos[U];
    unsigned long long r[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      p[u] = act[u] ? (uint32_t)(key[u] >> a.shift) : 0u;
      r[u] = rec[u] | (key[u] & ((1ull << a.shift) - 1ull));
      pos[u] = atomicAdd(&cnt[p[u]], act[u] ? 1u : 0u);
    }
    bool fl[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      fl[u] = false;
      if (act[u] && pos[u] < (uint32_t)kBucketRecs) {
        bkt[p[u] * kBucketRecs + pos[u]] = r[u];
        fl[u] = __hip_atomic_fetch_add(&wrt[p[u]], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP) ==
                (uint32_t)kBucketRecs - 1;
      } else if (act[u]) {
        const uint32_t d = atomicAdd(&cur[p[u]], 1u);
        a.emit[d] = r[u];
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t fm = __ballot(fl[u]);
      if (!fm) continue;  // uniform
      const uint32_t dst = fl[u] ? atomicAdd(&cur[p[u]], (uint32_t)kBucketRecs) : 0u;
      const int nf = __popcll(fm);
      for (int f0 = 0; f0 < nf; f0 += 64 / kBucketRecs) {  // uniform: 8 buckets per wave instruction
        const int f = min(f0 + lane / kBucketRecs, nf - 1), i = lane % kBucketRecs;
        const int src = select_bit(fm, f);
        const uint32_t pf = (uint32_t)__shfl((int)p[u], src, 64), df = (uint32_t)__shfl((int)dst, src, 64);
        if (f0 + lane / kBucketRecs < nf) a.emit[df + i] = bkt[pf * kBucketRecs + i];
      }
      if (fl[u]) {
        __hip_atomic_store(&wrt[p[u]], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_store(&cnt[p[u]], 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
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

// GB_COUNT / GB_EMIT with every needed column prefetched: one global-memory round trip per kGroupPfUnroll
// words instead of one per column (the per-doc reads are latency-bound).
constexpr int kGroupPfUnroll = 4;

template <int MODE>
__device__ __forceinline__ void group_chunk_pf(const GroupArgs &a, const GroupSegment &sg, int64_t ch, uint64_t mask,
                                               int lane, uint32_t *plds) {
  constexpr int C = kGroupPfCols, U = kGroupPfUnroll;
  const int nc = MODE == GB_COUNT ? a.n_gcols : a.pf_nc;
  typedef uint32_t u32x2a __attribute__((ext_vector_type(2), aligned(4)));
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
        for (int u = 0; u < U; u++) {  // one 8-byte load per doc and column (the dword pair holding its bits)
          const u32x2a x = *reinterpret_cast<const u32x2a *>(reinterpret_cast<const uint32_t *>(fwd[c]) +
                                                             (((uint64_t)doc[u] * (uint32_t)bits[c]) >> 5));
          lo[c][u] = x.x;
          hi[c][u] = x.y;
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
    if (sg.admitted) {
#pragma unroll
      for (int u = 0; u < U; u++) act[u] = act[u] && ((sg.admitted[key[u] >> 5] >> (key[u] & 31)) & 1u);
    }
    group_sink<MODE, U>(a, plds, act, key, rec, lane);
  }
}

// ---------------------------------------------------------------- lane-owns-word path
// Each lane takes the 64-doc word its filter mask already describes: per half (32 docs) and column it reads
// the B contiguous dwords holding those docs' bits (a wave's reads cover the chunk's 256*B bytes exactly once,
// no per-doc gathers), decodes them with compile-time shifts and folds them into the docs' keys / records; the
// sink then walks the 32 docs of the half, four at a time across the wave.
typedef uint32_t u32x2a_ __attribute__((ext_vector_type(2), aligned(4)));

// Quarter Q (docs 16Q..16Q+15) of a half: only the dwords holding its bits are read.
template <int B, int Q>
__device__ __forceinline__ void load_quarter(const uint8_t *fwd, int64_t half, uint32_t (&D)[B]) {
  constexpr int k0 = (16 * Q * B) >> 5, k1 = (16 * (Q + 1) * B - 1) >> 5;
  const uint32_t *p = reinterpret_cast<const uint32_t *>(fwd) + half * B;
  int k = k0;
#pragma unroll
  for (; k + 3 <= k1; k += 4) {
    const u32x4a x = *reinterpret_cast<const u32x4a *>(p + k);
    D[k] = bswap32(x.x);
    D[k + 1] = bswap32(x.y);
    D[k + 2] = bswap32(x.z);
    D[k + 3] = bswap32(x.w);
  }
#pragma unroll
  for (; k + 1 <= k1; k += 2) {
    const u32x2a_ x = *reinterpret_cast<const u32x2a_ *>(p + k);
    D[k] = bswap32(x.x);
    D[k + 1] = bswap32(x.y);
  }
  if (k == k1) D[k] = bswap32(p[k]);
}

template <int B, int J, int JEND, typename F>
__device__ __forceinline__ void decode_apply(const uint32_t (&D)[B], F &f) {
  constexpr int q = J * B, k = q >> 5, o = q & 31;
  constexpr uint32_t mask = (uint32_t)((1ull << B) - 1ull);
  if constexpr (o + B <= 32) f.template put<J & 15>((D[k] >> (32 - o - B)) & mask);
  else f.template put<J & 15>(__builtin_amdgcn_alignbit(D[k], D[k + 1], 64 - o - B) & mask);
  if constexpr (J + 1 < JEND) decode_apply<B, J + 1, JEND>(D, f);
}

struct KeyFold {  // raw key += global id * stride (DictionaryBasedGroupKeyGenerator's mixed radix)
  uint32_t (&key)[16];
  const int32_t *remap;
  uint32_t stride;
  template <int J>
  __device__ __forceinline__ void put(uint32_t id) {
    key[J] += (remap ? (uint32_t)remap[id] : id) * stride;
  }
};

struct FieldFold {  // record |= dictId << field_shift
  unsigned long long (&rec)[16];
  int shift;
  template <int J>
  __device__ __forceinline__ void put(uint32_t id) {
    rec[J] |= (unsigned long long)id << shift;
  }
};

template <int Q, typename F>
__device__ __forceinline__ void decode_column_quarter(const uint8_t *fwd, int bits, int64_t half, F &f) {
#define PINOT_LW(B)                       \
  {                                       \
    uint32_t D[B];                        \
    load_quarter<B, Q>(fwd, half, D);     \
    decode_apply<B, 16 * Q, 16 * Q + 16>(D, f); \
  }
  switch (bits) {  // widths up to kGroupLwMaxBits (the host routes wider columns through group_chunk_pf)
    case 1: PINOT_LW(1); break;   case 2: PINOT_LW(2); break;   case 3: PINOT_LW(3); break;   case 4: PINOT_LW(4); break;
    case 5: PINOT_LW(5); break;   case 6: PINOT_LW(6); break;   case 7: PINOT_LW(7); break;   case 8: PINOT_LW(8); break;
    case 9: PINOT_LW(9); break;   case 10: PINOT_LW(10); break; case 11: PINOT_LW(11); break; case 12: PINOT_LW(12); break;
    case 13: PINOT_LW(13); break; case 14: PINOT_LW(14); break; case 15: PINOT_LW(15); break; case 16: PINOT_LW(16); break;
    case 17: PINOT_LW(17); break; case 18: PINOT_LW(18); break; case 19: PINOT_LW(19); break; case 20: PINOT_LW(20); break;
    default: break;
  }
#undef PINOT_LW
}

template <int MODE, int Q>
__device__ __forceinline__ void group_quarter_lw(const GroupArgs &a, const GroupSegment &sg, int64_t half, uint32_t mq,
                                                 int lane, uint32_t *plds) {
  constexpr int U = kGroupPfUnroll;
  const int nc = MODE == GB_COUNT ? a.n_gcols : a.pf_nc;
  uint32_t key[16];
  unsigned long long rec[16];
#pragma unroll
  for (int j = 0; j < 16; j++) {
    key[j] = 0;
    rec[j] = 0;
  }
#pragma unroll 1
  for (int c = 0; c < nc; c++) {  // uniform
    if (c < a.n_gcols) {
      const GroupColDev gc = load_const(a.gcols + sg.first_gcol + c);
      KeyFold f{key, gc.remap, (uint32_t)gc.stride};
      decode_column_quarter<Q>(gc.fwd, gc.bits, half, f);
    } else if constexpr (MODE != GB_COUNT) {
      const int ai = c == 1 ? a.pf_agg[1] : c == 2 ? a.pf_agg[2] : a.pf_agg[3];
      const GroupAggDev ag = load_const(a.aggs + sg.first_agg + ai);
      FieldFold f{rec, ag.field_shift};
      decode_column_quarter<Q>(ag.fwd, ag.bits, half, f);
    }
  }
#pragma unroll
  for (int j0 = 0; j0 < 16; j0 += U) {
    bool act[U];
    unsigned long long k[U], r[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      act[u] = (mq >> (j0 + u)) & 1u;
      k[u] = key[j0 + u];
      r[u] = rec[j0 + u];
    }
    if (sg.admitted) {
#pragma unroll
      for (int u = 0; u < U; u++) act[u] = act[u] && ((sg.admitted[k[u] >> 5] >> (k[u] & 31)) & 1u);
    }
    group_sink<MODE, U>(a, plds, act, k, r, lane);
  }
}

template <int MODE>
__device__ __forceinline__ void group_chunk_lw(const GroupArgs &a, const GroupSegment &sg, int64_t ch, uint64_t mask,
                                               int lane, uint32_t *plds) {
  const int64_t word = ch * 64 + lane;
#pragma unroll 1
  for (int h = 0; h < 2; h++) {
    const uint32_t mh = (uint32_t)(mask >> (32 * h));
    if (__any((mh & 0xFFFFu) != 0)) group_quarter_lw<MODE, 0>(a, sg, word * 2 + h, mh & 0xFFFFu, lane, plds);
    if (__any((mh >> 16) != 0)) group_quarter_lw<MODE, 1>(a, sg, word * 2 + h, mh >> 16, lane, plds);
  }
}

// ---------------------------------------------------------------- lane-owns-quarter path (contiguous)
// Pass q of a chunk covers its docs [1024q, 1024q + 1024); lane l takes the 16 docs 1024q + 16l .. +15, i.e. the
// packed quarter qi = 256 ch + 64q + l, whose 16*B bits start at bit 16*B*qi. A wave's loads of one column are
// then the pass's 128*B contiguous bytes, every lane ceil(B/2) contiguous dwords: each cache line is consumed by
// one burst of loads (the lane-owns-word quarters revisit a line after the sink work of the previous quarter, by
// which time L2 has evicted it — twice the algorithmic bytes fetched). For odd B an odd quarter starts 16 bits
// into its first dword: the loaded dwords are funnel-shifted by 16 first. The lane's 16 filter bits are bits
// 16(l & 3) .. +15 of the chunk word 16q + l/4, fetched from the lane that holds it.
template <int B>
__device__ __forceinline__ void load_quarter_lq(const uint8_t *fwd, int64_t qi, uint32_t (&D)[(B + 1) / 2 + 1]) {
  constexpr int N = (B + 1) / 2 + (B & 1);  // dwords covering 16*B bits from a 16-bit offset (odd B)
  const uint32_t *p = reinterpret_cast<const uint32_t *>(fwd) + ((qi * B) >> 1);
  uint32_t R[N];
  int k = 0;
#pragma unroll
  for (; k + 4 <= N; k += 4) {
    const u32x4a x = *reinterpret_cast<const u32x4a *>(p + k);
    R[k] = bswap32(x.x);
    R[k + 1] = bswap32(x.y);
    R[k + 2] = bswap32(x.z);
    R[k + 3] = bswap32(x.w);
  }
#pragma unroll
  for (; k + 2 <= N; k += 2) {
    const u32x2a_ x = *reinterpret_cast<const u32x2a_ *>(p + k);
    R[k] = bswap32(x.x);
    R[k + 1] = bswap32(x.y);
  }
  if (k < N) R[k] = bswap32(p[k]);
  if constexpr (B & 1) {
    const bool odd = qi & 1;
#pragma unroll
    for (int i = 0; i + 1 < N; i++) D[i] = odd ? __builtin_amdgcn_alignbit(R[i], R[i + 1], 16) : R[i];
    D[N - 1] = R[N - 1];
  } else {
#pragma unroll
    for (int i = 0; i < N; i++) D[i] = R[i];
  }
}


template <typename F>
__device__ __forceinline__ void decode_column_lq(const uint8_t *fwd, int bits, int64_t qi, F &f) {
#define PINOT_LQ(B)                        \
  {                                        \
    uint32_t D[(B + 1) / 2 + 1];           \
    load_quarter_lq<B>(fwd, qi, D);        \
    decode_quarter_apply<B, 0>(D, f);      \
  }
  switch (bits) {  // widths up to kGroupLwMaxBits (the host routes wider columns through group_chunk_pf)
    case 1: PINOT_LQ(1); break;   case 2: PINOT_LQ(2); break;   case 3: PINOT_LQ(3); break;   case 4: PINOT_LQ(4); break;
    case 5: PINOT_LQ(5); break;   case 6: PINOT_LQ(6); break;   case 7: PINOT_LQ(7); break;   case 8: PINOT_LQ(8); break;
    case 9: PINOT_LQ(9); break;   case 10: PINOT_LQ(10); break; case 11: PINOT_LQ(11); break; case 12: PINOT_LQ(12); break;
    case 13: PINOT_LQ(13); break; case 14: PINOT_LQ(14); break; case 15: PINOT_LQ(15); break; case 16: PINOT_LQ(16); break;
    case 17: PINOT_LQ(17); break; case 18: PINOT_LQ(18); break; case 19: PINOT_LQ(19); break; case 20: PINOT_LQ(20); break;
    default: break;
  }
#undef PINOT_LQ
}

// GB_EMIT2 sink of a lane's 16 records, every stage batched over them (one LDS round trip per stage instead of
// one per record): claim a slot of the partition's LDS bucket (count), store the record with its valid bit (bit
// 63; records use <= 63 bits), and the record that claimed the last slot flushes the bucket once the quarter's
// stores are issued. Per round every flushing lane takes one bucket: it claims the bucket's run position, lists
// (partition, position) in the wave's LDS flush list at its rank among the flushing lanes (mbcnt), and the wave
// then moves the listed buckets eight lanes per bucket (one coalesced 64-B piece each), waiting for a slot to turn
// valid where its writer has not stored yet (writers claim before the flusher and store with no wait in between,
// so the wait ends), clears the slots and reopens the buckets (count 0: the clears precede it in this wave's LDS
// order). A record that finds its bucket full goes straight to its run slot.
constexpr unsigned long long kRecValid = 1ull << 63;

__device__ __forceinline__ uint32_t rec_partition(unsigned long long r) {
  return (uint32_t)(r >> kRecPartShift) & ((1u << (63 - kRecPartShift)) - 1u);
}

__device__ __forceinline__ void emit2_sink16(const GroupArgs &a, uint32_t *plds, uint32_t act,
                                             const unsigned long long (&rec)[16], int lane) {
  uint32_t *cur = plds, *cnt = plds + a.P;
  unsigned long long *bkt = reinterpret_cast<unsigned long long *>(plds + ((3 * a.P + 3) & ~3));
  unsigned long long *flist = bkt + (size_t)a.P * kBucketRecs + (threadIdx.x >> 6) * 64;
  uint32_t pos[16];
#pragma unroll
  for (int j = 0; j < 16; j++) {
    pos[j] = 0;
    if ((act >> j) & 1u) pos[j] = atomicAdd(&cnt[rec_partition(rec[j])], 1u);
  }
  // bucket stores (no LDS returns: no waits); records that found their bucket full are marked for the run slots
  uint32_t flush = 0, over = 0;
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const bool in = ((act >> j) & 1u) && pos[j] < (uint32_t)kBucketRecs;
    if (in)
      __hip_atomic_store(&bkt[rec_partition(rec[j]) * kBucketRecs + pos[j]], rec[j] | kRecValid, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_WORKGROUP);
    flush |= (in && pos[j] == (uint32_t)kBucketRecs - 1) ? (1u << j) : 0u;
    over |= (((act >> j) & 1u) && !in) ? (1u << j) : 0u;
  }
  if (__any(over != 0)) {  // aligned runs: from the run end backwards, so the flushes stay 64-B aligned
    uint32_t d[16];
    uint32_t *back = plds + 2 * a.P;
#pragma unroll
    for (int j = 0; j < 16; j++)
      if ((over >> j) & 1u)
        d[j] = a.aligned_runs ? atomicSub(&back[rec_partition(rec[j])], 1u) - 1u : atomicAdd(&cur[rec_partition(rec[j])], 1u);
#pragma unroll
    for (int j = 0; j < 16; j++)
      if ((over >> j) & 1u) a.emit[d[j]] = rec[j];
  }
  while (true) {
    const uint64_t fm = __ballot(flush != 0);
    if (!fm) break;  // uniform
    uint32_t p = 0;
    if (flush) {
      const int j = __builtin_ctz(flush);
      unsigned long long pr = 0;
#pragma unroll
      for (int t = 0; t < 16; t++) pr = t == j ? rec[t] : pr;
      p = rec_partition(pr);
      const uint32_t dst = atomicAdd(&cur[p], (uint32_t)kBucketRecs);
      const int f = __builtin_amdgcn_mbcnt_hi((uint32_t)(fm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u));
      flist[f] = ((unsigned long long)dst << 32) | p;
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);  // list writes before the list reads (wave LDS order)
    const int nf = __popcll(fm);
    for (int f0 = 0; f0 < nf; f0 += 64 / kBucketRecs) {  // uniform: 8 buckets per wave instruction
      const int f = f0 + lane / kBucketRecs, i = lane % kBucketRecs;
      if (f < nf) {
        const unsigned long long e = flist[f];
        unsigned long long *slot = &bkt[(uint32_t)e * kBucketRecs + i];
        unsigned long long v = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        while (!(v & kRecValid)) v = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        a.emit[(uint32_t)(e >> 32) + i] = v & ~kRecValid;
        __hip_atomic_store(slot, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    // reopen: a relaxed LDS store after the clears (one wave's LDS operations execute in issue order; the compiler
    // fence keeps that order). A release here would wait for every outstanding HBM store of the wave (vmcnt(0)).
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (flush) {
      __hip_atomic_store(&cnt[p], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      flush &= flush - 1u;
    }
  }
}


// The columns a quarter reads (group columns, then GB_EMIT's aggregated fields): per segment, uniform. The COUNT
// pass (128 VGPRs at 16 waves) keeps raw registers for at most kLqCountCols group columns (the host picks the
// lane-owns-word path for more).
constexpr int kLqCountCols = 2;
struct LqCols {
  const uint8_t *fwd[kGroupPfCols];
  const int32_t *remap[kGroupPfCols];
  uint32_t stride[kGroupPfCols];
  int bits[kGroupPfCols], fsh[kGroupPfCols];  // bits 0 = unused slot; fsh -1 = a group column (key fold)
};

template <int MODE>
__device__ __forceinline__ LqCols lq_cols(const GroupArgs &a, const GroupSegment &sg) {
  const int nc = MODE == GB_COUNT ? a.n_gcols : a.pf_nc;
  LqCols k;
#pragma unroll
  for (int c = 0; c < kGroupPfCols; c++) {
    k.fwd[c] = nullptr;
    k.remap[c] = nullptr;
    k.stride[c] = 0;
    k.bits[c] = 0;
    k.fsh[c] = -1;
    if (c < nc) {
      if (c < a.n_gcols) {
        const GroupColDev gc = load_const(a.gcols + sg.first_gcol + c);
        k.fwd[c] = gc.fwd;
        k.remap[c] = gc.remap;
        k.stride[c] = (uint32_t)gc.stride;
        k.bits[c] = gc.bits;
      } else if (MODE != GB_COUNT) {
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

template <int NC>
__device__ __forceinline__ void lq_load(const LqCols &k, int64_t qi, uint32_t (&R)[NC][12]) {
#pragma unroll
  for (int c = 0; c < NC; c++)
    if (k.bits[c]) load_raw_lq(k.fwd[c], k.bits[c], qi, R[c]);
}

// GB_LDS: column slot C (an aggregated column, compile-time so its raw registers stay registers) folded into the
// block's LDS accumulators of its function, 16 docs per lane.
template <int C, int NC>
__device__ __forceinline__ void lds_sink_col(const GroupArgs &a, const GroupSegment &sg, const LqCols &k,
                                             const uint32_t (&R)[NC][12], int64_t qi, uint32_t act,
                                             const uint32_t (&key)[16], uint32_t *plds) {
  if constexpr (C < NC) {
    if (!k.bits[C] || k.fsh[C] < 0) return;
    const GroupAggDev ag = load_const(a.aggs + sg.first_agg + a.pf_agg[C]);
    uint8_t *acc = reinterpret_cast<uint8_t *>(plds) + ag.lds_off;
    const bool pack = a.lds_pack == a.pf_agg[C];
    decode_raw_lq(R[C], k.bits[C], qi, [&](const uint32_t (&id)[16]) {
      if (pack) {  // count << sbits + Σ dictId in one 64-bit add
#pragma unroll
        for (int j = 0; j < 16; j++)
          if ((act >> j) & 1u)
            atomicAdd(reinterpret_cast<unsigned long long *>(acc) + key[j], (1ull << a.lds_sbits) + (unsigned long long)id[j]);
      } else if (ag.acc_kind == 0 && ag.affine) {  // Σ dictId (converted at the flush)
#pragma unroll
        for (int j = 0; j < 16; j++)
          if ((act >> j) & 1u) atomicAdd(reinterpret_cast<unsigned long long *>(acc) + key[j], (unsigned long long)id[j]);
      } else {
#pragma unroll
        for (int j = 0; j < 16; j++)
          if ((act >> j) & 1u) agg_update<true>(ag, acc, (long long)key[j], id[j]);
      }
    });
  }
}

// Decode a quarter's loaded columns into keys / records, then the sink. The group columns (slots [0, n_gcols)) come
// first; for GB_EMIT2 the key then folds into the record right away (local key | partition << kRecPartShift) so the
// key array is dead while the aggregated columns are decoded (register pressure).
template <int MODE, int NC>
__device__ __forceinline__ void lq_process(const GroupArgs &a, const GroupSegment &sg, const LqCols &k,
                                           const uint32_t (&R)[NC][12], int64_t qi, uint32_t mq, int lane,
                                           uint32_t *plds) {
  constexpr int U = kGroupPfUnroll;
  uint32_t key[16];
#pragma unroll
  for (int j = 0; j < 16; j++) key[j] = 0;
#pragma unroll
  for (int c = 0; c < NC; c++) {
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
  if constexpr (MODE == GB_LDS) {  // block-private LDS accumulators: the count, then each aggregated column's slot
    uint32_t act = mq;
    if (sg.admitted) {
#pragma unroll
      for (int j = 0; j < 16; j++)
        if (!((gload<uint32_t>(sg.admitted + (key[j] >> 5)) >> (key[j] & 31)) & 1u)) act &= ~(1u << j);
    }
    if (a.lds_pack < 0) {
#pragma unroll
      for (int j = 0; j < 16; j++)
        if ((act >> j) & 1u) atomicAdd(plds + key[j], 1u);
    }
    lds_sink_col<1, NC>(a, sg, k, R, qi, act, key, plds);
    lds_sink_col<2, NC>(a, sg, k, R, qi, act, key, plds);
    lds_sink_col<3, NC>(a, sg, k, R, qi, act, key, plds);
    return;
  }
  if constexpr (MODE == GB_EMIT2 || MODE == GB_COUNT) {
    uint32_t act = mq;
    if (sg.admitted) {
#pragma unroll
      for (int j = 0; j < 16; j++)
        if (!((gload<uint32_t>(sg.admitted + (key[j] >> 5)) >> (key[j] & 31)) & 1u)) act &= ~(1u << j);
    }
    if constexpr (MODE == GB_EMIT2) {
      const uint32_t lmask = (1u << a.shift) - 1u;
      unsigned long long rec[16];
#pragma unroll
      for (int j = 0; j < 16; j++)
        rec[j] = (unsigned long long)(key[j] & lmask) | ((unsigned long long)(key[j] >> a.shift) << kRecPartShift);
#pragma unroll
      for (int c = 0; c < NC; c++) {
        if (!k.bits[c] || k.fsh[c] < 0) continue;
        const int fsh = k.fsh[c];
        decode_raw_lq(R[c], k.bits[c], qi, [&](const uint32_t (&id)[16]) {
#pragma unroll
          for (int j = 0; j < 16; j++) rec[j] |= (unsigned long long)id[j] << fsh;
        });
      }
      emit2_sink16(a, plds, act, rec, lane);
    } else {  // partition histogram: LDS adds without return
#pragma unroll
      for (int j = 0; j < 16; j++)
        if ((act >> j) & 1u) atomicAdd(&plds[key[j] >> a.shift], 1u);
    }
    return;
  }
  unsigned long long rec[16];
#pragma unroll
  for (int j = 0; j < 16; j++) rec[j] = 0;
#pragma unroll
  for (int c = 0; c < NC; c++) {
    if (!k.bits[c] || k.fsh[c] < 0) continue;
    const int fsh = k.fsh[c];
    decode_raw_lq(R[c], k.bits[c], qi, [&](const uint32_t (&id)[16]) {
#pragma unroll
      for (int j = 0; j < 16; j++) rec[j] |= (unsigned long long)id[j] << fsh;
    });
  }
#pragma unroll
  for (int j0 = 0; j0 < 16; j0 += U) {
    bool act[U];
    unsigned long long kk[U], r[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      act[u] = (mq >> (j0 + u)) & 1u;
      kk[u] = key[j0 + u];
      r[u] = rec[j0 + u];
    }
    if (sg.admitted) {
#pragma unroll
      for (int u = 0; u < U; u++) act[u] = act[u] && ((gload<uint32_t>(sg.admitted + (kk[u] >> 5)) >> (kk[u] & 31)) & 1u);
    }
    group_sink<MODE, U>(a, plds, act, kk, r, lane);
  }
}

// A lane's raw dwords of a quarter of a column of <= 12 bits (7 dwords at most: two 16-B loads).
__device__ __forceinline__ void load_raw_lq8(const uint8_t *fwd, int bits, int64_t qi, uint32_t (&R)[8]) {
  const uint32_t *p = reinterpret_cast<const uint32_t *>(fwd) + ((qi * bits) >> 1);
  const u32x4a x0 = gload<u32x4a>(p), x1 = gload<u32x4a>(p + 4);
  R[0] = x0.x; R[1] = x0.y; R[2] = x0.z; R[3] = x0.w;
  R[4] = x1.x; R[5] = x1.y; R[6] = x1.z; R[7] = x1.w;
}

// The predicate bits (bit j = value j) of a quarter-form scan leaf (FusedStep of <= 12 bits) over a lane's 16 values.
struct LeafQuarterBits {
  const FusedStep &st;
  uint32_t m;
  template <int J>
  __device__ __forceinline__ void put(uint32_t id) {
    uint32_t x;
    if (st.kind == FK_LEAF_RANGE) x = id - st.lo < st.span ? 1u : 0u;
    else if (st.kind == FK_LEAF_LUT64) x = (uint32_t)(st.lut64 >> (id & 63u)) & 1u;
    else x = (gload<uint32_t>(static_cast<const uint32_t *>(st.table) + (id >> 5)) >> (id & 31u)) & 1u;
    m |= x << J;
  }
};

template <int B>
__device__ __forceinline__ uint32_t leaf_quarter_b(const FusedStep &st, const uint32_t (&Rin)[8], int64_t qi) {
  constexpr int N = (B + 1) / 2 + (B & 1);
  static_assert(N <= 8, "leaf quarter");
  uint32_t R[N];
#pragma unroll
  for (int i = 0; i < N; i++) {
    R[i] = Rin[i];
    asm volatile("" : "+v"(R[i]));
  }
  uint32_t D[(B + 1) / 2 + 1];
  if constexpr (B & 1) {
    const bool odd = qi & 1;
#pragma unroll
    for (int i = 0; i + 1 < N; i++) D[i] = odd ? __builtin_amdgcn_alignbit(bswap32(R[i]), bswap32(R[i + 1]), 16) : bswap32(R[i]);
    D[N - 1] = bswap32(R[N - 1]);
  } else {
#pragma unroll
    for (int i = 0; i < N; i++) D[i] = bswap32(R[i]);
  }
  LeafQuarterBits f{st, 0u};
  decode_quarter_apply<B, 0>(D, f);
  return (st.negate ? ~f.m : f.m) & 0xFFFFu;
}

__device__ __forceinline__ uint32_t leaf_quarter(const FusedStep &st, const uint32_t (&R)[8], int64_t qi) {
  uint32_t m = 0xFFFFu;
#define PINOT_LQF(B) m = leaf_quarter_b<B>(st, R, qi)
  PINOT_WIDTH_SWITCH_12(st.bits, PINOT_LQF)
#undef PINOT_LQF
  return m;
}

// GB_LDS with the filter in quarter form (GroupArgs.qfilter): per quarter the leaf's raw dwords are loaded with the
// group and aggregated columns', the leaf evaluated from registers, the matching docs counted (numDocsScanned), then
// the sink. `mask` holds the `pre` words only.
template <int MODE, int NCOL>
__device__ __forceinline__ void group_chunk_lq_qf(const GroupArgs &a, const GroupSegment &sg, const FusedStep *leaves,
                                                  int64_t ch, uint64_t mask, int lane, uint32_t *plds,
                                                  unsigned long long &matched) {
  const int64_t q0 = ch * 256 + lane;
#pragma unroll 1
  for (int q = 0; q < 4; q++) {
    const int src = 16 * q + (lane >> 2);
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)mask, src, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(mask >> 32), src, 64);
    uint32_t m = (((lane & 2) ? hi : lo) >> (16 * (lane & 1))) & 0xFFFFu;
    if (!__any(m != 0)) continue;
    const LqCols k = lq_cols<MODE>(a, sg);
    const int64_t qi = q0 + 64 * q;
    const bool leaf = sg.n_leaves > 0;  // uniform
    FusedStep st{};
    uint32_t F[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (leaf) {
      st = load_const(leaves);
      load_raw_lq8(st.fwd, st.bits, qi, F);
    }
    uint32_t R[NCOL][12];
    lq_load<NCOL>(k, qi, R);
    if (leaf) m &= leaf_quarter(st, F, qi);
    matched += (unsigned long long)__popc(m);
    if (!__any(m != 0)) continue;
    lq_process<MODE, NCOL>(a, sg, k, R, qi, m, lane, plds);
  }
}

template <int MODE, int NCOL = kGroupPfCols>
__device__ __forceinline__ void group_chunk_lq(const GroupArgs &a, const GroupSegment &sg, int64_t ch, uint64_t mask,
                                               int lane, uint32_t *plds) {
  const int64_t q0 = ch * 256 + lane;
  {
    // (measured: prefetching the next quarter into a second register set was slower — the sink's data-dependent
    // HBM stores also count in vmcnt, so the prefetched quarter's first use waits for everything: vmcnt(0))
#pragma unroll 1
    for (int q = 0; q < 4; q++) {
      const int src = 16 * q + (lane >> 2);
      const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)mask, src, 64);
      const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(mask >> 32), src, 64);
      const uint32_t m = (((lane & 2) ? hi : lo) >> (16 * (lane & 1))) & 0xFFFFu;
      if (!__any(m != 0)) continue;
      const LqCols k = lq_cols<MODE>(a, sg);
      constexpr int NC = MODE == GB_COUNT ? kLqCountCols : NCOL;  // COUNT reads the group columns only
      uint32_t R[NC][12];
      lq_load<NC>(k, q0 + 64 * q, R);
      lq_process<MODE, NC>(a, sg, k, R, q0 + 64 * q, m, lane, plds);
    }
  }
}

// LDS accumulator identities (GB_LDS): counts 0, sums 0, min all-ones, max 0, HLL 0.
__device__ __forceinline__ void init_group_lds(const GroupArgs &a, const GroupSegment &sg, uint8_t *acc_lds, int tid) {
  uint32_t *w = reinterpret_cast<uint32_t *>(acc_lds);
  for (int i = tid; i < a.lds_acc_bytes / 4; i += (int)blockDim.x) w[i] = 0;
  __syncthreads();
  for (int g = 0; g < a.n_aggs; g++) {
    const GroupAggDev ag = load_const(a.aggs + sg.first_agg + g);
    if (ag.acc_kind == 2) {
      unsigned long long *m = reinterpret_cast<unsigned long long *>(acc_lds + ag.lds_off);
      for (long long i = tid; i < a.G; i += (long long)blockDim.x) m[i] = ~0ull;
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void flush_group_lds(const GroupArgs &a, const GroupSegment &sg, uint8_t *acc_lds, int tid) {
  __syncthreads();
  const uint32_t *cnt = reinterpret_cast<const uint32_t *>(acc_lds);
  const unsigned long long *packed =
      a.lds_pack >= 0 ? reinterpret_cast<const unsigned long long *>(acc_lds + load_const(a.aggs + sg.first_agg + a.lds_pack).lds_off)
                      : nullptr;
  const unsigned long long low = a.lds_pack >= 0 ? (1ull << a.lds_sbits) - 1ull : ~0ull;
  for (long long k = tid; k < a.G; k += (long long)blockDim.x) {
    const uint32_t c = packed ? (uint32_t)(packed[k] >> a.lds_sbits) : cnt[k];
    if (!c) continue;
    atomicAdd(a.counts + k, (unsigned long long)c);
    for (int g = 0; g < a.n_aggs; g++) {
      const GroupAggDev ag = load_const(a.aggs + sg.first_agg + g);
      const uint8_t *src = acc_lds + ag.lds_off;
      switch (ag.acc_kind) {
        case 0: {
          unsigned long long v = reinterpret_cast<const unsigned long long *>(src)[k];
          if (g == a.lds_pack) v &= low;
          if (ag.affine) v = (unsigned long long)ag.affine_base * c + (unsigned long long)ag.affine_step * v;  // mod 2^64
          atomicAdd(static_cast<unsigned long long *>(ag.acc) + k, v);
          break;
        }
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

// PATH: 0 = per-column loop, 1 = per-doc prefetch (group_chunk_pf), 2 = lane-owns-word (group_chunk_lw),
// 3 = lane-owns-quarter, contiguous across the wave (group_chunk_lq).
// A block walks groups of kGroupWaves consecutive chunks with stride bps * kGroupWaves whatever its wave count,
// so blocks of every BLK own the same chunks (the COUNT pass's per-block histograms stay valid for EMIT).
template <int MODE, int PATH = 0, int BLK = kGroupBlock, int MINW = 1>  // MINW: minimum waves per SIMD
__global__ __launch_bounds__(BLK, MINW) void k_group_query(GroupArgs a) {
  constexpr int NW = BLK / 64;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = blockIdx.x / a.bps, b = blockIdx.x % a.bps;
  const int nblk = a.nsegs * a.bps;
  const GroupSegment sg = load_const(a.segs + g);
  const FusedStep *leaves = a.leaves + sg.first_leaf;
  uint8_t *stage = lds + wave * a.stage_bytes;
  uint8_t *acc_lds = lds + (size_t)NW * a.stage_bytes;
  uint32_t *plds = reinterpret_cast<uint32_t *>(acc_lds);
  if constexpr (MODE == GB_LDS) init_group_lds(a, sg, acc_lds, tid);
  if constexpr (MODE == GB_COUNT) {
    for (int p = tid; p < a.P; p += BLK) plds[p] = 0;
    __syncthreads();
  }
  if constexpr (MODE == GB_EMIT2) {  // [cursor P][count P][aligned runs: backward cursor = run start + count P]
    for (int p = tid; p < a.P; p += BLK) {
      const size_t i = (size_t)p * nblk + blockIdx.x;
      plds[p] = a.offsets[i];
      plds[a.P + p] = 0;
      plds[2 * a.P + p] = a.aligned_runs ? a.offsets[i] + a.hist[i] : 0u;
    }
    __syncthreads();
  }
  if constexpr (MODE == GB_EMIT) {
    if (a.split == 0) {
      for (int p = tid; p < a.P; p += BLK) plds[p] = a.offsets[(size_t)p * nblk + blockIdx.x];
    } else {  // coarse run (q, block) starts where run q starts + this block's share of q's earlier blocks
      const int F = 1 << a.split, Q = (a.P + F - 1) >> a.split;
      for (int q = tid; q < Q; q += BLK) {
        uint32_t c = a.pstart[q * F];
        for (int p = q * F; p < min(a.P, (q + 1) * F); p++) c += a.offsets[(size_t)p * nblk + blockIdx.x] - a.pstart[p];
        plds[q] = c;
      }
    }
    __syncthreads();
  }
  const int64_t nchunks = min((sg.nwords + 63) >> 6, sg.ch_end);
  unsigned long long matched = 0;
  for (int64_t ch0 = sg.ch_begin + (int64_t)b * kGroupWaves; ch0 < nchunks; ch0 += (int64_t)a.bps * kGroupWaves)
  for (int i = wave; i < kGroupWaves; i += NW) {
    const int64_t ch = ch0 + i;
    if (ch >= nchunks) break;  // uniform
    uint64_t mask;
    const int64_t w = ch * 64 + lane;
    if constexpr (PATH == 5) {  // GB_LDS, quarter-form filter: the `pre` words here, the leaf per quarter
      mask = chunk_word(sg.pre, sg.nwords, sg.num_docs, ch, lane);
      if (__any(mask != 0)) group_chunk_lq_qf<MODE, 3>(a, sg, leaves, ch, mask, lane, plds, matched);
      continue;
    }
    if constexpr (MODE == GB_EMIT2) {  // the filter words the COUNT pass wrote
      mask = w < sg.nwords ? a.filter_out[(size_t)g * a.filter_stride + w] : 0ull;
    } else {
      mask = chunk_word(sg.pre, sg.nwords, sg.num_docs, ch, lane);
      mask = eval_filter<true, 12>(leaves, sg.n_leaves, mask, w, sg.nwords, sg.num_docs, lane,
                                   [&](int, const FusedStep &st) -> const uint8_t * {
                                     stage_chunk_rt(st.fwd, st.bits, ch, stage, lane);
                                     wait_stage();
                                     return stage;
                                   });
      if ((MODE == GB_COUNT || MODE == GB_FILTER) && a.filter_out && w < sg.nwords)
        a.filter_out[(size_t)g * a.filter_stride + w] = mask;
    }
    matched += __popcll(mask);
    if constexpr (MODE == GB_FILTER) continue;  // the filter words only (the ring plan reads them)
    if (__any(mask != 0)) {
      if constexpr (PATH == 3) group_chunk_lq<MODE>(a, sg, ch, mask, lane, plds);
      else if constexpr (PATH == 4) group_chunk_lq<MODE, 3>(a, sg, ch, mask, lane, plds);  // <= 3 columns read
      else if constexpr (PATH == 2) group_chunk_lw<MODE>(a, sg, ch, mask, lane, plds);
      else if constexpr (PATH == 1) group_chunk_pf<MODE>(a, sg, ch, mask, lane, plds);
      else group_chunk<MODE>(a, sg, ch, mask, lane, acc_lds, plds);
    }
  }
  matched = wave_sum(matched);  // the EMIT pass re-reads what the COUNT pass already counted
  if (MODE != GB_EMIT && MODE != GB_EMIT2 && MODE != GB_VERIFY && MODE != GB_FIRST && lane == 0 && matched)
    atomicAdd(a.matched + g, matched);
  if constexpr (MODE == GB_EMIT2) {  // the partially filled buckets, 8 lanes per bucket (+ aligned runs' padding)
    __syncthreads();
    const unsigned long long *bkt = reinterpret_cast<const unsigned long long *>(plds + ((3 * a.P + 3) & ~3));
    const int i = tid % kBucketRecs;
    for (int p = tid / kBucketRecs; p < a.P; p += BLK / kBucketRecs) {
      if ((uint32_t)i < plds[a.P + p]) a.emit[plds[p] + i] = bkt[p * kBucketRecs + i] & ~kRecValid;
      if (a.aligned_runs) {  // run [start, start + count) is full; slots up to the next multiple of 8 are padding
        const size_t r = (size_t)p * nblk + blockIdx.x;
        const uint32_t end = a.offsets[r] + a.hist[r], pad = (uint32_t)(-(int32_t)a.hist[r]) & (kBucketRecs - 1);
        if ((uint32_t)i < pad) a.emit[end + i] = kRecInvalid;
      }
    }
  }
  if constexpr (MODE == GB_LDS) flush_group_lds(a, sg, acc_lds, tid);
  if constexpr (MODE == GB_COUNT) {
    __syncthreads();
    for (int p = tid; p < a.P; p += BLK) a.hist[(size_t)p * nblk + blockIdx.x] = plds[p];
  }
}

// Lane-owns-word EMIT kernels run 512-thread blocks (their 32-doc key / record arrays need the registers).
constexpr int kGroupLwEmitBlock = 512;
// group.emit_block=1024: the lane-owns-quarter bucketed EMIT at 16 waves per block (the sink is LDS-latency bound)
constexpr int kGroupLqEmitBlockWide = 1024;

static int group_block_threads(const GroupArgs &a) {
  if (a.mode == GB_LDS && a.lw == 2 && a.pf_nc > 0) return a.emit_block == 256 ? 256 : kGroupLwEmitBlock;
  if (a.lw == 2 && a.mode == GB_EMIT2 && a.emit_block == kGroupLqEmitBlockWide) return kGroupLqEmitBlockWide;
  return (a.lw && (a.mode == GB_EMIT || a.mode == GB_EMIT2)) ? kGroupLwEmitBlock : kGroupBlock;
}

// Every instance launch_group_query may pick for `a`, through one visitor (occupancy and launch agree); the visitor
// also gets the instance's code (mode * 10000 + read path * 1000 + threads per block, group.last_instance).
template <typename V>
static void with_group_kernel(const GroupArgs &a, V &&v) {
  const bool lw = a.lw && a.pf_nc > 0, lh = lw && a.lw == 2;
#define PINOT_GQ(M, P, B, W) v(&k_group_query<M, P, B, W>, B, (int)(M) * 10000 + (P) * 1000 + (B))
  switch (a.mode) {
    case GB_GLOBAL: PINOT_GQ(GB_GLOBAL, 0, kGroupBlock, 1); break;
    case GB_LDS:
      if (lh && a.emit_block == 256) PINOT_GQ(GB_LDS, 3, 256, 3);  // 3 blocks of 4 waves per CU
      else if (lh && a.pf_nc <= 3 && a.qfilter) PINOT_GQ(GB_LDS, 5, kGroupLwEmitBlock, 4);
      else if (lh && a.pf_nc <= 3) PINOT_GQ(GB_LDS, 4, kGroupLwEmitBlock, 4);
      else if (lh) PINOT_GQ(GB_LDS, 3, kGroupLwEmitBlock, 4);  // 4 waves per SIMD: 2 blocks per CU
      else PINOT_GQ(GB_LDS, 0, kGroupBlock, 1);
      break;
    case GB_COUNT:
      if (lh && a.n_gcols <= kLqCountCols) PINOT_GQ(GB_COUNT, 3, kGroupBlock, 1);
      else if (lw) PINOT_GQ(GB_COUNT, 2, kGroupBlock, 1);
      else if (a.pf_nc > 0) PINOT_GQ(GB_COUNT, 1, kGroupBlock, 1);
      else PINOT_GQ(GB_COUNT, 0, kGroupBlock, 1);
      break;
    case GB_EMIT:
      if (lh) PINOT_GQ(GB_EMIT, 3, kGroupLwEmitBlock, 1);
      else if (lw) PINOT_GQ(GB_EMIT, 2, kGroupLwEmitBlock, 1);
      else if (a.pf_nc > 0) PINOT_GQ(GB_EMIT, 1, kGroupBlock, 1);
      else PINOT_GQ(GB_EMIT, 0, kGroupBlock, 1);
      break;
    case GB_FIRST: PINOT_GQ(GB_FIRST, 0, kGroupBlock, 1); break;
    case GB_FILTER: PINOT_GQ(GB_FILTER, 0, kGroupBlock, 1); break;
    case GB_EMIT2:
      if (lh && a.emit_block == kGroupLqEmitBlockWide) PINOT_GQ(GB_EMIT2, 3, kGroupLqEmitBlockWide, 1);
      else if (lh) PINOT_GQ(GB_EMIT2, 3, kGroupLwEmitBlock, 1);
      else if (lw) PINOT_GQ(GB_EMIT2, 2, kGroupLwEmitBlock, 1);
      else PINOT_GQ(GB_EMIT2, 1, kGroupBlock, 1);
      break;
    default: PINOT_GQ(GB_VERIFY, 0, kGroupBlock, 1); break;
  }
#undef PINOT_GQ
}

}  // namespace

int group_query_instance(const GroupArgs &a) {
  int code = 0;
  with_group_kernel(a, [&](auto, int, int c) { code = c; });
  return code;
}

size_t group_query_lds_bytes(const GroupArgs &a) {
  size_t acc = 0;
  if (a.mode == GB_LDS) acc = (size_t)a.lds_acc_bytes;
  if (a.mode == GB_COUNT || a.mode == GB_EMIT) acc = (size_t)a.P * 4;
  if (a.mode == GB_EMIT2)  // + the per-wave flush lists of the lane-owns-quarter sink
    acc = (size_t)((3 * a.P + 3) & ~3) * 4 + (size_t)a.P * 8 * kBucketRecs + (size_t)(group_block_threads(a) / 64) * 64 * 8;
  return (size_t)(group_block_threads(a) / 64) * a.stage_bytes + acc;
}

int group_query_blocks_per_cu(const GroupArgs &a) {
  int n = 0;
  const size_t lds = group_query_lds_bytes(a);
  hipError_t err = hipErrorInvalidValue;
  with_group_kernel(a, [&](auto kern, int threads, int) { err = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, threads, lds); });
  return (err != hipSuccess || n < 1) ? 1 : n;
}

void launch_group_query(const GroupArgs &a, hipStream_t stream) {
  if (a.nsegs <= 0 || a.bps <= 0) return;
  const size_t lds = group_query_lds_bytes(a);
  with_group_kernel(a, [&](auto kern, int threads, int) {
    hipLaunchKernelGGL(kern, dim3((unsigned)(a.nsegs * a.bps)), dim3(threads), lds, stream, a);
  });
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
