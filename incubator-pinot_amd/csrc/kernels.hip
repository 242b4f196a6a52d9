// HIP/CDNA4 (gfx950) kernels of the Pinot segment executor, besides the fused scan (scan.hip).
//
// K2 ranges_to_bitset SortedInvertedIndexBasedFilterOperator (PC/operator/filter/SortedInvertedIndexBasedFilterOperator.java:59-158)
// K3 roaring_expand   BitmapBasedFilterOperator + BitmapDocIdSet (PC/operator/filter/BitmapBasedFilterOperator.java:69-84,
//                      PC/operator/docidsets/BitmapDocIdSet.java:33-58)
// K6 group_by         DictionaryBasedGroupKeyGenerator + DefaultGroupByExecutor
//                      (PC/query/aggregation/groupby/DictionaryBasedGroupKeyGenerator.java:195-302)
// K7 HLL update       DistinctCountHLLAggregationFunction (register/rank precomputed per dictId on the host)
// plus the device-side packers (synthetic bench columns, sorted-column forward index).
#include "kernels.h"
#include "mv_hash.h"
#include "common.h"

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>

namespace pinot {

namespace {

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ uint64_t tail_mask(int64_t w, int64_t nwords, int32_t num_docs) {
  if (w != nwords - 1) return ~0ull;
  int rem = num_docs - (int)(w * 64);
  return rem >= 64 ? ~0ull : ((1ull << rem) - 1ull);
}

// ------------------------------------------------------------------ K2: sorted ranges
__device__ __forceinline__ void store_mode(uint64_t *out, int64_t w, uint64_t v, int32_t mode) {
  if (mode == CM_AND) v &= out[w];
  else if (mode == CM_OR) v |= out[w];
  out[w] = v;
}

__global__ void k_bitset_combine(uint64_t *__restrict__ dst, const uint64_t *__restrict__ src, int64_t nwords,
                                 int32_t num_docs, int32_t mode, int32_t fill) {
  for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t v = src ? src[w] : (fill ? ~0ull : 0ull);
    store_mode(dst, w, v & tail_mask(w, nwords, num_docs), mode);
  }
}

__global__ void k_ranges_to_bitset(const int32_t *__restrict__ ranges, int32_t n, int64_t nwords, int32_t num_docs,
                                   int32_t mode, uint64_t *__restrict__ out) {
  int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= nwords) return;
  const int64_t lo = w * 64, hi = lo + 63;
  int l = 0, r = n;
  while (l < r) {
    int m = (l + r) >> 1;
    if (ranges[2 * m + 1] < lo) l = m + 1; else r = m;
  }
  uint64_t word = 0;
  for (int i = l; i < n && ranges[2 * i] <= hi; i++) {
    int64_t s = ranges[2 * i] > lo ? ranges[2 * i] - lo : 0;
    int64_t e = ranges[2 * i + 1] < hi ? ranges[2 * i + 1] - lo : 63;
    if (e < s) continue;
    word |= (~0ull >> (63 - e)) & (~0ull << s);
  }
  store_mode(out, w, word & tail_mask(w, nwords, num_docs), mode);
}

// ------------------------------------------------------------------ multi-value scan leaf
// Entry idx of a fixed-bit packed stream (MSB first, big-endian: PinotDataBitSet.readInt); the stream is padded, so
// the second dword is always inside the allocation.
__device__ __forceinline__ uint32_t read_packed(const uint8_t *__restrict__ fwd, int bits, uint64_t idx) {
  const uint64_t bitpos = idx * (uint64_t)bits;
  const uint32_t *p = reinterpret_cast<const uint32_t *>(fwd) + (bitpos >> 5);
  const uint64_t x = ((uint64_t)bswap32(p[0]) << 32) | bswap32(p[1]);
  return (uint32_t)((x << (bitpos & 31)) >> (64 - bits));
}

// One lane per doc, one wave per bitset word: the lane walks its doc's entries (applyMV: any entry in the LUT, or
// for an exclusive predicate every entry), the wave's ballot is the word.
__global__ __launch_bounds__(kBlock) void k_mv_leaf(MvLeafArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t w = wave0; w < a.nwords; w += nwaves) {
    const int64_t doc = w * 64 + lane;
    bool match = false;
    if (doc < a.num_docs) {
      const uint32_t b = a.offsets[doc], e = a.offsets[doc + 1];
      match = a.all != 0;
      for (uint32_t v = b; v < e; v++) {
        const uint32_t id = read_packed(a.fwd, a.bits, v);
        const bool in = (a.lut[id >> 5] >> (id & 31)) & 1u;
        if (a.all ? !in : in) {
          match = !a.all;
          break;
        }
      }
    }
    const uint64_t word = __ballot(match);
    if (lane == 0) store_mode(a.dst, w, word & tail_mask(w, a.nwords, a.num_docs), a.mode);
  }
}

// ------------------------------------------------------------------ aggregations over multi-value columns
__device__ __forceinline__ unsigned long long ordered_u64(double d) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(d);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
  for (int o = 32; o > 0; o >>= 1) v += (unsigned long long)__shfl_xor((long long)v, o, 64);
  return v;
}

// One lane per doc of the bitset (grid-stride); per aggregation register partials folded with wave reductions and
// one memory-side atomic per wave (integer sums exact; double sums within rounding of the reference's own
// summation order, which its combine leaves unspecified).
__global__ __launch_bounds__(kBlock) void k_mv_aggregate(MvAggArgs a) {
  const int lane = threadIdx.x & 63;
  unsigned long long docs = 0;
  unsigned long long cnt[kMaxAggs], isum[kMaxAggs], mn[kMaxAggs], mx[kMaxAggs];
  double dsum[kMaxAggs];
#pragma unroll
  for (int g = 0; g < kMaxAggs; g++) {
    cnt[g] = isum[g] = mx[g] = 0;
    mn[g] = ~0ull;
    dsum[g] = 0.0;
  }
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t ndocs = ((int64_t)a.num_docs + 63) / 64 * 64;
  for (int64_t doc = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; doc < ndocs; doc += stride) {
    bool m = doc < a.num_docs;
    if (m && a.bitset) m = (a.bitset[doc >> 6] >> (doc & 63)) & 1ull;
    if (!m) continue;
    docs++;
#pragma unroll
    for (int g = 0; g < kMaxAggs; g++) {
      if (g >= a.n) break;
      const MvAggSpec &sp = a.specs[g];
      if (sp.kind == MVA_COUNT_DOCS) continue;
      if (sp.kind == MVA_REGS) {  // HyperLogLog.addAll of the doc's registers
        const uint8_t *r = static_cast<const uint8_t *>(sp.dict) + doc * 256;
        for (int j = 0; j < 256; j++)
          if (r[j]) atomicMax(a.hll + g * 256 + j, (uint32_t)r[j]);
        cnt[g]++;
        continue;
      }
      uint32_t b = (uint32_t)doc, e = (uint32_t)doc + 1;
      if (sp.offsets) {
        b = sp.offsets[doc];
        e = sp.offsets[doc + 1];
      }
      for (uint32_t v = b; v < e; v++) {
        const uint32_t id = read_packed(sp.fwd, sp.bits, v);
        cnt[g]++;
        if (sp.kind == MVA_HLL) {
          const uint32_t h = sp.hll_lut[id];
          atomicMax(a.hll + g * 256 + (h >> 8), h & 0xFFu);
          continue;
        }
        if (!sp.numeric) continue;
        double x;
        if (sp.value_kind == 0) {
          const long long iv = static_cast<const int32_t *>(sp.dict)[id];
          isum[g] += (unsigned long long)iv;
          x = (double)iv;
        } else if (sp.value_kind == 1) {
          const long long iv = static_cast<const long long *>(sp.dict)[id];
          isum[g] += (unsigned long long)iv;
          x = (double)iv;
        } else {
          x = static_cast<const double *>(sp.dict)[id];
          dsum[g] += x;
        }
        const unsigned long long o = ordered_u64(x);
        mn[g] = o < mn[g] ? o : mn[g];
        mx[g] = o > mx[g] ? o : mx[g];
      }
    }
  }
  docs = wave_sum_u64(docs);
  if (lane == 0 && docs) atomicAdd(a.docs, docs);
  for (int g = 0; g < a.n; g++) {
    const unsigned long long c = wave_sum_u64(cnt[g]), s = wave_sum_u64(isum[g]);
    double d = dsum[g];
    unsigned long long lo = mn[g], hi = mx[g];
    for (int o = 32; o > 0; o >>= 1) {
      d += __shfl_xor(d, o, 64);
      const unsigned long long l2 = (unsigned long long)__shfl_xor((long long)lo, o, 64);
      const unsigned long long h2 = (unsigned long long)__shfl_xor((long long)hi, o, 64);
      lo = l2 < lo ? l2 : lo;
      hi = h2 > hi ? h2 : hi;
    }
    if (lane == 0 && c) {
      unsigned long long *o = a.out + 5 * g;
      atomicAdd(o, c);
      atomicAdd(o + 1, s);
      if (d != 0.0) atomicAdd(reinterpret_cast<double *>(o + 2), d);
      atomicMin(o + 3, lo);
      atomicMax(o + 4, hi);
    }
  }
}

// ------------------------------------------------------------------ K3: roaring containers -> dense tile
__device__ __forceinline__ uint32_t ld_u16(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }

__global__ __launch_bounds__(kBlock) void k_roaring_expand(const uint8_t *__restrict__ payload,
                                                            const RoaringContainer *__restrict__ containers,
                                                            const int32_t *__restrict__ dir,
                                                            const int32_t *__restrict__ ids, int32_t nids,
                                                            int exclusive, int64_t nwords, int32_t num_docs,
                                                            int32_t mode, uint64_t *__restrict__ out) {
  __shared__ uint32_t tile[2048];  // 65536 docs = one roaring container key
  const int tid = threadIdx.x;
  const uint32_t key = blockIdx.x;
  for (int i = tid; i < 2048; i += kBlock) tile[i] = 0;
  __syncthreads();
  for (int i = 0; i < nids; i++) {
    const int id = ids[i];
    int l = dir[id], r = dir[id + 1];
    while (l < r) {  // first container with key >= this tile's key
      int m = (l + r) >> 1;
      if (containers[m].key < key) l = m + 1; else r = m;
    }
    if (l >= dir[id + 1] || containers[l].key != key) continue;
    const RoaringContainer c = containers[l];
    const uint8_t *p = payload + c.payload_offset;
    if (c.type == 0) {
      for (uint32_t t = tid; t < c.cardinality; t += kBlock) {
        uint32_t low = ld_u16(p + 2 * t);
        atomicOr(&tile[low >> 5], 1u << (low & 31));
      }
    } else if (c.type == 1) {
      for (int t = tid; t < 2048; t += kBlock) {
        uint32_t v = ld_u16(p + 4 * t) | (ld_u16(p + 4 * t + 2) << 16);
        if (v) atomicOr(&tile[t], v);
      }
    } else {
      for (uint32_t t = tid; t < c.cardinality; t += kBlock) {
        uint32_t s = ld_u16(p + 4 * t), len = ld_u16(p + 4 * t + 2);
        uint32_t e = s + len;  // inclusive
        for (uint32_t x = s; x <= e;) {
          uint32_t wd = x >> 5, b0 = x & 31;
          uint32_t b1 = (e >> 5) == wd ? (e & 31) : 31;
          uint32_t mask = (b1 == 31 ? 0xFFFFFFFFu : ((1u << (b1 + 1)) - 1u)) & (0xFFFFFFFFu << b0);
          atomicOr(&tile[wd], mask);
          x = (wd + 1) << 5;
        }
      }
    }
  }
  __syncthreads();
  const int64_t base = (int64_t)key * 1024;
  for (int i = tid; i < 1024; i += kBlock) {
    int64_t w = base + i;
    if (w >= nwords) break;
    uint64_t v = (uint64_t)tile[2 * i] | ((uint64_t)tile[2 * i + 1] << 32);
    if (exclusive) v = ~v;
    store_mode(out, w, v & tail_mask(w, nwords, num_docs), mode);
  }
}

// ------------------------------------------------------------------ K6: group-by (one doc per lane)
__device__ __forceinline__ uint32_t decode_doc(const DevColumn &c, int64_t doc) {
  const uint64_t bitpos = (uint64_t)doc * (uint32_t)c.bits;
  const uint32_t *p = reinterpret_cast<const uint32_t *>(c.fwd) + (bitpos >> 5);
  const uint64_t x = ((uint64_t)bswap32(p[0]) << 32) | bswap32(p[1]);
  return (uint32_t)((x << (bitpos & 31)) >> (64 - c.bits));
}

__device__ __forceinline__ unsigned long long ordered_bits(double d) {
  unsigned long long u = (unsigned long long)__double_as_longlong(d);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}

__device__ __forceinline__ bool group_key(const GroupByProgram &prog, int64_t doc, long long &key) {
  long long k = 0;
#pragma unroll
  for (int j = 0; j < kMaxGroupCols; j++) {
    if (j >= prog.n_gcols) break;
    int32_t id = (int32_t)decode_doc(prog.cols[prog.gcol[j]], doc);
    if (prog.remap[j]) id = prog.remap[j][id];
    k += (long long)id * prog.stride[j];
  }
  key = k;
  if (prog.admitted) return (prog.admitted[k >> 5] >> (k & 31)) & 1u;
  return true;
}

__device__ __forceinline__ double dict_value(const AggSpecDev &s, int value_kind, uint32_t v) {
  switch (value_kind) {
    case 0: return (double)static_cast<const int32_t *>(s.dict)[v];
    case 1: return (double)static_cast<const long long *>(s.dict)[v];
    default: return static_cast<const double *>(s.dict)[v];
  }
}

__global__ __launch_bounds__(kBlock) void k_group_by(GroupByProgram prog, const uint64_t *__restrict__ bitset,
                                                      int64_t nwords, int32_t num_docs) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t waves = (int64_t)gridDim.x * (kBlock / 64);
  for (int64_t w = (int64_t)blockIdx.x * (kBlock / 64) + wave; w < nwords; w += waves) {
    uint64_t m = bitset ? bitset[w] : ~0ull;
    m &= tail_mask(w, nwords, num_docs);
    if (m == 0) continue;
    if (!((m >> lane) & 1ull)) continue;
    const int64_t doc = w * 64 + lane;
    long long key;
    if (!group_key(prog, doc, key)) continue;
    atomicAdd(&prog.counts[key], 1ull);
#pragma unroll
    for (int a = 0; a < kMaxAggs; a++) {
      if (a >= prog.n_aggs) break;
      const int ak = prog.acc_kind[a];
      if (ak == 5) continue;
      const AggSpecDev &s = prog.aggs[a];
      const uint32_t v = decode_doc(prog.cols[s.col], doc);
      switch (ak) {
        case 0:
          atomicAdd(static_cast<unsigned long long *>(prog.acc[a]) + key,
                    (unsigned long long)(long long)static_cast<const int32_t *>(s.dict)[v]);
          break;
        case 1:
          atomicAdd(static_cast<double *>(prog.acc[a]) + key, dict_value(s, prog.value_kind[a], v));
          break;
        case 2:
          atomicMin(static_cast<unsigned long long *>(prog.acc[a]) + key,
                    ordered_bits(dict_value(s, prog.value_kind[a], v)));
          break;
        case 3:
          atomicMax(static_cast<unsigned long long *>(prog.acc[a]) + key,
                    ordered_bits(dict_value(s, prog.value_kind[a], v)));
          break;
        case 4: {
          const uint32_t e = s.hll_lut[v];
          atomicMax(static_cast<uint32_t *>(prog.acc[a]) + key * 256 + (e >> 8), e & 0xFFu);
          break;
        }
        default: break;
      }
    }
  }
}

__device__ __forceinline__ void mv_fold(const MvGroupArgs &a, int g, long long key, uint32_t b, uint32_t e) {
  const int ak = a.acc_kind[g];
  if (ak == 6) {
    atomicAdd(static_cast<unsigned long long *>(a.acc[g]) + key, (unsigned long long)(e - b));
    return;
  }
  if (ak == 8) {  // a star-tree's HyperLogLog column: the doc's 256 registers max-merged (HyperLogLog.addAll)
    const uint8_t *r = static_cast<const uint8_t *>(a.dict[g]) + (size_t)b * 256;
    for (int j = 0; j < 256; j++)
      if (r[j]) atomicMax(static_cast<uint32_t *>(a.acc[g]) + key * 256 + j, (uint32_t)r[j]);
    return;
  }
  for (uint32_t v = b; v < e; v++) {
    const uint32_t id = read_packed(a.afwd[g], a.abits[g], v);
    switch (ak) {
      case 0:
        atomicAdd(static_cast<unsigned long long *>(a.acc[g]) + key,
                  (unsigned long long)(long long)static_cast<const int32_t *>(a.dict[g])[id]);
        break;
      case 1:
      case 2:
      case 3: {
        double x;
        switch (a.value_kind[g]) {
          case 0: x = (double)static_cast<const int32_t *>(a.dict[g])[id]; break;
          case 1: x = (double)static_cast<const long long *>(a.dict[g])[id]; break;
          default: x = static_cast<const double *>(a.dict[g])[id]; break;
        }
        if (ak == 1) atomicAdd(static_cast<double *>(a.acc[g]) + key, x);
        else if (ak == 2) atomicMin(static_cast<unsigned long long *>(a.acc[g]) + key, ordered_bits(x));
        else atomicMax(static_cast<unsigned long long *>(a.acc[g]) + key, ordered_bits(x));
        break;
      }
      case 4: {
        const uint32_t h = a.hll_lut[g][id];
        atomicMax(static_cast<uint32_t *>(a.acc[g]) + key * 256 + (h >> 8), h & 0xFFu);
        break;
      }
      case 7:  // exact int64 sum over an int64 dictionary (a star-tree's count__* column)
        atomicAdd(static_cast<unsigned long long *>(a.acc[g]) + key,
                  (unsigned long long)static_cast<const long long *>(a.dict[g])[id]);
        break;
      default: break;
    }
  }
}

__device__ __forceinline__ unsigned long long mv_mix(unsigned long long x) {
  x ^= x >> 33;
  x *= 0xFF51AFD7ED558CCDull;
  x ^= x >> 33;
  x *= 0xC4CEB9FE1A85EC53ull;
  x ^= x >> 33;
  return x;
}

// global id of group column j at entry position v
__device__ __forceinline__ int32_t mv_gid(const MvGroupArgs &a, int j, uint32_t v) {
  const int32_t id = (int32_t)read_packed(a.gfwd[j], a.gbits[j], v);
  return a.remap[j] ? a.remap[j][id] : id;
}

// the tuple's fingerprint (never 0: 0 marks an empty slot)
__device__ __forceinline__ unsigned long long mv_fingerprint(const MvGroupArgs &a, const MvHash &h, const uint32_t *cur) {
  unsigned long long fp = h.hseed;
  for (int j = 0; j < a.n_gcols; j++)
    fp = mv_mix(fp ^ ((unsigned long long)(uint32_t)mv_gid(a, j, cur[j]) + 0x9E3779B97F4A7C15ull * (unsigned long long)(j + 1)));
  return fp | 1ull;
}

// The key of the odometer position `cur`: the dense mixed-radix key, or (H) the slot of its tuple; -1 = the slot holds
// another tuple under the same fingerprint (reported, the key dropped: the host retries with another seed).
template <bool H>
__device__ __forceinline__ long long mv_key(const MvGroupArgs &a, const MvHash &h, const uint32_t *cur) {
  if constexpr (!H) {
    long long key = 0;
    for (int j = 0; j < a.n_gcols; j++) key += (long long)mv_gid(a, j, cur[j]) * a.stride[j];
    return key;
  } else {
    const unsigned long long fp = mv_fingerprint(a, h, cur);
    const unsigned long long m = (unsigned long long)h.hcap - 1ull;
    unsigned long long slot = fp & m;
    for (long long probe = 0; probe < h.hcap; probe++) {
      const unsigned long long c = h.htable[slot];
      if (c == fp) break;
      if (c == 0) {
        atomicOr(h.verify_err, 1u);  // inserted by the previous pass: unreachable
        return -1;
      }
      slot = (slot + 1) & m;
    }
    const int32_t *t = h.tuples + (size_t)slot * a.n_gcols;
    for (int j = 0; j < a.n_gcols; j++)
      if (t[j] != mv_gid(a, j, cur[j])) {
        atomicOr(h.verify_err, 1u);
        return -1;
      }
    return (long long)slot;
  }
}

// the doc's entry ranges per group column; false = some column has no entry (no keys)
__device__ __forceinline__ bool mv_ranges(const MvGroupArgs &a, int64_t doc, uint32_t *lo, uint32_t *hi, uint32_t *cur) {
  bool empty = false;
  for (int j = 0; j < a.n_gcols; j++) {
    lo[j] = a.goff[j] ? a.goff[j][doc] : (uint32_t)doc;
    hi[j] = a.goff[j] ? a.goff[j][doc + 1] : (uint32_t)doc + 1;
    cur[j] = lo[j];
    empty = empty || hi[j] <= lo[j];
  }
  return !empty;
}

// odometer step, column 0 fastest; false after the last combination
__device__ __forceinline__ bool mv_next(int n, const uint32_t *lo, const uint32_t *hi, uint32_t *cur) {
  for (int j = 0; j < n; j++) {
    if (++cur[j] < hi[j]) return true;
    cur[j] = lo[j];
  }
  return false;
}

template <bool H>
__global__ __launch_bounds__(kBlock) void k_group_by_mv(MvGroupArgs a, MvHash h) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t doc = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; doc < a.num_docs; doc += stride) {
    if (a.bitset && !((a.bitset[doc >> 6] >> (doc & 63)) & 1ull)) continue;
    uint32_t lo[kMaxGroupCols], hi[kMaxGroupCols], cur[kMaxGroupCols];
    if (!mv_ranges(a, doc, lo, hi, cur)) continue;  // a row without entries yields no group key
    uint32_t ab[kMaxAggs], ae[kMaxAggs];
    for (int g = 0; g < a.n_aggs; g++) {
      ab[g] = a.aoff[g] ? a.aoff[g][doc] : (uint32_t)doc;
      ae[g] = a.aoff[g] ? a.aoff[g][doc + 1] : (uint32_t)doc + 1;
    }
    do {
      const long long key = mv_key<H>(a, h, cur);
      // dropped: a fingerprint collision, or INVALID_ID (holder full: not admitted)
      if (key < 0 || (a.admitted && !((a.admitted[key >> 5] >> (key & 31)) & 1u))) continue;
      atomicAdd(a.counts + key, 1ull);
      for (int g = 0; g < a.n_aggs; g++)
        if (a.acc_kind[g] != 5) mv_fold(a, g, key, ab[g], ae[g]);
    } while (mv_next(a.n_gcols, lo, hi, cur));
  }
}

__global__ __launch_bounds__(kBlock) void k_mv_key_count(MvGroupArgs a, unsigned long long *total) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  unsigned long long mine = 0;
  for (int64_t doc = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; doc < a.num_docs; doc += stride) {
    if (a.bitset && !((a.bitset[doc >> 6] >> (doc & 63)) & 1ull)) continue;
    unsigned long long p = 1;
    for (int j = 0; j < a.n_gcols; j++)
      p *= a.goff[j] ? (unsigned long long)(a.goff[j][doc + 1] - a.goff[j][doc]) : 1ull;
    mine += p;
  }
  for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o);
  if ((threadIdx.x & 63) == 0 && mine) atomicAdd(total, mine);
}

__global__ __launch_bounds__(kBlock) void k_mv_hash_insert(MvGroupArgs a, MvHash h) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const unsigned long long m = (unsigned long long)h.hcap - 1ull;
  for (int64_t doc = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; doc < a.num_docs; doc += stride) {
    if (a.bitset && !((a.bitset[doc >> 6] >> (doc & 63)) & 1ull)) continue;
    uint32_t lo[kMaxGroupCols], hi[kMaxGroupCols], cur[kMaxGroupCols];
    if (!mv_ranges(a, doc, lo, hi, cur)) continue;
    do {
      const unsigned long long fp = mv_fingerprint(a, h, cur);
      unsigned long long slot = fp & m;
      for (long long probe = 0; probe < h.hcap; probe++) {
        unsigned long long c = __hip_atomic_load(h.htable + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (c == 0) {
          c = atomicCAS(h.htable + slot, 0ull, fp);
          if (c == 0) {  // this lane owns the slot: its tuple (read by the later passes only)
            int32_t *t = h.tuples + (size_t)slot * a.n_gcols;
            for (int j = 0; j < a.n_gcols; j++) t[j] = mv_gid(a, j, cur[j]);
            break;
          }
        }
        if (c == fp) break;
        slot = (slot + 1) & m;
      }
    } while (mv_next(a.n_gcols, lo, hi, cur));
  }
}

__global__ void k_mv_hash_tuples(MvHash h, int n_gcols, const long long *__restrict__ slots, long long n,
                                 int32_t *__restrict__ ids) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n * n_gcols;
       i += (long long)gridDim.x * blockDim.x) {
    const long long g = i / n_gcols;
    ids[i] = h.tuples[(size_t)slots[g] * n_gcols + (i - g * n_gcols)];
  }
}

// Keys of a doc in getIntRawKeys order: the highest-index multi-value column fastest (its values outermost-first
// build the array, each lower-index column's values then repeat the array: DictionaryBasedGroupKeyGenerator
// .java:344-410); position = the key's index in that list. Keys repeat when a row repeats a value; the first one counts.
template <bool H>
__global__ __launch_bounds__(kBlock) void k_first_pos_mv(MvGroupArgs a, MvHash h, unsigned long long *first_pos) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t doc = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; doc < a.num_docs; doc += stride) {
    if (a.bitset && !((a.bitset[doc >> 6] >> (doc & 63)) & 1ull)) continue;
    uint32_t lo[kMaxGroupCols], hi[kMaxGroupCols], cur[kMaxGroupCols];
    if (!mv_ranges(a, doc, lo, hi, cur)) continue;
    unsigned long long pos = (unsigned long long)doc << 32;
    while (true) {
      const long long key = mv_key<H>(a, h, cur);
      // values only decrease: a stale read still takes it
      if (key >= 0 && first_pos[key] > pos) atomicMin(first_pos + key, pos);
      pos++;
      int j = a.n_gcols - 1;
      for (; j >= 0; j--) {
        if (++cur[j] < hi[j]) break;
        cur[j] = lo[j];
      }
      if (j < 0) break;
    }
  }
}

__global__ void k_admit_bitmap_u64(const unsigned long long *__restrict__ first_pos, long long G,
                                   const unsigned long long *__restrict__ sorted, long long upper,
                                   uint32_t *__restrict__ bitmap, long long words) {
  const unsigned long long t = (sorted && upper <= G) ? sorted[upper - 1] : ~0ull - 1ull;
  for (long long w = (long long)blockIdx.x * blockDim.x + threadIdx.x; w < words; w += (long long)gridDim.x * blockDim.x) {
    uint32_t m = 0;
    for (int b = 0; b < 32; b++) {
      const long long k = w * 32 + b;
      if (k >= G) break;
      const unsigned long long fp = first_pos[k];
      m |= (fp != ~0ull && fp <= t) ? (1u << b) : 0u;
    }
    bitmap[w] = m;
  }
}

__global__ __launch_bounds__(kBlock) void k_first_doc(GroupByProgram prog, const uint64_t *__restrict__ bitset,
                                                       int64_t nwords, int32_t num_docs, uint32_t *first_doc) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t waves = (int64_t)gridDim.x * (kBlock / 64);
  GroupByProgram p = prog;
  p.admitted = nullptr;
  for (int64_t w = (int64_t)blockIdx.x * (kBlock / 64) + wave; w < nwords; w += waves) {
    uint64_t m = bitset ? bitset[w] : ~0ull;
    m &= tail_mask(w, nwords, num_docs);
    if (!((m >> lane) & 1ull)) continue;
    const int64_t doc = w * 64 + lane;
    long long key;
    group_key(p, doc, key);
    atomicMin(first_doc + key, (uint32_t)doc);
  }
}

__global__ void k_compact_keys(int64_t G, const unsigned long long *__restrict__ counts, long long *keys,
                               unsigned long long *n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < G; i += (int64_t)gridDim.x * blockDim.x) {
    if (counts[i]) keys[atomicAdd(n, 1ull)] = i;
  }
}

// Gather the accumulators of the non-empty keys into dense per-group arrays.
__global__ void k_gather_groups(GroupByProgram prog, const long long *__restrict__ keys, int64_t n,
                                unsigned long long *__restrict__ out_counts, unsigned long long *__restrict__ out_acc,
                                uint8_t *__restrict__ out_hll) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const long long k = keys[i];
    out_counts[i] = prog.counts[k];
    int h = 0;
    for (int a = 0; a < prog.n_aggs; a++) {
      const int ak = prog.acc_kind[a];
      if (ak == 4) {
        const uint32_t *r = static_cast<const uint32_t *>(prog.acc[a]) + k * 256;
        uint8_t *o = out_hll + ((int64_t)h * n + i) * 256;
        for (int j = 0; j < 256; j++) o[j] = (uint8_t)r[j];
        h++;
      } else if (ak != 5) {
        out_acc[(int64_t)a * n + i] = static_cast<const unsigned long long *>(prog.acc[a])[k];
      }
    }
  }
}

// ------------------------------------------------------------------ packing (synthetic + sorted columns)
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Packs 64 values of super-word w (MSB-first, big-endian) as 2*bits dwords.
template <typename F>
__device__ __forceinline__ void pack_superword(int64_t w, int32_t bits, uint8_t *out, F value) {
  uint32_t *o = reinterpret_cast<uint32_t *>(out + (size_t)w * 8 * bits);
  uint64_t acc = 0;
  int nb = 0, k = 0;
  for (int j = 0; j < 64; j++) {
    acc = (acc << bits) | (uint64_t)value(w * 64 + j);
    nb += bits;
    while (nb >= 32) {
      o[k++] = bswap32((uint32_t)(acc >> (nb - 32)));
      nb -= 32;
      acc &= (nb == 0) ? 0ull : ((1ull << nb) - 1ull);
    }
  }
}

__global__ void k_synth_column(uint64_t seed, int32_t card, int32_t bits, int32_t num_docs, int64_t nwords,
                               uint8_t *out) {
  int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= nwords) return;
  pack_superword(w, bits, out, [&](int64_t d) -> uint32_t {
    if (d >= num_docs) return 0u;
    if (d < card) return (uint32_t)d;
    return (uint32_t)(splitmix64(seed ^ ((uint64_t)d * 0x9E3779B97F4A7C15ull)) % (uint64_t)card);
  });
}

__global__ void k_sorted_to_fwd(const int32_t *__restrict__ starts, int32_t card, int32_t bits, int32_t num_docs,
                                int64_t nwords, uint8_t *out) {
  int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= nwords) return;
  // id = last dictId whose start <= first doc of the word
  int64_t d0 = w * 64;
  int l = 0, r = card;
  while (l < r) {
    int m = (l + r) >> 1;
    if (starts[m + 1] <= d0) l = m + 1; else r = m;
  }
  int id = l;
  pack_superword(w, bits, out, [&](int64_t d) -> uint32_t {
    if (d >= num_docs) return 0u;
    while (id + 1 < card && starts[id + 1] <= d) id++;
    return (uint32_t)id;
  });
}

}  // namespace

// ------------------------------------------------------------------ launchers
static int grid_for(int64_t items, int per_block, int cap) {
  int64_t g = (items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

namespace {
unsigned mv_blocks(const MvGroupArgs &a) {
  return (unsigned)std::min<int64_t>(((int64_t)a.num_docs + kBlock - 1) / kBlock, 4096);
}
}  // namespace

void launch_group_by_mv(const MvGroupArgs &a, hipStream_t stream) {
  if (a.num_docs <= 0) return;
  hipLaunchKernelGGL(k_group_by_mv<false>, dim3(mv_blocks(a)), dim3(kBlock), 0, stream, a, MvHash{});
}

void launch_first_pos_mv(const MvGroupArgs &a, unsigned long long *first_pos, hipStream_t stream) {
  if (a.num_docs <= 0) return;
  hipLaunchKernelGGL(k_first_pos_mv<false>, dim3(mv_blocks(a)), dim3(kBlock), 0, stream, a, MvHash{}, first_pos);
}

void launch_mv_key_count(const MvGroupArgs &a, unsigned long long *total, hipStream_t stream) {
  if (a.num_docs <= 0) return;
  hipLaunchKernelGGL(k_mv_key_count, dim3(mv_blocks(a)), dim3(kBlock), 0, stream, a, total);
}

void launch_mv_hash_insert(const MvGroupArgs &a, const MvHash &h, hipStream_t stream) {
  if (a.num_docs <= 0) return;
  hipLaunchKernelGGL(k_mv_hash_insert, dim3(mv_blocks(a)), dim3(kBlock), 0, stream, a, h);
}

void launch_group_by_mv_hashed(const MvGroupArgs &a, const MvHash &h, hipStream_t stream) {
  if (a.num_docs <= 0) return;
  hipLaunchKernelGGL(k_group_by_mv<true>, dim3(mv_blocks(a)), dim3(kBlock), 0, stream, a, h);
}

void launch_first_pos_mv_hashed(const MvGroupArgs &a, const MvHash &h, unsigned long long *first_pos,
                                hipStream_t stream) {
  if (a.num_docs <= 0) return;
  hipLaunchKernelGGL(k_first_pos_mv<true>, dim3(mv_blocks(a)), dim3(kBlock), 0, stream, a, h, first_pos);
}

void launch_mv_hash_tuples(const MvHash &h, int n_gcols, const long long *slots, long long n, int32_t *ids,
                           hipStream_t stream) {
  if (n <= 0) return;
  const long long grid = std::min<long long>((n * n_gcols + 255) / 256, 8192);
  hipLaunchKernelGGL(k_mv_hash_tuples, dim3((unsigned)grid), dim3(256), 0, stream, h, n_gcols, slots, n, ids);
}

size_t admission_scratch_bytes_u64(long long G) {
  size_t need = 0;
  PINOT_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, need, (const unsigned long long *)nullptr,
                                              (unsigned long long *)nullptr, (int)G));
  return ((size_t)G * 8 + 255) / 256 * 256 + need + 256;
}

void launch_admission_bitmap_u64(const unsigned long long *first_pos, long long G, long long upper, uint32_t *bitmap,
                                 long long words, void *scratch, size_t scratch_bytes, hipStream_t stream) {
  auto *sorted = static_cast<unsigned long long *>(scratch);
  const size_t sorted_b = ((size_t)G * 8 + 255) / 256 * 256;
  const bool limited = upper < G;
  if (limited) {
    size_t tb = scratch_bytes - sorted_b;
    PINOT_HIP(hipcub::DeviceRadixSort::SortKeys(static_cast<uint8_t *>(scratch) + sorted_b, tb, first_pos, sorted,
                                                (int)G, 0, 64, stream));
  }
  const int grid = (int)std::min<long long>((words + 255) / 256, 4096);
  hipLaunchKernelGGL(k_admit_bitmap_u64, dim3(grid), dim3(256), 0, stream, first_pos, G, limited ? sorted : nullptr,
                     limited ? upper : G + 1, bitmap, words);
}

void launch_mv_aggregate(const MvAggArgs &a, hipStream_t stream) {
  if (a.num_docs <= 0) return;
  const int64_t blocks = std::min<int64_t>(((int64_t)a.num_docs + kBlock - 1) / kBlock, 4096);
  hipLaunchKernelGGL(k_mv_aggregate, dim3((unsigned)blocks), dim3(kBlock), 0, stream, a);
}

void launch_mv_leaf(const MvLeafArgs &a, hipStream_t stream) {
  if (a.nwords <= 0) return;
  const int64_t blocks = std::min<int64_t>((a.nwords * 64 + kBlock - 1) / kBlock, 8192);
  hipLaunchKernelGGL(k_mv_leaf, dim3((unsigned)blocks), dim3(kBlock), 0, stream, a);
}

void launch_ranges_to_bitset(const int32_t *ranges, int32_t nranges, int64_t nwords, int32_t num_docs,
                             int32_t mode, uint64_t *out, hipStream_t stream) {
  if (nwords <= 0) return;
  hipLaunchKernelGGL(k_ranges_to_bitset, dim3((unsigned)((nwords + 255) / 256)), dim3(256), 0, stream, ranges,
                     nranges, nwords, num_docs, mode, out);
}

void launch_roaring_expand(const uint8_t *payload, const RoaringContainer *containers, const int32_t *dir,
                           const int32_t *ids, int32_t nids, int exclusive, int64_t nwords, int32_t num_docs,
                           int32_t mode, uint64_t *out, hipStream_t stream) {
  if (nwords <= 0) return;
  unsigned tiles = (unsigned)((nwords + 1023) / 1024);
  hipLaunchKernelGGL(k_roaring_expand, dim3(tiles), dim3(kBlock), 0, stream, payload, containers, dir, ids, nids,
                     exclusive, nwords, num_docs, mode, out);
}

void launch_bitset_combine(uint64_t *dst, const uint64_t *src, int64_t nwords, int32_t num_docs, int32_t mode,
                           int32_t fill, hipStream_t stream) {
  if (nwords <= 0) return;
  hipLaunchKernelGGL(k_bitset_combine, dim3(grid_for(nwords, 256, 4096)), dim3(256), 0, stream, dst, src, nwords,
                     num_docs, mode, fill);
}

void launch_group_by(const GroupByProgram &prog, const uint64_t *bitset, int64_t nwords, int32_t num_docs,
                     hipStream_t stream) {
  if (nwords <= 0) return;
  int grid = grid_for(nwords, 4 * 16, 4096);
  hipLaunchKernelGGL(k_group_by, dim3(grid), dim3(kBlock), 0, stream, prog, bitset, nwords, num_docs);
}

void launch_first_doc(const GroupByProgram &prog, const uint64_t *bitset, int64_t nwords, int32_t num_docs,
                      uint32_t *first_doc, hipStream_t stream) {
  if (nwords <= 0) return;
  int grid = grid_for(nwords, 4 * 16, 4096);
  hipLaunchKernelGGL(k_first_doc, dim3(grid), dim3(kBlock), 0, stream, prog, bitset, nwords, num_docs, first_doc);
}

void launch_gather_groups(const GroupByProgram &prog, const long long *keys, int64_t n, unsigned long long *out_counts,
                          unsigned long long *out_acc, uint8_t *out_hll, hipStream_t stream) {
  if (n <= 0) return;
  int grid = grid_for(n, 256, 4096);
  hipLaunchKernelGGL(k_gather_groups, dim3(grid), dim3(256), 0, stream, prog, keys, n, out_counts, out_acc, out_hll);
}

void launch_compact_keys(int64_t G, const unsigned long long *counts, long long *keys_out, unsigned long long *n_out,
                         hipStream_t stream) {
  int grid = grid_for(G, 256, 8192);
  hipLaunchKernelGGL(k_compact_keys, dim3(grid), dim3(256), 0, stream, G, counts, keys_out, n_out);
}

void launch_synth_column(uint64_t seed, int32_t card, int32_t bits, int32_t num_docs, uint8_t *out,
                         hipStream_t stream) {
  int64_t nwords = (num_docs + 63) / 64;
  hipLaunchKernelGGL(k_synth_column, dim3((unsigned)((nwords + 255) / 256)), dim3(256), 0, stream, seed, card, bits,
                     num_docs, nwords, out);
}

void launch_sorted_to_fwd(const int32_t *starts, int32_t card, int32_t bits, int32_t num_docs, uint8_t *out,
                          hipStream_t stream) {
  int64_t nwords = (num_docs + 63) / 64;
  if (nwords <= 0) return;
  hipLaunchKernelGGL(k_sorted_to_fwd, dim3((unsigned)((nwords + 255) / 256)), dim3(256), 0, stream, starts, card,
                     bits, num_docs, nwords, out);
}

}  // namespace pinot
