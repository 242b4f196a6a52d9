// HIP/CDNA4 (gfx950) kernels of the Pinot segment executor.
//
// K1 filter_scan      PinotDataBitSet.readInt + ScanBasedFilterOperator/SVScanDocIdIterator + AND/OR
//                     (PC/io/util/PinotDataBitSet.java:79-100, PC/operator/dociditerators/SVScanDocIdIterator.java:85-159,
//                      PC/operator/docidsets/AndBlockDocIdSet.java:144-227, OrBlockDocIdSet.java:78-120)
// K2 ranges_to_bitset SortedInvertedIndexBasedFilterOperator (PC/operator/filter/SortedInvertedIndexBasedFilterOperator.java:59-158)
// K3 roaring_expand   BitmapBasedFilterOperator + BitmapDocIdSet (PC/operator/filter/BitmapBasedFilterOperator.java:69-84,
//                      PC/operator/docidsets/BitmapDocIdSet.java:33-58)
// K5 aggregate        AggregationOperator / DefaultAggregationExecutor (PC/operator/query/AggregationOperator.java:56-82)
// K6 group_by         DictionaryBasedGroupKeyGenerator + DefaultGroupByExecutor
//                      (PC/query/aggregation/groupby/DictionaryBasedGroupKeyGenerator.java:195-302)
// K7 HLL update       DistinctCountHLLAggregationFunction (register/rank precomputed per dictId on the host)
//
// Wave64 everywhere: a 64-doc filter word is one u64, produced either by one lane decoding a
// 64-doc super-word (K1) or by one wave with one doc per lane (K5/K6).
#include "kernels.h"

#include <hip/hip_runtime.h>

namespace pinot {

namespace {

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ uint64_t tail_mask(int64_t w, int64_t nwords, int32_t num_docs) {
  if (w != nwords - 1) return ~0ull;
  int rem = num_docs - (int)(w * 64);
  return rem >= 64 ? ~0ull : ((1ull << rem) - 1ull);
}

// ------------------------------------------------------------------ K1: templated super-word decode
// The 64 docs of word w are the 8*B bytes at offset 8*B*w: 2*B big-endian dwords.
template <int B>
__device__ __forceinline__ void load_superword(const uint8_t *__restrict__ fwd, int64_t w, uint32_t (&D)[2 * B]) {
  const uint8_t *p = fwd + (size_t)w * (size_t)(8 * B);
  if constexpr (B % 2 == 0) {
    const uint4 *q = reinterpret_cast<const uint4 *>(p);
#pragma unroll
    for (int i = 0; i < B / 2; i++) {
      uint4 v = q[i];
      D[4 * i + 0] = bswap32(v.x);
      D[4 * i + 1] = bswap32(v.y);
      D[4 * i + 2] = bswap32(v.z);
      D[4 * i + 3] = bswap32(v.w);
    }
  } else {
    const uint2 *q = reinterpret_cast<const uint2 *>(p);
#pragma unroll
    for (int i = 0; i < B; i++) {
      uint2 v = q[i];
      D[2 * i + 0] = bswap32(v.x);
      D[2 * i + 1] = bswap32(v.y);
    }
  }
}

template <int B, int J>
__device__ __forceinline__ uint32_t extract(const uint32_t (&D)[2 * B]) {
  constexpr int p = J * B;
  constexpr int k = p >> 5;
  constexpr int o = p & 31;
  constexpr uint32_t mask = B == 32 ? 0xFFFFFFFFu : ((1u << B) - 1u);
  if constexpr (o + B <= 32) {
    return (D[k] >> (32 - o - B)) & mask;
  } else {
    return __builtin_amdgcn_alignbit(D[k], D[k + 1], 64 - o - B) & mask;
  }
}

template <int B, int J>
struct RangeBits {
  __device__ __forceinline__ static void run(const uint32_t (&D)[2 * B], uint32_t lo, uint32_t span, uint32_t &m0,
                                             uint32_t &m1) {
    uint32_t v = extract<B, J>(D);
    uint32_t bit = (v - lo) < span ? 1u : 0u;
    if constexpr (J < 32) m0 |= bit << J; else m1 |= bit << (J - 32);
    if constexpr (J + 1 < 64) RangeBits<B, J + 1>::run(D, lo, span, m0, m1);
  }
};

template <int B, int J>
struct LutBits {
  __device__ __forceinline__ static void run(const uint32_t (&D)[2 * B], const uint32_t *__restrict__ lut,
                                             uint32_t &m0, uint32_t &m1) {
    uint32_t v = extract<B, J>(D);
    uint32_t bit = (lut[v >> 5] >> (v & 31)) & 1u;
    if constexpr (J < 32) m0 |= bit << J; else m1 |= bit << (J - 32);
    if constexpr (J + 1 < 64) LutBits<B, J + 1>::run(D, lut, m0, m1);
  }
};

template <int B, int J>
struct Lut64Bits {
  __device__ __forceinline__ static void run(const uint32_t (&D)[2 * B], uint64_t lut, uint32_t &m0, uint32_t &m1) {
    uint32_t v = extract<B, J>(D);
    uint32_t bit = (uint32_t)(lut >> v) & 1u;
    if constexpr (J < 32) m0 |= bit << J; else m1 |= bit << (J - 32);
    if constexpr (J + 1 < 64) Lut64Bits<B, J + 1>::run(D, lut, m0, m1);
  }
};

template <int B>
__device__ __noinline__ uint64_t scan_leaf(const FilterInstr &in, const DevColumn &c, int64_t w,
                                           const uint32_t *__restrict__ luts) {
  uint32_t D[2 * B];
  load_superword<B>(c.fwd, w, D);
  uint32_t m0 = 0, m1 = 0;
  if (in.op == OP_LEAF_RANGE) {
    RangeBits<B, 0>::run(D, (uint32_t)in.a, (uint32_t)(in.b - in.a), m0, m1);
  } else if (c.card <= 64) {
    const uint32_t *l = luts + in.a;
    uint64_t lut = (uint64_t)l[0] | ((uint64_t)(c.card > 32 ? l[1] : 0u) << 32);
    Lut64Bits<B, 0>::run(D, lut, m0, m1);
  } else {
    LutBits<B, 0>::run(D, luts + in.a, m0, m1);
  }
  uint64_t m = ((uint64_t)m1 << 32) | m0;
  return (in.flags & 1) ? ~m : m;
}

__device__ uint64_t eval_scan_leaf(const FilterInstr &in, const DevColumn &c, int64_t w,
                                   const uint32_t *__restrict__ luts) {
  switch (c.bits) {
#define PINOT_CASE(B) \
  case B:             \
    return scan_leaf<B>(in, c, w, luts);
    PINOT_CASE(1) PINOT_CASE(2) PINOT_CASE(3) PINOT_CASE(4) PINOT_CASE(5) PINOT_CASE(6) PINOT_CASE(7) PINOT_CASE(8)
    PINOT_CASE(9) PINOT_CASE(10) PINOT_CASE(11) PINOT_CASE(12) PINOT_CASE(13) PINOT_CASE(14) PINOT_CASE(15)
    PINOT_CASE(16) PINOT_CASE(17) PINOT_CASE(18) PINOT_CASE(19) PINOT_CASE(20) PINOT_CASE(21) PINOT_CASE(22)
    PINOT_CASE(23) PINOT_CASE(24) PINOT_CASE(25) PINOT_CASE(26) PINOT_CASE(27) PINOT_CASE(28) PINOT_CASE(29)
    PINOT_CASE(30) PINOT_CASE(31) PINOT_CASE(32)
#undef PINOT_CASE
    default:
      return 0;
  }
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(kBlock) void k_filter_scan(FilterProgram prog, int64_t nwords, int32_t num_docs,
                                                         uint64_t *__restrict__ out, unsigned long long *count) {
  __shared__ uint64_t stk[kMaxStack][kBlock];
  __shared__ unsigned long long wsum[kBlock / 64];
  const int tid = threadIdx.x;
  unsigned long long cnt = 0;
  for (int64_t w = (int64_t)blockIdx.x * kBlock + tid; w < nwords; w += (int64_t)gridDim.x * kBlock) {
    int sp = 0;
    for (int i = 0; i < prog.n_instr; i++) {
      const FilterInstr &in = prog.ins[i];
      uint64_t r;
      switch (in.op) {
        case OP_LEAF_RANGE:
        case OP_LEAF_LUT:
          r = eval_scan_leaf(in, prog.cols[in.col], w, prog.luts);
          break;
        case OP_LEAF_BITSET:
          r = prog.bitsets[(int64_t)in.a * prog.bitset_stride + w];
          break;
        case OP_AND: {
          r = ~0ull;
          for (int k = 0; k < in.a; k++) r &= stk[--sp][tid];
          break;
        }
        case OP_OR: {
          r = 0;
          for (int k = 0; k < in.a; k++) r |= stk[--sp][tid];
          break;
        }
        case OP_ALL:
          r = ~0ull;
          break;
        default:
          r = 0;
          break;
      }
      stk[sp++][tid] = r;
    }
    uint64_t m = (sp > 0 ? stk[sp - 1][tid] : ~0ull) & tail_mask(w, nwords, num_docs);
    if (out) out[w] = m;
    cnt += __popcll(m);
  }
  cnt = wave_sum_u64(cnt);
  if ((tid & 63) == 0) wsum[tid >> 6] = cnt;
  __syncthreads();
  if (tid == 0) {
    unsigned long long t = 0;
    for (int i = 0; i < kBlock / 64; i++) t += wsum[i];
    if (t) atomicAdd(count, t);
  }
}

// ------------------------------------------------------------------ K2: sorted ranges
__global__ void k_ranges_to_bitset(const int32_t *__restrict__ ranges, int32_t n, int64_t nwords, int32_t num_docs,
                                   uint64_t *__restrict__ out) {
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
  out[w] = word & tail_mask(w, nwords, num_docs);
}

// ------------------------------------------------------------------ K3: roaring containers -> dense tile
__device__ __forceinline__ uint32_t ld_u16(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }

__global__ __launch_bounds__(kBlock) void k_roaring_expand(const uint8_t *__restrict__ payload,
                                                            const RoaringContainer *__restrict__ containers,
                                                            const int32_t *__restrict__ dir,
                                                            const int32_t *__restrict__ ids, int32_t nids,
                                                            int exclusive, int64_t nwords, int32_t num_docs,
                                                            uint64_t *__restrict__ out) {
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
    out[w] = v & tail_mask(w, nwords, num_docs);
  }
}

// ------------------------------------------------------------------ K5/K6: runtime-width single-doc decode
__device__ __forceinline__ uint32_t decode_doc(const DevColumn &c, int64_t doc) {
  const uint64_t bitpos = (uint64_t)doc * (uint32_t)c.bits;
  const uint32_t *p = reinterpret_cast<const uint32_t *>(c.fwd) + (bitpos >> 5);
  const uint64_t x = ((uint64_t)bswap32(p[0]) << 32) | bswap32(p[1]);
  return (uint32_t)((x << (bitpos & 31)) >> (64 - c.bits));
}

__device__ __forceinline__ double shfl_xor_d(double v, int o) {
  long long b = __double_as_longlong(v);
  b = __shfl_xor(b, o, 64);
  return __longlong_as_double(b);
}

__global__ __launch_bounds__(kBlock) void k_aggregate(AggProgram prog, const uint64_t *__restrict__ bitset,
                                                       int64_t nwords, int32_t num_docs,
                                                       AggPartial *__restrict__ partials,
                                                       uint32_t *__restrict__ hll_regs) {
  __shared__ uint32_t hll[4][256];
  __shared__ long long red_i[kBlock / 64];
  __shared__ double red_f[kBlock / 64];
  __shared__ int red_mn[kBlock / 64], red_mx[kBlock / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < 4 * 256; i += kBlock) (&hll[0][0])[i] = 0;
  __syncthreads();

  // per-lane accumulators, one 64-bit slot per aggregation (registers: every index is compile-time)
  long long acc_i[kMaxAggs];
  double acc_f[kMaxAggs];
  int mn[kMaxAggs], mx[kMaxAggs];
#pragma unroll
  for (int a = 0; a < kMaxAggs; a++) { acc_i[a] = 0; acc_f[a] = 0.0; mn[a] = 0x7FFFFFFF; mx[a] = -1; }

  const int64_t waves = (int64_t)gridDim.x * (kBlock / 64);
  for (int64_t w = (int64_t)blockIdx.x * (kBlock / 64) + wave; w < nwords; w += waves) {
    uint64_t m = bitset ? bitset[w] : ~0ull;
    m &= tail_mask(w, nwords, num_docs);
    if (m == 0) continue;
    if (!((m >> lane) & 1ull)) continue;
    const int64_t doc = w * 64 + lane;
    int hslot = 0;
#pragma unroll
    for (int a = 0; a < kMaxAggs; a++) {
      if (a >= prog.n_aggs) break;
      const AggSpecDev &s = prog.aggs[a];
      if (s.kind == AGG_NOP) continue;
      const uint32_t v = decode_doc(prog.cols[s.col], doc);
      switch (s.kind) {
        case AGG_SUM_I32: acc_i[a] += (long long)static_cast<const int32_t *>(s.dict)[v]; break;
        case AGG_SUM_I64: acc_f[a] += (double)static_cast<const long long *>(s.dict)[v]; break;
        case AGG_SUM_F64: acc_f[a] += static_cast<const double *>(s.dict)[v]; break;
        case AGG_MINMAX:
          mn[a] = min(mn[a], (int)v);
          mx[a] = max(mx[a], (int)v);
          break;
        case AGG_HLL: {
          const uint32_t e = s.hll_lut[v];
          atomicMax(&hll[hslot & 3][e >> 8], e & 0xFF);
          break;
        }
        default: break;
      }
      if (s.kind == AGG_HLL) hslot++;
    }
  }

  // block reduction per aggregation
  int hslot = 0;
#pragma unroll
  for (int a = 0; a < kMaxAggs; a++) {
    if (a >= prog.n_aggs) break;
    long long si = acc_i[a];
    double sf = acc_f[a];
    int lmn = mn[a], lmx = mx[a];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      si += __shfl_xor(si, o, 64);
      sf += shfl_xor_d(sf, o);
      lmn = min(lmn, __shfl_xor(lmn, o, 64));
      lmx = max(lmx, __shfl_xor(lmx, o, 64));
    }
    if (lane == 0) { red_i[wave] = si; red_f[wave] = sf; red_mn[wave] = lmn; red_mx[wave] = lmx; }
    __syncthreads();
    if (tid == 0) {
      AggPartial p;
      p.sum_i64 = 0; p.sum_f64 = 0.0; p.min_id = 0x7FFFFFFF; p.max_id = -1;
      for (int i = 0; i < kBlock / 64; i++) {
        p.sum_i64 += red_i[i];
        p.sum_f64 += red_f[i];
        p.min_id = min(p.min_id, red_mn[i]);
        p.max_id = max(p.max_id, red_mx[i]);
      }
      partials[(int64_t)a * gridDim.x + blockIdx.x] = p;
    }
    __syncthreads();
    if (prog.aggs[a].kind == AGG_HLL) {
      for (int i = tid; i < 256; i += kBlock) {
        uint32_t r = hll[hslot & 3][i];
        if (r) atomicMax(&hll_regs[a * 256 + i], r);
      }
      hslot++;
    }
  }
}

// ------------------------------------------------------------------ K6: group-by
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

// Deterministic reduction of per-workgroup partials: one block per aggregation, fixed order.
__global__ __launch_bounds__(kBlock) void k_reduce_partials(const AggPartial *__restrict__ in, int grid,
                                                             AggPartial *__restrict__ out) {
  __shared__ long long si[kBlock];
  __shared__ double sf[kBlock];
  __shared__ int smn[kBlock], smx[kBlock];
  const int a = blockIdx.x, tid = threadIdx.x;
  long long i64 = 0;
  double f64 = 0.0;
  int mn = 0x7FFFFFFF, mx = -1;
  for (int i = tid; i < grid; i += kBlock) {
    const AggPartial p = in[(int64_t)a * grid + i];
    i64 += p.sum_i64;
    f64 += p.sum_f64;
    mn = min(mn, p.min_id);
    mx = max(mx, p.max_id);
  }
  si[tid] = i64; sf[tid] = f64; smn[tid] = mn; smx[tid] = mx;
  __syncthreads();
  for (int s = kBlock / 2; s > 0; s >>= 1) {
    if (tid < s) {
      si[tid] += si[tid + s];
      sf[tid] += sf[tid + s];
      smn[tid] = min(smn[tid], smn[tid + s]);
      smx[tid] = max(smx[tid], smx[tid + s]);
    }
    __syncthreads();
  }
  if (tid == 0) out[a] = AggPartial{si[0], sf[0], smn[0], smx[0]};
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

void launch_filter_scan(const FilterProgram &prog, int64_t nwords, int32_t num_docs, uint64_t *out_bitset,
                        unsigned long long *count, hipStream_t stream) {
  if (nwords <= 0) return;
  int grid = grid_for(nwords, kBlock, 4096);
  hipLaunchKernelGGL(k_filter_scan, dim3(grid), dim3(kBlock), 0, stream, prog, nwords, num_docs, out_bitset, count);
}

void launch_ranges_to_bitset(const int32_t *ranges, int32_t nranges, int64_t nwords, int32_t num_docs,
                             uint64_t *out, hipStream_t stream) {
  if (nwords <= 0) return;
  hipLaunchKernelGGL(k_ranges_to_bitset, dim3((unsigned)((nwords + 255) / 256)), dim3(256), 0, stream, ranges,
                     nranges, nwords, num_docs, out);
}

void launch_roaring_expand(const uint8_t *payload, const RoaringContainer *containers, const int32_t *dir,
                           const int32_t *ids, int32_t nids, int exclusive, int64_t nwords, int32_t num_docs,
                           uint64_t *out, hipStream_t stream) {
  if (nwords <= 0) return;
  unsigned tiles = (unsigned)((nwords + 1023) / 1024);
  hipLaunchKernelGGL(k_roaring_expand, dim3(tiles), dim3(kBlock), 0, stream, payload, containers, dir, ids, nids,
                     exclusive, nwords, num_docs, out);
}

int aggregate_grid(int64_t nwords) { return grid_for(nwords, 4 * 16, 2048); }

int launch_aggregate(const AggProgram &prog, const uint64_t *bitset, int64_t nwords, int32_t num_docs,
                     AggPartial *partials, uint32_t *hll_regs, hipStream_t stream) {
  int grid = aggregate_grid(nwords);
  if (nwords <= 0) return grid;
  hipLaunchKernelGGL(k_aggregate, dim3(grid), dim3(kBlock), 0, stream, prog, bitset, nwords, num_docs, partials,
                     hll_regs);
  return grid;
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

void launch_reduce_partials(const AggPartial *in, int grid, int n_aggs, AggPartial *out, hipStream_t stream) {
  if (n_aggs <= 0) return;
  hipLaunchKernelGGL(k_reduce_partials, dim3(n_aggs), dim3(kBlock), 0, stream, in, grid, out);
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
