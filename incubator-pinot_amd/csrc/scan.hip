// K1 + K5: streaming filter-leaf and aggregation kernels over packed forward indexes.
//
// One lane owns one 64-doc word w: it loads the word's packed super-word (the 8*B bytes at offset
// 8*B*w, B = bits per value) with 16-B (even B) / 8-B loads, byte-swaps it once and extracts the 64
// dictIds with compile-time shifts. Each kernel is instantiated per bit width (1..32) so every
// instance is small, register-light and runs at full occupancy; the host picks the instance.
//
//   k_leaf<B, KIND>   predicate on dictIds (RANGE [lo,hi) / 64-entry LUT / LUT in memory), result
//                     written to or AND-ed / OR-ed into a doc bitset (filter trees = launch sequences)
//   k_colagg<B, OPS>  for the docs of a bitset: COUNT, Σ dictId (SUM/AVG over an arithmetic-progression
//                     dictionary), min/max dictId (MIN/MAX: dictionaries are sorted)
//   k_gather_agg      for the docs of a bitset: dictionary / HLL-LUT gathers (other SUM/AVG, HLL)
//   k_reduce_slots    deterministic fixed-order reduction of per-block partial slots
//
// Restates: PinotDataBitSet.readInt (PC/io/util/PinotDataBitSet.java:79-100), ScanBasedFilterOperator /
// SVScanDocIdIterator (PC/operator/dociditerators/SVScanDocIdIterator.java:85-159), AND/OR doc-id sets
// (PC/operator/docidsets/AndBlockDocIdSet.java:144-227, OrBlockDocIdSet.java:78-120), AggregationOperator and
// the Count/Sum/Min/Max/Avg/DistinctCountHLL aggregate() loops (PC/operator/query/AggregationOperator.java:56-82).
#include <hip/hip_runtime.h>
#include <type_traits>

#include "device.h"
#include "kernels.h"

namespace pinot {
namespace {
using namespace dev;

// The packed columns are streamed once per query: non-temporal loads.
template <int B>
__device__ __forceinline__ void load_superword(const uint8_t *__restrict__ fwd, int64_t w, uint32_t (&D)[2 * B]) {
  const uint8_t *p = fwd + (size_t)w * (size_t)(8 * B);
  if constexpr (B % 2 == 0) {
    const u32x4 *q = reinterpret_cast<const u32x4 *>(p);
#pragma unroll
    for (int i = 0; i < B / 2; i++) {
      const u32x4 v = __builtin_nontemporal_load(q + i);
      D[4 * i + 0] = bswap32(v.x);
      D[4 * i + 1] = bswap32(v.y);
      D[4 * i + 2] = bswap32(v.z);
      D[4 * i + 3] = bswap32(v.w);
    }
  } else {
    const u32x2 *q = reinterpret_cast<const u32x2 *>(p);
#pragma unroll
    for (int i = 0; i < B; i++) {
      const u32x2 v = __builtin_nontemporal_load(q + i);
      D[2 * i + 0] = bswap32(v.x);
      D[2 * i + 1] = bswap32(v.y);
    }
  }
}

// ---------------------------------------------------------------- LDS-staged super-words
// A wave handles a chunk of 64 consecutive words (4096 docs): the chunk's 512*B contiguous bytes are
// DMA'd into the wave's LDS region with coalesced 1-KiB global_load_lds_dwordx4 pieces, then every lane
// reads its own 8*B-byte super-word from LDS. (Loading the super-words straight from HBM with a lane
// stride of 8*B bytes touches 64 cache lines per instruction and thrashes the 32 KiB L1.)

template <int B>
struct Stage {
  static constexpr int kPieces = (B + 1) / 2;       // 1-KiB DMA pieces per chunk (odd B over-reads 512 B)
  static constexpr int kBytes = kPieces * 1024;     // LDS bytes per wave
};

template <int B>
__device__ __forceinline__ void stage_chunk(const uint8_t *__restrict__ fwd, int64_t chunk, uint8_t *lds_wave,
                                            int lane) {
  const uint8_t *src = fwd + (size_t)chunk * (size_t)(512 * B) + lane * 16;
#pragma unroll
  for (int i = 0; i < Stage<B>::kPieces; i++)
    __builtin_amdgcn_global_load_lds((glob_void_t *)(src + i * 1024), (lds_void_t *)(lds_wave + i * 1024), 16, 0, 0);
}


template <int B>
__device__ __forceinline__ void lds_superword(const uint8_t *lds_wave, int lane, uint32_t (&D)[2 * B]) {
  const uint8_t *p = lds_wave + lane * (8 * B);
  if constexpr (B % 2 == 0) {
#pragma unroll
    for (int i = 0; i < B / 2; i++) {
      const u32x4 v = *reinterpret_cast<const u32x4 *>(p + 16 * i);
      D[4 * i + 0] = bswap32(v.x);
      D[4 * i + 1] = bswap32(v.y);
      D[4 * i + 2] = bswap32(v.z);
      D[4 * i + 3] = bswap32(v.w);
    }
  } else {
#pragma unroll
    for (int i = 0; i < B; i++) {
      const u32x2 v = *reinterpret_cast<const u32x2 *>(p + 8 * i);
      D[2 * i + 0] = bswap32(v.x);
      D[2 * i + 1] = bswap32(v.y);
    }
  }
}

// dictId of doc J of the super-word: bits [J*B, J*B + B) of the big-endian stream
template <int B, int J>
__device__ __forceinline__ uint32_t extract(const uint32_t (&D)[2 * B]) {
  constexpr int p = J * B, k = p >> 5, o = p & 31;
  constexpr uint32_t mask = B == 32 ? 0xFFFFFFFFu : ((1u << B) - 1u);
  if constexpr (o + B <= 32) {
    return (D[k] >> (32 - o - B)) & mask;
  } else {
    return __builtin_amdgcn_alignbit(D[k], D[k + 1], 64 - o - B) & mask;
  }
}

template <int B, int J, typename F>
__device__ __forceinline__ void for_each_value(const uint32_t (&D)[2 * B], F &f) {
  f.template step<J>(extract<B, J>(D));
  if constexpr (J + 1 < 64) for_each_value<B, J + 1>(D, f);
}

template <int KIND>
struct LeafTest {
  uint32_t lo, span;
  uint64_t lut64;
  const uint32_t *__restrict__ lut;
  uint32_t m0 = 0, m1 = 0;
  template <int J>
  __device__ __forceinline__ void step(uint32_t v) {
    uint32_t bit;
    if constexpr (KIND == LEAF_RANGE) bit = (v - lo) < span ? 1u : 0u;
    else if constexpr (KIND == LEAF_LUT64) bit = (uint32_t)(lut64 >> v) & 1u;
    else bit = (lut[v >> 5] >> (v & 31)) & 1u;
    if constexpr (J < 32) m0 |= bit << J; else m1 |= bit << (J - 32);
  }
};

template <int OPS, typename SumT>
struct ColFold {
  uint32_t m0, m1;
  SumT s = 0;  // 64 values of B <= 26 bits fit a uint32_t sum
  uint32_t mn = 0xFFFFFFFFu, mx = 0;
  template <int J>
  __device__ __forceinline__ void step(uint32_t v) {
    const bool bit = ((J < 32 ? (m0 >> (J & 31)) : (m1 >> (J & 31))) & 1u) != 0;
    if constexpr (OPS & COLAGG_IDSUM) s += bit ? v : 0u;
    if constexpr (OPS & COLAGG_MINMAX) {
      mn = bit ? min(mn, v) : mn;
      mx = bit ? max(mx, v) : mx;
    }
  }
};

// Block-reduces one slot value (fixed order) and writes it to out[block] (lanes 0 of each wave -> LDS).
template <int NW>
__device__ __forceinline__ void block_store(int kind, unsigned long long v, unsigned long long (&red)[NW],
                                            unsigned long long *out) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = combine(kind, v, shfl_xor_u64(v, o));
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long r = red[0];
    for (int i = 1; i < NW; i++) r = combine(kind, r, red[i]);
    out[blockIdx.x] = r;
  }
}

template <int B, int KIND>
__global__ __launch_bounds__(kBlock) void k_leaf(LeafArgs a) {
  constexpr int kWaves = kBlock / 64;
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWaves][Stage<B>::kBytes];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t nchunks = (a.nwords + 63) / 64;
  for (int64_t ch = (int64_t)blockIdx.x * kWaves + wave; ch < nchunks; ch += (int64_t)gridDim.x * kWaves) {
    stage_chunk<B>(a.fwd, ch, lds[wave], lane);
    const int64_t w = ch * 64 + lane;
    uint64_t prev = 0;
    if (a.mode != CM_WRITE && w < a.nwords) prev = a.dst[w];
    wait_stage();
    uint32_t D[2 * B];
    lds_superword<B>(lds[wave], lane, D);
    LeafTest<KIND> f{a.lo, a.span, a.lut64, a.lut};
    for_each_value<B, 0>(D, f);
    uint64_t m = ((uint64_t)f.m1 << 32) | f.m0;
    if (a.negate) m = ~m;
    if (w < a.nwords) {
      m &= tail_mask(w, a.nwords, a.num_docs);
      if (a.mode == CM_AND) m &= prev;
      else if (a.mode == CM_OR) m |= prev;
      a.dst[w] = m;
    }
  }
}

template <int B, int OPS>
__global__ __launch_bounds__(kBlock) void k_colagg(ColAggArgs a) {
  constexpr int kWaves = kBlock / 64;
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWaves][Stage<B>::kBytes];
  __shared__ unsigned long long red[kBlock / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  unsigned long long cnt = 0, s = 0;
  uint32_t mn = 0xFFFFFFFFu, mx = 0;
  const int64_t nchunks = (a.nwords + 63) / 64;
  for (int64_t ch = (int64_t)blockIdx.x * kWaves + wave; ch < nchunks; ch += (int64_t)gridDim.x * kWaves) {
    stage_chunk<B>(a.fwd, ch, lds[wave], lane);
    const int64_t w = ch * 64 + lane;
    uint64_t m = 0;
    if (w < a.nwords) m = (a.bitset ? a.bitset[w] : ~0ull) & tail_mask(w, a.nwords, a.num_docs);
    cnt += __popcll(m);
    wait_stage();
    uint32_t D[2 * B];
    lds_superword<B>(lds[wave], lane, D);
    using SumT = typename std::conditional<(B <= 26), uint32_t, unsigned long long>::type;
    ColFold<OPS, SumT> f{(uint32_t)m, (uint32_t)(m >> 32)};
    for_each_value<B, 0>(D, f);
    s += f.s;
    mn = min(mn, f.mn);
    mx = max(mx, f.mx);
  }
  block_store(SLOT_SUM_U64, cnt, red, a.out_count);
  if (OPS & COLAGG_IDSUM) block_store(SLOT_SUM_U64, s, red, a.out_idsum);
  if (OPS & COLAGG_MINMAX) block_store(SLOT_MINMAX, ((unsigned long long)mx << 32) | mn, red, a.out_minmax);
}

// runtime-width decode of one doc (gather paths: only docs whose filter bit is set)
__device__ __forceinline__ uint32_t decode_doc(const uint8_t *fwd, int bits, int64_t doc) {
  const uint64_t bitpos = (uint64_t)doc * (uint32_t)bits;
  const uint32_t *p = reinterpret_cast<const uint32_t *>(fwd) + (bitpos >> 5);
  const uint64_t x = ((uint64_t)bswap32(p[0]) << 32) | bswap32(p[1]);
  return (uint32_t)((x << (bitpos & 31)) >> (64 - bits));
}

__global__ __launch_bounds__(kBlock) void k_gather_agg(GatherArgs a) {
  __shared__ uint32_t hll[kMaxHll][256];
  __shared__ unsigned long long acc[kMaxAggs][kBlock];
  __shared__ unsigned long long red[kBlock / 64];
  const int tid = threadIdx.x;
  for (int i = tid; i < kMaxHll * 256; i += kBlock) (&hll[0][0])[i] = 0;
  for (int g = 0; g < a.n; g++) acc[g][tid] = 0;
  __syncthreads();
  unsigned long long cnt = 0;
  for (int64_t w = (int64_t)blockIdx.x * kBlock + tid; w < a.nwords; w += (int64_t)gridDim.x * kBlock) {
    uint64_t m0 = a.bitset ? a.bitset[w] : ~0ull;
    m0 &= tail_mask(w, a.nwords, a.num_docs);
    cnt += __popcll(m0);
    for (int g = 0; g < a.n; g++) {
      const GatherSpec &s = a.specs[g];
      uint64_t mm = m0;
      if (s.kind == GA_SUM_I32) {
        long long t = 0;
        while (mm) {
          const int j = __builtin_ctzll(mm);
          mm &= mm - 1;
          t += static_cast<const int32_t *>(s.table)[decode_doc(s.fwd, s.bits, w * 64 + j)];
        }
        acc[g][tid] += (unsigned long long)t;
      } else if (s.kind == GA_SUM_I64 || s.kind == GA_SUM_F64) {
        double t = 0.0;
        while (mm) {
          const int j = __builtin_ctzll(mm);
          mm &= mm - 1;
          const uint32_t v = decode_doc(s.fwd, s.bits, w * 64 + j);
          t += s.kind == GA_SUM_I64 ? (double)static_cast<const long long *>(s.table)[v]
                                    : static_cast<const double *>(s.table)[v];
        }
        acc[g][tid] = (unsigned long long)__double_as_longlong(
            __longlong_as_double((long long)acc[g][tid]) + t);
      } else {  // GA_HLL
        while (mm) {
          const int j = __builtin_ctzll(mm);
          mm &= mm - 1;
          const uint32_t e = static_cast<const uint16_t *>(s.table)[decode_doc(s.fwd, s.bits, w * 64 + j)];
          atomicMax(&hll[s.hll_slot][e >> 8], e & 0xFFu);
        }
      }
    }
  }
  block_store(SLOT_SUM_U64, cnt, red, a.out_count);
  for (int g = 0; g < a.n; g++) {
    const GatherSpec &s = a.specs[g];
    if (s.kind == GA_HLL) continue;
    block_store(s.kind == GA_SUM_I32 ? SLOT_SUM_U64 : SLOT_SUM_F64, acc[g][tid], red, s.out);
  }
  __syncthreads();
  for (int g = 0; g < a.n; g++) {
    const GatherSpec &s = a.specs[g];
    if (s.kind != GA_HLL) continue;
    for (int i = tid; i < 256; i += kBlock) {
      const uint32_t r = hll[s.hll_slot][i];
      if (r) atomicMax(&s.hll_out[i], r);
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_popcount(const uint64_t *__restrict__ bitset, int64_t nwords,
                                                      int32_t num_docs, unsigned long long *out) {
  __shared__ unsigned long long red[kBlock / 64];
  unsigned long long cnt = 0;
  for (int64_t w = (int64_t)blockIdx.x * kBlock + threadIdx.x; w < nwords; w += (int64_t)gridDim.x * kBlock)
    cnt += __popcll(bitset[w] & tail_mask(w, nwords, num_docs));
  block_store(SLOT_SUM_U64, cnt, red, out);
}

// One block per slot: fixed-order reduction of `grid` partials (slot s at in + s * stride) into out[s].
__global__ __launch_bounds__(kBlock) void k_reduce_slots(ReduceArgs a) {
  __shared__ unsigned long long sm[kBlock];
  const int slot = blockIdx.x, tid = threadIdx.x;
  const int kind = a.kinds[slot];
  const unsigned long long *in = a.in + (int64_t)slot * a.stride;
  unsigned long long v = slot_init(kind);
  for (int i = tid; i < a.grid; i += kBlock) v = combine(kind, v, in[i]);
  sm[tid] = v;
  __syncthreads();
  for (int st = kBlock / 2; st > 0; st >>= 1) {
    if (tid < st) sm[tid] = combine(kind, sm[tid], sm[tid + st]);
    __syncthreads();
  }
  if (tid == 0) a.out[a.out_index[slot]] = sm[0];
}

typedef void (*LeafKernel)(LeafArgs);
typedef void (*ColAggKernel)(ColAggArgs);

template <int B>
struct Tables {
  static constexpr LeafKernel leaf[3] = {k_leaf<B, LEAF_RANGE>, k_leaf<B, LEAF_LUT64>, k_leaf<B, LEAF_LUT>};
  static constexpr ColAggKernel colagg[3] = {k_colagg<B, 1>, k_colagg<B, 2>, k_colagg<B, 3>};
};

template <int... Bs>
struct AllTables {
  static constexpr LeafKernel leaf[32][3] = {{Tables<Bs>::leaf[0], Tables<Bs>::leaf[1], Tables<Bs>::leaf[2]}...};
  static constexpr ColAggKernel colagg[32][3] = {
      {Tables<Bs>::colagg[0], Tables<Bs>::colagg[1], Tables<Bs>::colagg[2]}...};
};
using KT = AllTables<1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26,
                     27, 28, 29, 30, 31, 32>;

}  // namespace

int scan_grid(int64_t nwords) {
  int64_t g = (nwords + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  if (g > kMaxScanGrid) g = kMaxScanGrid;
  return (int)g;
}

void launch_leaf(int bits, int kind, const LeafArgs &a, hipStream_t stream) {
  if (a.nwords <= 0) return;
  hipLaunchKernelGGL(KT::leaf[bits - 1][kind], dim3(scan_grid(a.nwords)), dim3(kBlock), 0, stream, a);
}

void launch_colagg(int bits, int ops, const ColAggArgs &a, hipStream_t stream) {
  hipLaunchKernelGGL(KT::colagg[bits - 1][ops - 1], dim3(scan_grid(a.nwords)), dim3(kBlock), 0, stream, a);
}

void launch_gather_agg(const GatherArgs &a, hipStream_t stream) {
  hipLaunchKernelGGL(k_gather_agg, dim3(scan_grid(a.nwords)), dim3(kBlock), 0, stream, a);
}

void launch_popcount(const uint64_t *bitset, int64_t nwords, int32_t num_docs, unsigned long long *out,
                     hipStream_t stream) {
  hipLaunchKernelGGL(k_popcount, dim3(scan_grid(nwords)), dim3(kBlock), 0, stream, bitset, nwords, num_docs, out);
}

void launch_reduce_slots(const ReduceArgs &a, int nslots, hipStream_t stream) {
  if (nslots <= 0) return;
  hipLaunchKernelGGL(k_reduce_slots, dim3(nslots), dim3(kBlock), 0, stream, a);
}

}  // namespace pinot
