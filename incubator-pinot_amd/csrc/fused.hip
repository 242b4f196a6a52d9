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
// Block partials go to HBM per segment; k_reduce_fused reduces them in a fixed order.
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
// Half h of the lane's super-word is the B dwords at byte 8*B*lane + 4*B*h; the 32-way switch over B
// selects an unrolled decoder whose shifts are constants, the evaluation after it is width-free.
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

__device__ __forceinline__ void decode_half_rt(int bits, const uint8_t *p, uint32_t (&v)[32]) {
  switch (bits) {
#define PINOT_DECODE_CASE(B) \
  case B:                    \
    decode_half<B>(p, v);    \
    break;
    PINOT_DECODE_CASE(1) PINOT_DECODE_CASE(2) PINOT_DECODE_CASE(3) PINOT_DECODE_CASE(4) PINOT_DECODE_CASE(5)
    PINOT_DECODE_CASE(6) PINOT_DECODE_CASE(7) PINOT_DECODE_CASE(8) PINOT_DECODE_CASE(9) PINOT_DECODE_CASE(10)
    PINOT_DECODE_CASE(11) PINOT_DECODE_CASE(12) PINOT_DECODE_CASE(13) PINOT_DECODE_CASE(14) PINOT_DECODE_CASE(15)
    PINOT_DECODE_CASE(16) PINOT_DECODE_CASE(17) PINOT_DECODE_CASE(18) PINOT_DECODE_CASE(19) PINOT_DECODE_CASE(20)
    PINOT_DECODE_CASE(21) PINOT_DECODE_CASE(22) PINOT_DECODE_CASE(23) PINOT_DECODE_CASE(24) PINOT_DECODE_CASE(25)
    PINOT_DECODE_CASE(26) PINOT_DECODE_CASE(27) PINOT_DECODE_CASE(28) PINOT_DECODE_CASE(29) PINOT_DECODE_CASE(30)
    PINOT_DECODE_CASE(31) PINOT_DECODE_CASE(32)
#undef PINOT_DECODE_CASE
    default:
      break;
  }
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

template <bool G>
__device__ __forceinline__ uint32_t leaf_half(const FusedStep &st, const uint32_t (&v)[32]) {
  uint32_t m = 0;
  if (st.kind == FK_LEAF_RANGE) {
#pragma unroll
    for (int j = 0; j < 32; j++) m |= ((v[j] - st.lo) < st.span ? 1u : 0u) << j;
  } else if (!G || st.kind == FK_LEAF_LUT64) {
#pragma unroll
    for (int j = 0; j < 32; j++) m |= (uint32_t)((st.lut64 >> v[j]) & 1ull) << j;
  } else {
    const uint32_t *__restrict__ lut = static_cast<const uint32_t *>(st.table);
#pragma unroll
    for (int j = 0; j < 32; j++) m |= ((lut[v[j] >> 5] >> (v[j] & 31)) & 1u) << j;
  }
  return m;
}

constexpr int kFusedWaves = kBlock / 64;

struct FusedLds {
  unsigned long long sum[kMaxFusedFolds][64];  // per-lane Σ (dictId or dictionary value) of fold f
  uint32_t mn[kMaxFusedFolds][64], mx[kMaxFusedFolds][64];
  uint32_t hll[kMaxHll][256];
  unsigned long long red[kFusedWaves];
};

// Per-lane fold accumulators, held in registers for the whole kernel (the fold loop is unrolled over
// kMaxFusedFolds so fold f indexes them at compile time). LDS is touched only once, at the flush: an
// LDS atomic inside the chunk loop would make the compiler wait (vmcnt) for the in-flight LDS-DMA.
struct FoldAcc {
  unsigned long long sum[kMaxFusedFolds];
  uint32_t mn[kMaxFusedFolds], mx[kMaxFusedFolds];
};

template <bool G>
__device__ __forceinline__ void fold_half(const FusedStep &st, uint32_t mh, const uint32_t (&v)[32],
                                          unsigned long long &sum, uint32_t &mn, uint32_t &mx, FusedLds &L) {
  if (st.ops & FOLD_IDSUM) {
    if (st.bits <= 27) {  // 32 values of <= 27 bits cannot overflow 32 bits
      uint32_t t = 0;
#pragma unroll
      for (int j = 0; j < 32; j++) t += ((mh >> j) & 1u) ? v[j] : 0u;
      sum += t;
    } else {
#pragma unroll
      for (int j = 0; j < 32; j++) sum += ((mh >> j) & 1u) ? (unsigned long long)v[j] : 0ull;
    }
  }
  if (G && (st.ops & FOLD_DICT32)) {
    const int32_t *__restrict__ dict = static_cast<const int32_t *>(st.table);
    long long s = 0;
#pragma unroll
    for (int j = 0; j < 32; j++)
      if ((mh >> j) & 1u) s += dict[v[j]];
    sum += (unsigned long long)s;
  }
  if (st.ops & FOLD_MINMAX) {
#pragma unroll
    for (int j = 0; j < 32; j++) {
      const bool b = (mh >> j) & 1u;
      mn = b ? min(mn, v[j]) : mn;
      mx = b ? max(mx, v[j]) : mx;
    }
  }
  if (G && (st.ops & FOLD_HLL)) {
    uint32_t *regs = L.hll[st.hll_set];
#pragma unroll
    for (int j = 0; j < 32; j++)
      if ((mh >> j) & 1u) {
        const uint32_t e = st.hll_lut[v[j]];
        atomicMax(&regs[e >> 8], e & 0xFFu);
      }
  }
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

__device__ __forceinline__ void init_lds(FusedLds &L, int tid) {
  for (int i = tid; i < kMaxFusedFolds * 64; i += kBlock) {
    (&L.sum[0][0])[i] = 0;
    (&L.mn[0][0])[i] = 0xFFFFFFFFu;
    (&L.mx[0][0])[i] = 0;
  }
  for (int i = tid; i < kMaxHll * 256; i += kBlock) (&L.hll[0][0])[i] = 0;
  __syncthreads();
}

// block partials, fixed order: wave sums -> LDS -> thread 0; folds reduced by wave 0; HLL atomicMax
__device__ __forceinline__ void flush_block(const FusedArgs &a, FusedLds &L, const FoldAcc &A, unsigned long long cnt,
                                            int g, int b, int tid, int lane, int wave) {
#pragma unroll
  for (int f = 0; f < kMaxFusedFolds; f++) {
    if (A.sum[f]) atomicAdd(&L.sum[f][lane], A.sum[f]);
    atomicMin(&L.mn[f][lane], A.mn[f]);
    atomicMax(&L.mx[f][lane], A.mx[f]);
  }
  cnt = wave_sum(cnt);
  if (lane == 0) L.red[wave] = cnt;
  __syncthreads();
  const int64_t nblk = (int64_t)a.nsegs * a.bps;
  unsigned long long *out = a.part + (int64_t)g * a.bps + b;
  if (tid == 0) {
    unsigned long long c = 0;
    for (int i = 0; i < kFusedWaves; i++) c += L.red[i];
    out[0] = c;
  }
  const int nfolds = (a.nslots - 1) / 2;
  if (wave == 0) {
    for (int f = 0; f < nfolds; f++) {
      const unsigned long long s = wave_sum(L.sum[f][lane]);
      uint32_t lo = L.mn[f][lane], hi = L.mx[f][lane];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, (uint32_t)__shfl_xor((int)lo, o, 64));
        hi = max(hi, (uint32_t)__shfl_xor((int)hi, o, 64));
      }
      if (lane == 0) {
        out[(1 + 2 * f) * nblk] = s;
        out[(2 + 2 * f) * nblk] = ((unsigned long long)hi << 32) | lo;
      }
    }
  }
  for (int h = 0; h < a.n_hll; h++)
    for (int i = tid; i < 256; i += kBlock) {
      const uint32_t r = L.hll[h][i];
      if (r) atomicMax(&a.hll_out[h * 256 + i], r);
    }
}

// One chunk of the segment program: leaves AND-ed into `mask` (early exit once the wave's mask is
// empty), then the folds over the surviving docs. `src(i, st)` returns the LDS address of step i's
// staged chunk (staging it first in the stepwise kernel). Returns the chunk's matching doc count.
template <bool G, typename Src>
__device__ __forceinline__ unsigned long long eval_chunk(const FusedStep *__restrict__ steps, int n_leaves,
                                                         int n_folds, uint64_t mask, FoldAcc &A, FusedLds &L,
                                                         int lane, Src &&src) {
  for (int i = 0; i < n_leaves; i++) {
    if (!__any(mask != 0)) break;  // wave-uniform: nothing left in this chunk, skip its other columns
    const FusedStep st = load_const(steps + i);
    const uint8_t *p = src(i, st) + lane * (8 * st.bits);
    uint32_t v[32];
    decode_half_rt(st.bits, p, v);
    const uint32_t m0 = leaf_half<G>(st, v);
    decode_half_rt(st.bits, p + 4 * st.bits, v);
    const uint32_t m1 = leaf_half<G>(st, v);
    const uint64_t m = ((uint64_t)m1 << 32) | m0;
    mask &= st.negate ? ~m : m;
  }
  const unsigned long long cnt = __popcll(mask);
#pragma unroll
  for (int i = 0; i < kMaxFusedFolds; i++) {
    if (i >= n_folds || !__any(mask != 0)) break;
    const FusedStep st = load_const(steps + n_leaves + i);  // st.fold == i (host order)
    const uint8_t *p = src(n_leaves + i, st) + lane * (8 * st.bits);
    uint32_t v[32];
    decode_half_rt(st.bits, p, v);
    fold_half<G>(st, (uint32_t)mask, v, A.sum[i], A.mn[i], A.mx[i], L);
    decode_half_rt(st.bits, p + 4 * st.bits, v);
    fold_half<G>(st, (uint32_t)(mask >> 32), v, A.sum[i], A.mn[i], A.mx[i], L);
  }
  return cnt;
}

__device__ __forceinline__ uint64_t chunk_word(const FusedSegment &sg, int64_t ch, int lane) {
  const int64_t w = ch * 64 + lane;
  if (w >= sg.nwords) return 0;
  return (sg.pre ? sg.pre[w] : ~0ull) & tail_mask(w, sg.nwords, sg.num_docs);
}

// Stepwise shape: per chunk, each step's column is staged into the wave's single LDS stage and
// decoded before the next step is fetched (a step is fetched only while the chunk still has matches).
// G = false: streaming-only program (RANGE / 64-entry LUT leaves, Σ dictId and min/max folds), register-light;
// G = true: also memory-LUT leaves, dictionary-value sums and HLL (per-value gathers).
template <bool G>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3))) void k_scan_query(FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t stage_lds[];
  __shared__ FusedLds L;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  init_lds(L, tid);
  const int g = blockIdx.x / a.bps, b = blockIdx.x % a.bps;
  const FusedSegment sg = load_const(a.segs + g);
  const FusedStep *steps = a.steps + sg.first_step;
  uint8_t *lds_wave = stage_lds + wave * a.stage_bytes;
  unsigned long long cnt = 0;
  FoldAcc A;
  init_acc(A);
  const int64_t nchunks = (sg.nwords + 63) >> 6;
  for (int64_t ch = (int64_t)b * kFusedWaves + wave; ch < nchunks; ch += (int64_t)a.bps * kFusedWaves) {
    cnt += eval_chunk<G>(steps, sg.n_leaves, sg.n_folds, chunk_word(sg, ch, lane), A, L, lane,
                         [&](int, const FusedStep &st) -> const uint8_t * {
                           stage_chunk_rt(st.fwd, st.bits, ch, lds_wave, lane);
                           wait_stage();
                           return lds_wave;
                         });
  }
  flush_block(a, L, A, cnt, g, b, tid, lane, wave);
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
  __shared__ FusedLds L;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  init_lds(L, tid);
  const int g = blockIdx.x / a.bps, b = blockIdx.x % a.bps;
  const FusedSegment sg = load_const(a.segs + g);
  const FusedStep *steps = a.steps + sg.first_step;
  const int nsteps = sg.n_leaves + sg.n_folds;
  uint8_t *const slots = stage_lds + (size_t)wave * 2 * a.stage_bytes;
  const int64_t nchunks = (sg.nwords + 63) >> 6;
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
  int64_t ch = (int64_t)b * kFusedWaves + wave;
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
      cnt += eval_chunk<G>(steps, sg.n_leaves, sg.n_folds, m0, A, L, lane,
                           [&](int, const FusedStep &st) -> const uint8_t * { return cur + st.stage_off; });
    m0 = m1;
    live0 = live1;
    par ^= 1;
  }
  wait_stage();
  flush_block(a, L, A, cnt, g, b, tid, lane, wave);
}

// One block per (segment, slot): fixed-order reduction of the segment's bps block partials.
__global__ __launch_bounds__(kBlock) void k_reduce_fused(const unsigned long long *__restrict__ part, int32_t nsegs,
                                                          int32_t bps, int32_t nslots, unsigned long long *out,
                                                          int32_t out_stride) {
  __shared__ unsigned long long sm[kBlock];
  const int g = blockIdx.x / nslots, s = blockIdx.x % nslots, tid = threadIdx.x;
  const int kind = (s == 0 || (s & 1)) ? SLOT_SUM_U64 : SLOT_MINMAX;
  const unsigned long long *in = part + (int64_t)s * nsegs * bps + (int64_t)g * bps;
  unsigned long long v = slot_init(kind);
  for (int i = tid; i < bps; i += kBlock) v = combine(kind, v, in[i]);
  sm[tid] = v;
  __syncthreads();
  for (int st = kBlock / 2; st > 0; st >>= 1) {
    if (tid < st) sm[tid] = combine(kind, sm[tid], sm[tid + st]);
    __syncthreads();
  }
  if (tid == 0) out[(int64_t)g * out_stride + s] = sm[0];
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

void launch_reduce_fused(const unsigned long long *part, int32_t nsegs, int32_t bps, int32_t nslots,
                         unsigned long long *out, int32_t out_stride, hipStream_t stream) {
  if (nsegs <= 0 || nslots <= 0) return;
  hipLaunchKernelGGL(k_reduce_fused, dim3((unsigned)(nsegs * nslots)), dim3(kBlock), 0, stream, part, nsegs, bps,
                     nslots, out, out_stride);
}

}  // namespace pinot
