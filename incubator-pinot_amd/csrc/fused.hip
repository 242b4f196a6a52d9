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

#include "fused_common.h"

namespace pinot {
namespace {
using namespace dev;

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

template <int B, bool G>
__device__ __forceinline__ void fold_step(const FusedStep &st, const uint8_t *stage, uint32_t off, uint64_t mask,
                                          FoldPart &r, HllRegs *hll) {
  uint32_t v[32];
  decode_half<B>(stage, off, v);
  fold_half<B, G>(st, (uint32_t)mask, v, r, hll);
  decode_half<B>(stage, off + 4 * B, v);
  fold_half<B, G>(st, (uint32_t)(mask >> 32), v, r, hll);
}


template <bool G>
__device__ __forceinline__ void fold_rt(const FusedStep &st, const uint8_t *stage, uint32_t off, uint64_t mask,
                                        FoldPart &r, HllRegs *hll) {
#define PINOT_FOLD(B) fold_step<B, G>(st, stage, off, mask, r, hll)
  PINOT_WIDTH_SWITCH(st.bits, PINOT_FOLD)
#undef PINOT_FOLD
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
  if (a.seq) {
    __threadfence_system();  // this thread's result stores, visible to the host
    __syncthreads();
    if (tid == 0) {
      unsigned long long *tail = reinterpret_cast<unsigned long long *>(reinterpret_cast<uint8_t *>(a.result) +
                                                                        a.result_tail_off);
      tail[1] = wall_clock64() - *a.clock_start;
      *a.clock_start = ~0ull;
      __hip_atomic_store(reinterpret_cast<uint32_t *>(tail), a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}


// One chunk of the segment program: the filter program, then the folds over the surviving docs.
// `src(i, st)` returns the LDS address of step i's staged chunk (staging it first in the stepwise kernel). Returns the chunk's matching doc count.
template <bool G, typename Src>
__device__ __forceinline__ unsigned long long eval_chunk(const FusedStep *__restrict__ steps, int n_leaves,
                                                         int n_folds, uint64_t mask, FoldAcc &A, HllRegs *hll,
                                                         int64_t w, int64_t nwords, int32_t num_docs, int lane,
                                                         Src &&src) {
  mask = eval_filter<G, 32, kMaxFusedStack>(steps, n_leaves, mask, w, nwords, num_docs, lane, src);
  const unsigned long long cnt = __popcll(mask);
  for (int i = 0; i < n_folds; i++) {
    if (!__any(mask != 0)) break;
    const FusedStep st = load_const(steps + n_leaves + i);  // st.fold == i (host order)
    FoldPart r;
    fold_rt<G>(st, src(n_leaves + i, st), (uint32_t)(lane * (8 * st.bits)), mask, r, hll);
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


// Stepwise shape: per chunk, each step's column is staged into the wave's single LDS stage and
// decoded before the next step is fetched (a step is fetched only while the chunk still has matches).
// G = false: streaming-only program (RANGE / 64-entry LUT leaves, Σ dictId and min/max folds), register-light;
// G = true: also memory-LUT leaves, dictionary-value sums and HLL (per-value gathers).
template <bool G>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(G ? 2 : 4))) void k_scan_query(FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t stage_lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (a.seq && tid == 0) atomicMin(a.clock_start, wall_clock64());  // the launch's first block start
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
                           stage_chunk_rt(st.fwd, st.bits, ch, lds_wave, lane, a.nt != 0);
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
  if (a.seq && tid == 0) atomicMin(a.clock_start, wall_clock64());  // the launch's first block start
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


}  // namespace pinot
