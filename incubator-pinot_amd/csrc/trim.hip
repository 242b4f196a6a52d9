// Radix selection of the server trim's kept groups (trim.h): no sort of the group arrays.
//
//   k_trim_round   round r (digit bits [56 - 8r, 64 - 8r)): every block histograms the digit of the keys that match
//                  the prefix found so far, per function, in LDS, then adds its histogram to the global one; the last
//                  block to finish picks the digit holding the remaining rank, extends the prefix, and clears the
//                  histogram for the next round. After eight rounds the prefix is the trimSize-th key K and the rank
//                  is how many ties of K in group order precede it.
//   k_trim_ties    per block of 1024 groups, the ties of K per function.
//   k_trim_flags   per group, the functions keeping it: key < K, or key == K with fewer than rank + 1 earlier ties
//                  (the block's own earlier ties from an LDS scan, the earlier blocks' from k_trim_ties).
//
// Keys as k_trim_keys formed them for the stable sort this replaces: the value (AVG: sum / count; -0.0 as 0.0) as an
// order-preserving u64, complemented for the descending functions.
#include "trim.h"

#include <algorithm>

#include "common.h"

namespace pinot {
namespace {

constexpr int kTrimBlock = 256;
constexpr int kTrimPerThread = 4;                     // k_trim_ties / k_trim_flags: consecutive groups per thread
constexpr int kTrimTile = kTrimBlock * kTrimPerThread;  // groups per block

struct TrimState {
  unsigned long long prefix[kTrimMaxFns];
  unsigned long long rank[kTrimMaxFns];  // 0-based rank of the trimSize-th key among the keys matching the prefix
  uint32_t done;                         // blocks finished in the current round
};

struct TrimArgs {
  TrimFn fn[kTrimMaxFns];
  int32_t nf;
  const long long *counts;
  long long n;
  TrimState *st;
  uint32_t *hist;  // [nf][256]
};

__device__ __forceinline__ unsigned long long trim_key(const TrimArgs &a, int f, long long i) {
  double v = a.fn[f].vals[i];
  if (a.fn[f].avg) v = v / (double)a.counts[i];
  if (v == 0.0) v = 0.0;
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned long long o = (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
  return a.fn[f].asc ? o : ~o;
}

__global__ void k_trim_init(TrimArgs a, long long T) {
  for (int i = threadIdx.x; i < a.nf * 256; i += blockDim.x) a.hist[i] = 0;
  if (threadIdx.x < kTrimMaxFns) {
    a.st->prefix[threadIdx.x] = 0;
    a.st->rank[threadIdx.x] = (unsigned long long)(T - 1);
  }
  if (threadIdx.x == 0) a.st->done = 0;
}

__global__ __launch_bounds__(kTrimBlock) void k_trim_round(TrimArgs a, int round) {
  __shared__ uint32_t h[kTrimMaxFns][256];
  __shared__ bool last;
  const int tid = threadIdx.x;
  for (int i = tid; i < a.nf * 256; i += kTrimBlock) h[i >> 8][i & 255] = 0;
  __syncthreads();
  const int shift = 56 - 8 * round;
  unsigned long long pre[kTrimMaxFns];
  for (int f = 0; f < a.nf; f++) pre[f] = round ? a.st->prefix[f] >> (shift + 8) : 0ull;
  for (long long i = (long long)blockIdx.x * kTrimBlock + tid; i < a.n; i += (long long)gridDim.x * kTrimBlock)
    for (int f = 0; f < a.nf; f++) {
      const unsigned long long k = trim_key(a, f, i);
      if (round == 0 || (k >> (shift + 8)) == pre[f]) atomicAdd(&h[f][(k >> shift) & 255u], 1u);
    }
  __syncthreads();
  for (int i = tid; i < a.nf * 256; i += kTrimBlock)
    if (h[i >> 8][i & 255]) atomicAdd(a.hist + i, h[i >> 8][i & 255]);
  __threadfence();
  __syncthreads();
  if (tid == 0) last = atomicAdd(&a.st->done, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  __threadfence();
  if (tid < a.nf) {  // one thread per function: the digit holding the remaining rank
    const int f = tid;
    unsigned long long r = a.st->rank[f], cum = 0;
    int d = 0;
    for (; d < 256; d++) {
      const unsigned long long c = __hip_atomic_load(a.hist + f * 256 + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (r < cum + c) break;
      cum += c;
    }
    a.st->prefix[f] |= (unsigned long long)(d < 256 ? d : 255) << shift;
    a.st->rank[f] = r - cum;
  }
  __syncthreads();
  for (int i = tid; i < a.nf * 256; i += kTrimBlock) a.hist[i] = 0;
  if (tid == 0) a.st->done = 0;
}

__global__ __launch_bounds__(kTrimBlock) void k_trim_ties(TrimArgs a, uint32_t *ties) {
  __shared__ uint32_t s[kTrimMaxFns];
  const int tid = threadIdx.x;
  if (tid < a.nf) s[tid] = 0;
  __syncthreads();
  const long long i0 = (long long)blockIdx.x * kTrimTile + (long long)tid * kTrimPerThread;
  for (int f = 0; f < a.nf; f++) {
    const unsigned long long K = a.st->prefix[f];
    uint32_t c = 0;
    for (int j = 0; j < kTrimPerThread; j++)
      if (i0 + j < a.n) c += trim_key(a, f, i0 + j) == K;
    if (c) atomicAdd(&s[f], c);
  }
  __syncthreads();
  if (tid < a.nf) ties[(size_t)tid * gridDim.x + blockIdx.x] = s[tid];
}

__global__ __launch_bounds__(kTrimBlock) void k_trim_flags(TrimArgs a, const uint32_t *__restrict__ ties,
                                                           uint32_t *__restrict__ flags) {
  __shared__ uint32_t scan[kTrimBlock];
  __shared__ unsigned long long base[kTrimMaxFns];
  const int tid = threadIdx.x;
  const unsigned b = blockIdx.x;
  if (tid < a.nf) base[tid] = 0;
  __syncthreads();
  for (int f = 0; f < a.nf; f++) {  // ties of K in the earlier blocks
    unsigned long long c = 0;
    for (unsigned j = tid; j < b; j += kTrimBlock) c += ties[(size_t)f * gridDim.x + j];
    if (c) atomicAdd(&base[f], c);
  }
  __syncthreads();
  const long long i0 = (long long)b * kTrimTile + (long long)tid * kTrimPerThread;
  uint32_t m[kTrimPerThread] = {};
  for (int f = 0; f < a.nf; f++) {
    const unsigned long long K = a.st->prefix[f], need = a.st->rank[f] + 1;
    unsigned long long k[kTrimPerThread];
    uint32_t c = 0;
    for (int j = 0; j < kTrimPerThread; j++) {
      k[j] = i0 + j < a.n ? trim_key(a, f, i0 + j) : ~0ull;
      c += i0 + j < a.n && k[j] == K;
    }
    // exclusive scan of the threads' tie counts (thread order = group order)
    scan[tid] = c;
    __syncthreads();
    for (int o = 1; o < kTrimBlock; o <<= 1) {
      const uint32_t x = tid >= o ? scan[tid - o] : 0u;
      __syncthreads();
      scan[tid] += x;
      __syncthreads();
    }
    unsigned long long t = base[f] + scan[tid] - c;
    for (int j = 0; j < kTrimPerThread; j++) {
      if (i0 + j >= a.n) break;
      if (k[j] < K) {
        m[j] |= 1u << f;
      } else if (k[j] == K) {
        if (t < need) m[j] |= 1u << f;
        t++;
      }
    }
    __syncthreads();
  }
  for (int j = 0; j < kTrimPerThread; j++)
    if (i0 + j < a.n) flags[i0 + j] = m[j];
}

}  // namespace

size_t trim_radix_scratch_bytes(long long n, int nf) {
  const long long blocks = (n + kTrimTile - 1) / kTrimTile;
  return 256 + (size_t)nf * 256 * 4 + (size_t)nf * blocks * 4 + 256;
}

void launch_trim_radix(const TrimFn *fns, int nf, const long long *counts, long long n, long long T, uint32_t *flags,
                       void *scratch, size_t scratch_bytes, hipStream_t stream) {
  if (n <= 0) return;
  require(nf >= 1 && nf <= kTrimMaxFns && T >= 1 && T <= n && scratch_bytes >= trim_radix_scratch_bytes(n, nf),
          PINOT_ERR_DEVICE, "trim selection shape");
  TrimArgs a{};
  for (int f = 0; f < nf; f++) a.fn[f] = fns[f];
  a.nf = nf;
  a.counts = counts;
  a.n = n;
  uint8_t *p = static_cast<uint8_t *>(scratch);
  a.st = reinterpret_cast<TrimState *>(p);
  a.hist = reinterpret_cast<uint32_t *>(p + 256);
  auto *ties = reinterpret_cast<uint32_t *>(p + 256 + (size_t)nf * 256 * 4);
  static_assert(sizeof(TrimState) <= 256, "trim state");
  hipLaunchKernelGGL(k_trim_init, dim3(1), dim3(kTrimBlock), 0, stream, a, T);
  const int grid = (int)std::min<long long>((n + kTrimBlock * 16 - 1) / (kTrimBlock * 16), 1024);
  for (int r = 0; r < 8; r++) hipLaunchKernelGGL(k_trim_round, dim3(grid), dim3(kTrimBlock), 0, stream, a, r);
  const unsigned blocks = (unsigned)((n + kTrimTile - 1) / kTrimTile);
  hipLaunchKernelGGL(k_trim_ties, dim3(blocks), dim3(kTrimBlock), 0, stream, a, ties);
  hipLaunchKernelGGL(k_trim_flags, dim3(blocks), dim3(kTrimBlock), 0, stream, a, ties, flags);
}

}  // namespace pinot
