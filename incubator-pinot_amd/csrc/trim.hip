// Radix selection of the server trim's kept groups (trim.h): no sort of the group arrays.
//
//   k_trim_andor   the keys materialised once, with each block's AND / OR of them (a digit no key varies in is known
//                  without a histogram)
//   k_trim_round   round r (digit bits [56 - 8r, 64 - 8r)): every block histograms the digit of the keys that match
//                  the prefix found so far, per function, in LDS, then adds it into one of kTrimCopies global copies
//                  (a single copy puts every block's adds on the same 256 addresses: memory-side atomics serialise);
//   k_trim_pick    one block: the copies summed, the digit holding the remaining rank picked, the prefix extended.
//                  After eight rounds the prefix is the trimSize-th key K and the rank is how many ties of K in group
//                  order precede it.
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
constexpr size_t kTrimStateBytes = 512;
constexpr int kTrimCopies = 16;  // global histogram copies (block b adds into copy b % kTrimCopies)

struct TrimState {
  unsigned long long prefix[kTrimMaxFns];
  unsigned long long rank[kTrimMaxFns];  // 0-based rank of the trimSize-th key among the keys matching the prefix
  unsigned long long kand[kTrimMaxFns], kor[kTrimMaxFns];  // AND / OR of every key: a digit no key varies in is known
};

struct TrimArgs {
  TrimFn fn[kTrimMaxFns];
  int32_t nf;
  const long long *counts;
  long long n;
  TrimState *st;
  uint32_t *hist;              // [kTrimCopies][nf][256]
  unsigned long long *keys;    // [nf][n]: every group's key per function (k_trim_andor writes them)
  unsigned long long *bandor;  // [blocks][nf][2]: each block's AND / OR
};

__device__ __forceinline__ unsigned long long trim_key_of(const TrimArgs &a, int f, long long i) {
  double v = a.fn[f].vals[i];
  if (a.fn[f].avg) v = v / (double)a.counts[i];
  if (v == 0.0) v = 0.0;
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned long long o = (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
  return a.fn[f].asc ? o : ~o;
}

__device__ __forceinline__ unsigned long long trim_key(const TrimArgs &a, int f, long long i) {
  return a.keys[(size_t)f * a.n + i];
}

__global__ void k_trim_init(TrimArgs a, long long T) {
  for (int i = threadIdx.x; i < kTrimCopies * a.nf * 256; i += blockDim.x) a.hist[i] = 0;
  if (threadIdx.x < kTrimMaxFns) {
    a.st->prefix[threadIdx.x] = 0;
    a.st->rank[threadIdx.x] = (unsigned long long)(T - 1);
  }
}

// The keys, materialised (AVG's division once), and each block's AND / OR of them; kTrimPerThread groups per thread,
// their loads issued together.
__global__ __launch_bounds__(kTrimBlock) void k_trim_andor(TrimArgs a) {
  __shared__ unsigned long long sx[kTrimBlock / 64], so[kTrimBlock / 64];
  const long long i0 = (long long)blockIdx.x * kTrimTile + threadIdx.x;
  for (int f = 0; f < a.nf; f++) {
    unsigned long long k[kTrimPerThread], x = ~0ull, o = 0ull;
#pragma unroll
    for (int j = 0; j < kTrimPerThread; j++) {
      const long long i = i0 + (long long)j * kTrimBlock;
      k[j] = i < a.n ? trim_key_of(a, f, i) : 0ull;
    }
#pragma unroll
    for (int j = 0; j < kTrimPerThread; j++) {
      const long long i = i0 + (long long)j * kTrimBlock;
      if (i < a.n) {
        a.keys[(size_t)f * a.n + i] = k[j];
        x &= k[j];
        o |= k[j];
      }
    }
    for (int m = 32; m > 0; m >>= 1) {
      x &= __shfl_xor(x, m);
      o |= __shfl_xor(o, m);
    }
    if ((threadIdx.x & 63) == 0) {
      sx[threadIdx.x >> 6] = x;
      so[threadIdx.x >> 6] = o;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int w = 1; w < kTrimBlock / 64; w++) {
        x &= sx[w];
        o |= so[w];
      }
      a.bandor[((size_t)blockIdx.x * a.nf + f) * 2] = x;
      a.bandor[((size_t)blockIdx.x * a.nf + f) * 2 + 1] = o;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(kTrimBlock) void k_trim_andor_reduce(TrimArgs a, int blocks) {
  __shared__ unsigned long long sx[kTrimBlock / 64], so[kTrimBlock / 64];
  for (int f = 0; f < a.nf; f++) {
    unsigned long long x = ~0ull, o = 0ull;
    for (int b = threadIdx.x; b < blocks; b += kTrimBlock) {
      x &= a.bandor[((size_t)b * a.nf + f) * 2];
      o |= a.bandor[((size_t)b * a.nf + f) * 2 + 1];
    }
    for (int m = 32; m > 0; m >>= 1) {
      x &= __shfl_xor(x, m);
      o |= __shfl_xor(o, m);
    }
    if ((threadIdx.x & 63) == 0) {
      sx[threadIdx.x >> 6] = x;
      so[threadIdx.x >> 6] = o;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int w = 1; w < kTrimBlock / 64; w++) {
        x &= sx[w];
        o |= so[w];
      }
      a.st->kand[f] = x;
      a.st->kor[f] = o;
    }
    __syncthreads();
  }
}

__device__ __forceinline__ uint32_t trim_vary(const TrimArgs &a, int shift) {
  uint32_t vary = 0;  // functions whose keys differ in this digit (the others' digit is every key's)
  for (int f = 0; f < a.nf; f++)
    if (((a.st->kand[f] ^ a.st->kor[f]) >> shift) & 255ull) vary |= 1u << f;
  return vary;
}

__global__ __launch_bounds__(kTrimBlock) void k_trim_round(TrimArgs a, int round) {
  __shared__ uint32_t h[kTrimMaxFns][256];
  const int tid = threadIdx.x;
  const int shift = 56 - 8 * round;
  const uint32_t vary = trim_vary(a, shift);
  if (!vary) return;
  for (int i = tid; i < a.nf * 256; i += kTrimBlock) h[i >> 8][i & 255] = 0;
  __syncthreads();
  unsigned long long pre[kTrimMaxFns];
  for (int f = 0; f < a.nf; f++) pre[f] = round ? a.st->prefix[f] >> (shift + 8) : 0ull;
  const long long i0 = (long long)blockIdx.x * kTrimTile + tid;
  for (int f = 0; f < a.nf; f++) {
    if (!((vary >> f) & 1u)) continue;
    unsigned long long kk[kTrimPerThread];
#pragma unroll
    for (int j = 0; j < kTrimPerThread; j++) {  // every load first
      const long long i = i0 + (long long)j * kTrimBlock;
      kk[j] = i < a.n ? trim_key(a, f, i) : 0ull;
    }
#pragma unroll
    for (int j = 0; j < kTrimPerThread; j++) {
      const unsigned long long k = kk[j];
      const bool in = i0 + (long long)j * kTrimBlock < a.n && (round == 0 || (k >> (shift + 8)) == pre[f]);
      const uint32_t d = (uint32_t)(k >> shift) & 255u;
      // the wave's most common case first: every lane holding the first active lane's digit in one add
      const unsigned long long act = __ballot(in);
      bool done = !in;
      if (act) {
        const uint32_t d0 = (uint32_t)__shfl((int)d, (int)__builtin_ctzll(act), 64);
        const unsigned long long same = __ballot(in && d == d0);
        if (in && d == d0) {
          done = true;
          if ((tid & 63) == (int)__builtin_ctzll(same)) atomicAdd(&h[f][d0], (uint32_t)__popcll(same));
        }
      }
      if (!done) atomicAdd(&h[f][d], 1u);
    }
  }
  __syncthreads();
  uint32_t *g = a.hist + (size_t)(blockIdx.x % kTrimCopies) * a.nf * 256;
  for (int i = tid; i < a.nf * 256; i += kTrimBlock)
    if (h[i >> 8][i & 255]) atomicAdd(g + i, h[i >> 8][i & 255]);
}

// One block after each round: per function the digit holding the remaining rank (its copies summed), the prefix
// extended; the copies zeroed for the next round.
constexpr int kTrimPickBlock = 1024;
__global__ __launch_bounds__(kTrimPickBlock) void k_trim_pick(TrimArgs a, int round) {
  __shared__ uint32_t c[kTrimMaxFns][256];
  const int tid = threadIdx.x;
  const int shift = 56 - 8 * round;
  const uint32_t vary = trim_vary(a, shift);
  for (int i = tid; i < a.nf * 256; i += kTrimPickBlock) {  // one (function, digit) per thread, its copies loaded at once
    uint32_t v[kTrimCopies];
#pragma unroll
    for (int r = 0; r < kTrimCopies; r++) v[r] = a.hist[(size_t)r * a.nf * 256 + i];
    uint32_t t = 0;
#pragma unroll
    for (int r = 0; r < kTrimCopies; r++) {
      t += v[r];
      a.hist[(size_t)r * a.nf * 256 + i] = 0;
    }
    c[i >> 8][i & 255] = t;
  }
  __syncthreads();
  // wave f finds function f's digit: the first d (<= 255) whose inclusive count prefix exceeds the remaining rank, cum
  // the count below it (a wave scan over four digits per lane instead of one thread's 255-step walk)
  const int wv = tid >> 6, lane = tid & 63;
  if (wv < a.nf) {
    const int f = wv;
    const unsigned long long r = a.st->rank[f];
    if ((vary >> f) & 1u) {
      uint32_t c4[4];
      unsigned long long s = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        c4[k] = c[f][4 * lane + k];
        s += c4[k];
      }
      unsigned long long inc = s;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
      }
      const unsigned long long hit = __ballot(r < inc);
      const int L = hit ? (int)__builtin_ctzll(hit) : 63;
      if (lane == L) {
        unsigned long long cum = inc - s;
        int d = 4 * lane;
        for (int k = 0; k < 4 && d < 255; k++, d++) {
          if (r < cum + c4[k]) break;
          cum += c4[k];
        }
        a.st->prefix[f] |= (unsigned long long)d << shift;
        a.st->rank[f] = r - cum;
      }
    } else if (lane == 0) {  // every key's digit: the rank stays
      a.st->prefix[f] |= ((a.st->kand[f] >> shift) & 255ull) << shift;
    }
  }
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

// ties[f][*] -> its exclusive prefix sums in place (one block per function): the ties of K in each block's earlier
// blocks, read by k_trim_flags (linear in the blocks, whatever the group count).
__global__ __launch_bounds__(kTrimBlock) void k_trim_tie_scan(uint32_t *ties, unsigned blocks) {
  __shared__ uint32_t scan[kTrimBlock];
  const int tid = threadIdx.x;
  uint32_t *t = ties + (size_t)blockIdx.x * blocks;
  uint32_t carry = 0;
  for (unsigned c0 = 0; c0 < blocks; c0 += kTrimBlock) {
    const unsigned i = c0 + (unsigned)tid;
    const uint32_t v = i < blocks ? t[i] : 0u;
    scan[tid] = v;
    __syncthreads();
    for (int o = 1; o < kTrimBlock; o <<= 1) {
      const uint32_t x = tid >= o ? scan[tid - o] : 0u;
      __syncthreads();
      scan[tid] += x;
      __syncthreads();
    }
    if (i < blocks) t[i] = carry + scan[tid] - v;
    carry += scan[kTrimBlock - 1];
    __syncthreads();
  }
}

__global__ __launch_bounds__(kTrimBlock) void k_trim_flags(TrimArgs a, const uint32_t *__restrict__ ties,
                                                           uint32_t *__restrict__ flags) {
  __shared__ uint32_t scan[kTrimBlock];
  __shared__ unsigned long long base[kTrimMaxFns];
  const int tid = threadIdx.x;
  const unsigned b = blockIdx.x;
  if (tid < a.nf) base[tid] = ties[(size_t)tid * gridDim.x + b];  // ties of K in the earlier blocks (k_trim_tie_scan)
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

__global__ void k_key_digits(const long long *__restrict__ keys, long long n, long long key_base, KeyDigits kd,
                             int32_t *__restrict__ ids) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    unsigned long long k = (unsigned long long)(keys[i] + key_base);
    for (int j = 0; j < kd.nc; j++) {
      const unsigned long long c = (unsigned long long)kd.card[j];
      ids[i * kd.nc + j] = (int32_t)(k % c);
      k /= c;
    }
  }
}

}  // namespace

void launch_key_digits(const long long *keys, long long n, long long key_base, const KeyDigits &kd, int32_t *ids,
                       hipStream_t stream) {
  if (n <= 0) return;
  const int grid = (int)std::min<long long>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_key_digits, dim3(grid), dim3(256), 0, stream, keys, n, key_base, kd, ids);
}

size_t trim_radix_scratch_bytes(long long n, int nf) {
  const long long blocks = (n + kTrimTile - 1) / kTrimTile;
  auto up = [](size_t b) { return (b + 255) / 256 * 256; };
  return kTrimStateBytes + up((size_t)kTrimCopies * nf * 256 * 4) + up((size_t)nf * blocks * 4) +
         up((size_t)blocks * nf * 16) + (size_t)nf * n * 8 + 256;
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
  auto up = [](size_t b) { return (b + 255) / 256 * 256; };
  const long long blocks = (n + kTrimTile - 1) / kTrimTile;
  a.st = reinterpret_cast<TrimState *>(p);
  p += kTrimStateBytes;
  a.hist = reinterpret_cast<uint32_t *>(p);
  p += up((size_t)kTrimCopies * nf * 256 * 4);
  auto *ties = reinterpret_cast<uint32_t *>(p);
  p += up((size_t)nf * blocks * 4);
  a.bandor = reinterpret_cast<unsigned long long *>(p);
  p += up((size_t)blocks * nf * 16);
  a.keys = reinterpret_cast<unsigned long long *>(p);
  static_assert(sizeof(TrimState) <= kTrimStateBytes, "trim state");
  const unsigned grid = (unsigned)blocks;  // one tile of kTrimTile groups per block in every pass
  hipLaunchKernelGGL(k_trim_init, dim3(1), dim3(kTrimBlock), 0, stream, a, T);
  hipLaunchKernelGGL(k_trim_andor, dim3(grid), dim3(kTrimBlock), 0, stream, a);
  hipLaunchKernelGGL(k_trim_andor_reduce, dim3(1), dim3(kTrimBlock), 0, stream, a, (int)blocks);
  for (int r = 0; r < 8; r++) {
    hipLaunchKernelGGL(k_trim_round, dim3(grid), dim3(kTrimBlock), 0, stream, a, r);
    hipLaunchKernelGGL(k_trim_pick, dim3(1), dim3(kTrimPickBlock), 0, stream, a, r);
  }
  hipLaunchKernelGGL(k_trim_ties, dim3(grid), dim3(kTrimBlock), 0, stream, a, ties);
  hipLaunchKernelGGL(k_trim_tie_scan, dim3((unsigned)nf), dim3(kTrimBlock), 0, stream, ties, grid);
  hipLaunchKernelGGL(k_trim_flags, dim3(grid), dim3(kTrimBlock), 0, stream, a, ties, flags);
}

}  // namespace pinot
