// Group-by back half (gfx950): per-partition reduction of the partitioned plan, ordered compaction of
// the non-empty keys, and the per-group outputs the host finalises.
//
//   k_partition_reduce   one block owns one partition (2^shift consecutive raw keys): its records
//                        (local key | aggregated dictIds) are folded into LDS accumulators (count,
//                        int64 / double sums, ordered min/max, HLL registers), then written to the
//                        dense HBM accumulators with plain stores — no HBM atomics (the keys are the
//                        partition's alone). Restates DefaultGroupByExecutor.process + the
//                        aggregateGroupBySV loops (PC/query/aggregation/groupby/DefaultGroupByExecutor.java:70-168).
//   k_key_flags / k_key_scatter   counts != 0 -> ordered key list (exclusive scan in between), i.e. the
//                        raw keys in ascending order (GroupKeyGenerator.getUniqueGroupKeys, sorted).
//   k_group_final        per non-empty group, the host result arrays: key, count, each function's value and
//                        HyperLogLog.cardinality() from the exact fixed-point Σ 2^(32 - register) (the double sum
//                        of 1.0 / (1 << reg) is exact: <= 256 terms of >= 2^-25), bit-identical to the host's.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "common.h"
#include "device.h"
#include "kernels.h"

namespace pinot {
namespace {
using namespace dev;

constexpr int kReduceBlock = 1024;
constexpr int kReduceUnroll = 8;
constexpr int kReduceCountCopies = 4;  // private count copies (waves w, w + 4 share one)

__device__ __forceinline__ unsigned long long ordered_bits_r(double d) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(d);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}

__device__ __forceinline__ double dict_value_r(const void *dict, int value_kind, uint32_t id) {
  switch (value_kind) {
    case 0: return (double)static_cast<const int32_t *>(dict)[id];
    case 1: return (double)static_cast<const long long *>(dict)[id];
    default: return static_cast<const double *>(dict)[id];
  }
}

// stream-lib MurmurHash.hashLong and HyperLogLog (register << 8 | rank) — the device twins of hll.cpp's
// murmur_hash_long / hll_register_rank (bit-identical integer arithmetic).
__device__ __forceinline__ uint32_t murmur_hash_long_d(long long data) {
  constexpr uint32_t kM = 0x5bd1e995u;
  const unsigned long long d = (unsigned long long)data;
  uint32_t h = 0;
  uint32_t k = (uint32_t)d * kM;
  k ^= k >> 24;
  h ^= k * kM;
  k = (uint32_t)(d >> 32) * kM;
  k ^= k >> 24;
  h *= kM;
  h ^= k * kM;
  h ^= h >> 13;
  h *= kM;
  h ^= h >> 15;
  return h;
}

__device__ __forceinline__ uint32_t hll_register_rank_d(uint32_t h) {
  return ((h >> 24) << 8) | (uint32_t)(__builtin_clz((h << 8) | 129u) + 1);
}

template <bool SKIP_INVALID>
__global__ __launch_bounds__(kReduceBlock) void k_partition_reduce(PartitionReduceArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x;
  const int p = blockIdx.x;
  const int K = 1 << a.shift;
  uint32_t *cnt = reinterpret_cast<uint32_t *>(lds);
  for (int i = tid; i < a.lds_bytes / 4; i += kReduceBlock) reinterpret_cast<uint32_t *>(lds)[i] = 0;
  __syncthreads();
  for (int g = 0; g < a.n_aggs; g++)
    if (a.aggs[g].acc_kind == 2) {
      unsigned long long *m = reinterpret_cast<unsigned long long *>(lds + a.aggs[g].lds_off);
      for (int i = tid; i < K; i += kReduceBlock) m[i] = ~0ull;
    }
  __syncthreads();
  const uint32_t b = a.pstart[p], e = a.pstart[p + 1];
  const unsigned long long kmask = (unsigned long long)K - 1ull;
  // count folded into the first affine dictId SUM: one 64-bit LDS atomic adds (1 << sbits) + dictId, i.e. the
  // count above a sum field of sbits = bits + cbits (n records of < 2^bits each sum to < 2^sbits), when both
  // fields fit (block-uniform: n = this partition's records)
  const uint32_t n = e - b;
  const int cbits = n ? 32 - __builtin_clz(n) : 1;
  int pk = -1, sbits = 0;
  for (int g = 0; g < a.n_aggs; g++)
    if (pk < 0 && a.aggs[g].acc_kind == 0 && a.aggs[g].affine && a.aggs[g].bits + 2 * cbits <= 64) {
      pk = g;
      sbits = a.aggs[g].bits + cbits;
    }
  // counts: one private copy per wave (a partition has few keys: LDS atomics on one copy serialise)
  const int wave = tid >> 6;
  uint32_t *wcnt = cnt + a.wave_cnt_off / 4 + (wave & (kReduceCountCopies - 1)) * K;
  // kReduceUnroll records per thread per step, each stage batched across them (record loads, dictionary /
  // LUT loads, LDS atomics, HLL CAS attempts): the loop is latency-bound with one record in flight
  constexpr int U = kReduceUnroll;
  for (uint32_t r0 = b + tid; r0 < e; r0 += (uint32_t)U * kReduceBlock) {
    unsigned long long rec[U];
    bool ok[U];
    uint32_t k[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t r = r0 + (uint32_t)u * kReduceBlock;
      ok[u] = r < e;
      rec[u] = ok[u] ? __builtin_nontemporal_load(a.records + r) : 0ull;
      if constexpr (SKIP_INVALID) ok[u] = ok[u] && rec[u] != kRecInvalid;
      k[u] = (uint32_t)(rec[u] & kmask);
    }
    if (pk < 0) {
#pragma unroll
      for (int u = 0; u < U; u++)
        if (ok[u]) atomicAdd(wcnt + k[u], 1u);
    }
#pragma unroll
    for (int g = 0; g < kMaxGroupAggs; g++) {
      if (g >= a.n_aggs) break;
      const GroupAggDev &ag = a.aggs[g];
      if (ag.acc_kind == 5) continue;
      uint32_t id[U];
#pragma unroll
      for (int u = 0; u < U; u++) id[u] = ok[u] ? (uint32_t)((rec[u] >> ag.field_shift) & ((1ull << ag.bits) - 1ull)) : 0u;
      uint8_t *acc = lds + ag.lds_off;
      if (ag.acc_kind == 0) {
        long long v[U];  // affine: Σ dictId here, Σ value = base * count + step * Σ dictId at the end
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = ag.affine ? (long long)id[u] : (long long)static_cast<const int32_t *>(ag.dict)[id[u]];
        if (g == pk) {
#pragma unroll
          for (int u = 0; u < U; u++) v[u] += 1ll << sbits;
        }
#pragma unroll
        for (int u = 0; u < U; u++)
          if (ok[u]) atomicAdd(reinterpret_cast<unsigned long long *>(acc) + k[u], (unsigned long long)v[u]);
      } else if (ag.acc_kind == 4) {  // u8 registers: byte max by CAS on the containing dword
        uint32_t h[U];
#pragma unroll
        for (int u = 0; u < U; u++)
          h[u] = ag.affine ? hll_register_rank_d(murmur_hash_long_d(ag.affine_base + ag.affine_step * (long long)id[u]))
                           : (uint32_t)ag.hll_lut[id[u]];
        uint32_t *word[U], old[U], rank[U];
        int sh[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint32_t idx = k[u] * 256 + (h[u] >> 8);
          word[u] = reinterpret_cast<uint32_t *>(acc) + (idx >> 2);
          sh[u] = (int)(idx & 3) * 8;
          rank[u] = ok[u] ? (h[u] & 0xFFu) : 0u;
          old[u] = *word[u];
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
          if (((old[u] >> sh[u]) & 0xFFu) >= rank[u]) continue;
          uint32_t seen = atomicCAS(word[u], old[u], (old[u] & ~(0xFFu << sh[u])) | (rank[u] << sh[u]));
          while (seen != old[u]) {  // another lane / wave changed the dword: retry while still below
            old[u] = seen;
            if (((old[u] >> sh[u]) & 0xFFu) >= rank[u]) break;
            seen = atomicCAS(word[u], old[u], (old[u] & ~(0xFFu << sh[u])) | (rank[u] << sh[u]));
          }
        }
      } else {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = dict_value_r(ag.dict, ag.value_kind, id[u]);
#pragma unroll
        for (int u = 0; u < U; u++) {
          if (!ok[u]) continue;
          if (ag.acc_kind == 1) atomicAdd(reinterpret_cast<double *>(acc) + k[u], v[u]);
          else if (ag.acc_kind == 2) atomicMin(reinterpret_cast<unsigned long long *>(acc) + k[u], ordered_bits_r(v[u]));
          else atomicMax(reinterpret_cast<unsigned long long *>(acc) + k[u], ordered_bits_r(v[u]));
        }
      }
    }
  }
  __syncthreads();
  const long long base = (long long)p * K;
  for (int i = tid; i < K; i += kReduceBlock) {
    const long long key = base + i;
    if (key >= a.G) break;
    uint32_t c = 0;
    if (pk >= 0) c = (uint32_t)(reinterpret_cast<const unsigned long long *>(lds + a.aggs[pk].lds_off)[i] >> sbits);
    else
      for (int w = 0; w < kReduceCountCopies; w++) c += cnt[a.wave_cnt_off / 4 + w * K + i];
    a.counts[key] = c;
  }
  for (int g = 0; g < a.n_aggs; g++) {
    const GroupAggDev &ag = a.aggs[g];
    if (ag.acc_kind == 5) continue;
    const uint8_t *acc = lds + ag.lds_off;
    if (ag.acc_kind == 4) {  // u8 [K][256] -> u8 [G][256], 16 B per thread
      u32x4 *out = reinterpret_cast<u32x4 *>(static_cast<uint8_t *>(ag.acc) + base * 256);
      const long long nkeys = std::min<long long>((long long)K, a.G - base);
      for (long long i = tid; i < nkeys * 16; i += kReduceBlock) out[i] = reinterpret_cast<const u32x4 *>(acc)[i];
    } else {
      unsigned long long *out = static_cast<unsigned long long *>(ag.acc);
      for (int i = tid; i < K; i += kReduceBlock) {
        const long long key = base + i;
        if (key >= a.G) continue;
        unsigned long long v = reinterpret_cast<const unsigned long long *>(acc)[i];
        if (ag.acc_kind == 0 && ag.affine) {
          uint32_t c = 0;
          if (pk >= 0) {
            c = (uint32_t)(reinterpret_cast<const unsigned long long *>(lds + a.aggs[pk].lds_off)[i] >> sbits);
            if (g == pk) v &= (1ull << sbits) - 1ull;
          } else {
            for (int w = 0; w < kReduceCountCopies; w++) c += cnt[a.wave_cnt_off / 4 + w * K + i];
          }
          v = (unsigned long long)ag.affine_base * c + (unsigned long long)ag.affine_step * v;  // exact mod 2^64
        }
        out[key] = v;
      }
    }
  }
}

__global__ void k_key_flags(long long G, const unsigned long long *__restrict__ counts, uint32_t *flags) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < G; i += (long long)gridDim.x * blockDim.x)
    flags[i] = counts[i] != 0 ? 1u : 0u;
}

__global__ void k_key_scatter(long long G, const uint32_t *__restrict__ flags, const uint32_t *__restrict__ pos,
                              long long *keys, unsigned long long *n_out) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < G; i += (long long)gridDim.x * blockDim.x) {
    if (flags[i]) keys[pos[i]] = i;
    if (i == G - 1) *n_out = (unsigned long long)pos[i] + flags[i];
  }
}

// Final per-group arrays in the host result's own layout (copied straight into the pinned result arrays: no host
// fill): raw keys (+ key_base), counts, per function its intermediate value as a double and, for DISTINCTCOUNTHLL,
// HyperLogLog.cardinality() — the host's exact arithmetic (hll.cpp hll_cardinality_from_sum): Σ 2^(32 - reg) as an
// exact integer scaled by 2^-32, alpha_mm * (1 / sum), linear counting m * log(m / zeros) from the host-computed
// table when the estimate is <= 2.5 m, then floor(x + 0.5). IEEE double division / multiplication and no
// contractable multiply-add, so the device rounds exactly as the host does.
__device__ __forceinline__ double decode_ordered_d(unsigned long long o) {
  const unsigned long long u = (o & 0x8000000000000000ull) ? (o & ~0x8000000000000000ull) : ~o;
  return __longlong_as_double((long long)u);
}

__global__ void k_group_final(const unsigned long long *__restrict__ counts, const long long *__restrict__ keys,
                              long long n, GroupFinalArgs f) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const long long k = keys[i];
    const unsigned long long c = counts[k];
    f.out_keys[i] = k + f.key_base;
    f.out_counts[i] = (long long)c;
    if (f.out_counts32) {
      f.out_counts32[i] = (unsigned int)c;
      if (c >> 32) atomicOr(f.overflow, 1u);
    }
    for (int g = 0; g < f.n; g++) {
      double v;
      switch (f.kind[g]) {
        case 0:
        case 6:
        case 7: v = (double)static_cast<const long long *>(f.acc[g])[k]; break;
        case 1: v = static_cast<const double *>(f.acc[g])[k]; break;
        case 2:
        case 3: v = decode_ordered_d(static_cast<const unsigned long long *>(f.acc[g])[k]); break;
        case 4:
        case 9: {
          unsigned long long s = 0;
          uint32_t z = 0;
          if (f.kind[g] == 9) {  // the reduce's packed sums
            const unsigned long long x = static_cast<const unsigned long long *>(f.acc[g])[k];
            s = x & ((1ull << 48) - 1ull);
            z = (uint32_t)(x >> 48);
          }
          const u32x4 *r = reinterpret_cast<const u32x4 *>(static_cast<const uint8_t *>(f.acc[g]) + k * 256);
          for (int q = 0; f.kind[g] == 4 && q < 16; q++) {
            const u32x4 w4 = r[q];
            const uint32_t w[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
            for (int cc = 0; cc < 4; cc++)
#pragma unroll
              for (int bb = 0; bb < 4; bb++) {
                const uint32_t reg = (w[cc] >> (8 * bb)) & 0xFFu;
                s += 1ull << (32 - reg);
                z += reg == 0;
              }
          }
          const double sum = ldexp((double)s, -32);
          const double inv = 1.0 / sum;
          const double estimate = f.alpha_mm * inv;
          double x = estimate;
          if (estimate <= 640.0) x = f.linear[z];
          const long long card = isinf(x) ? 0x7FFFFFFFFFFFFFFFll : (long long)floor(x + 0.5);
          f.out_card[g][i] = card;
          if (f.out_card32[g]) {
            f.out_card32[g][i] = (unsigned int)card;
            if ((unsigned long long)card >> 32) atomicOr(f.overflow, 1u);
          }
          v = (double)card;
          break;
        }
        default: v = (double)c; break;
      }
      f.out_values[g][i] = v;
    }
  }
}

__global__ void k_partition_starts(const uint32_t *__restrict__ offsets, const uint32_t *__restrict__ hist, int32_t P,
                                   int32_t nblk, uint32_t *pstart) {
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p <= P; p += gridDim.x * blockDim.x) {
    if (p < P) pstart[p] = offsets[(size_t)p * nblk];
    else pstart[P] = offsets[(size_t)P * nblk - 1] + hist[(size_t)P * nblk - 1];
  }
}

// Second level of the two-level partitioned plan: block (q, b) moves coarse run (q, b) — the records block b
// of the EMIT pass wrote for partitions q*F .. q*F+F-1, in any order — to those partitions' final slots
// offsets[p][b] (the single-level layout, partition-major then block). Tiles of kSplitTile records are
// counting-sorted by partition in LDS first, so each partition's share of a tile leaves as one contiguous,
// coalesced piece (a per-record scatter costs a cache-line request per record in the address unit).
constexpr int kSplitBlock = 1024;
constexpr int kSplitTile = 8192;

__global__ __launch_bounds__(kSplitBlock) void k_partition_split(const uint32_t *__restrict__ hist, const uint32_t *__restrict__ offsets,
                                                                 const uint32_t *__restrict__ pstart, int32_t P, int32_t nblk,
                                                                 int32_t shift, int32_t split,
                                                                 const unsigned long long *__restrict__ runs,
                                                                 unsigned long long *__restrict__ records, int nt_store) {
  __shared__ unsigned long long sorted[kSplitTile];
  __shared__ uint32_t cur[256], bcount[256], bstart[256];
  __shared__ uint32_t run_b, run_e;
  const int F = 1 << split;
  const int q = blockIdx.x / nblk, b = blockIdx.x % nblk, tid = threadIdx.x;
  if (tid == 0) {
    uint32_t s0 = pstart[q * F], n = 0;
    for (int p = q * F; p < min(P, (q + 1) * F); p++) {
      const size_t i = (size_t)p * nblk + b;
      s0 += offsets[i] - pstart[p];
      n += hist[i];
    }
    run_b = s0;
    run_e = s0 + n;
  }
  if (tid < F) {
    cur[tid] = q * F + tid < P ? offsets[(size_t)(q * F + tid) * nblk + b] : 0u;
    bcount[tid] = 0;
  }
  __syncthreads();
  const uint32_t e = run_e;
  constexpr int R = kSplitTile / kSplitBlock;
  const unsigned long long smask = (unsigned long long)(F - 1);
  for (uint32_t t0 = run_b; t0 < e; t0 += kSplitTile) {
    const uint32_t tn = min((uint32_t)kSplitTile, e - t0);
    unsigned long long rec[R];
    uint32_t rank[R];
#pragma unroll
    for (int i = 0; i < R; i++) {
      const uint32_t j = (uint32_t)(i * kSplitBlock + tid);
      rec[i] = j < tn ? __builtin_nontemporal_load(runs + t0 + j) : 0ull;
    }
#pragma unroll
    for (int i = 0; i < R; i++)
      if ((uint32_t)(i * kSplitBlock + tid) < tn) rank[i] = atomicAdd(&bcount[(rec[i] >> shift) & smask], 1u);
    __syncthreads();
    if (tid < 64) {  // exclusive scan of the F <= 256 bucket counts by one wave
      uint32_t v[4], sum = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int s = tid * 4 + k;
        v[k] = s < F ? bcount[s] : 0u;
        sum += v[k];
      }
      uint32_t incl = sum;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d, 64);
        if (tid >= d) incl += o;
      }
      uint32_t run = incl - sum;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int s = tid * 4 + k;
        if (s < F) bstart[s] = run;
        run += v[k];
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < R; i++)
      if ((uint32_t)(i * kSplitBlock + tid) < tn) sorted[bstart[(rec[i] >> shift) & smask] + rank[i]] = rec[i];
    __syncthreads();
    for (uint32_t j = tid; j < tn; j += kSplitBlock) {
      const unsigned long long r = sorted[j];
      const uint32_t s = (uint32_t)((r >> shift) & smask);
      if (nt_store) __builtin_nontemporal_store(r, records + cur[s] + (j - bstart[s]));
      else records[cur[s] + (j - bstart[s])] = r;
    }
    __syncthreads();
    if (tid < F) {
      cur[tid] += bcount[tid];
      bcount[tid] = 0;
    }
    __syncthreads();
  }
}

__global__ void k_gather_hll(const uint8_t *__restrict__ regs, const long long *__restrict__ keys, long long n,
                             uint8_t *__restrict__ out) {
  // one 16-B piece per thread: 16 pieces per group
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n * 16; i += (long long)gridDim.x * blockDim.x) {
    const long long g = i >> 4, q = i & 15;
    reinterpret_cast<u32x4 *>(out)[i] = reinterpret_cast<const u32x4 *>(regs + keys[g] * 256)[q];
  }
}

__global__ void k_widen_u8(const uint8_t *__restrict__ in, long long n4, int32_t *__restrict__ out) {
  // u8 HLL registers (fused sinks, multi-GPU partial layout) -> u32 (4 registers per thread, one 16-B store)
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    const uint32_t w = reinterpret_cast<const uint32_t *>(in)[i];
    u32x4 o;
    o.x = w & 0xFF;
    o.y = (w >> 8) & 0xFF;
    o.z = (w >> 16) & 0xFF;
    o.w = w >> 24;
    reinterpret_cast<u32x4 *>(out)[i] = o;
  }
}

__global__ void k_narrow_u32(const uint32_t *__restrict__ in, long long n4, uint8_t *__restrict__ out) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    const u32x4 v = reinterpret_cast<const u32x4 *>(in)[i];  // registers are <= 64: no clamping
    reinterpret_cast<uint32_t *>(out)[i] = v.x | (v.y << 8) | (v.z << 16) | (v.w << 24);
  }
}

// Admission threshold of one segment: the upper-th smallest first doc (sorted ascending; 0xFFFFFFFF = absent key),
// or every present key when the segment has at most `upper` of them.
__global__ void k_admit_bitmap(const uint32_t *__restrict__ first_doc, long long G, const uint32_t *__restrict__ sorted,
                               long long upper, uint32_t *__restrict__ bitmap, long long words) {
  const uint32_t t = (sorted && upper <= G) ? sorted[upper - 1] : 0xFFFFFFFEu;
  for (long long w = (long long)blockIdx.x * blockDim.x + threadIdx.x; w < words; w += (long long)gridDim.x * blockDim.x) {
    uint32_t m = 0;
    for (int b = 0; b < 32; b++) {
      const long long k = w * 32 + b;
      if (k >= G) break;
      const uint32_t fd = first_doc[k];
      m |= (fd != 0xFFFFFFFFu && fd <= t) ? (1u << b) : 0u;
    }
    bitmap[w] = m;
  }
}

// AggregationGroupByTrimmingService's per-function selection on the device: the sort key of each group is its
// comparable value (COUNT / SUM / MIN / MAX the intermediate value, AVG sum / count, DISTINCTCOUNTHLL the cardinality:
// k_group_final's out_values, getSorter :160-176) as an order-preserving u64, flipped for the descending functions; a
// stable radix sort then ranks the groups with ties in ascending raw key order (the group index order).
__global__ void k_trim_keys(const double *__restrict__ vals, const long long *__restrict__ counts, int avg, int asc,
                            long long n, unsigned long long *__restrict__ keys, uint32_t *__restrict__ idx) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    double v = vals[i];
    if (avg) v = v / (double)counts[i];
    if (v == 0.0) v = 0.0;  // -0.0 ties with 0.0, as the host's comparison does
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned long long o = (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
    keys[i] = asc ? o : ~o;
    idx[i] = (uint32_t)i;
  }
}

__global__ void k_trim_mark(const uint32_t *__restrict__ idx, long long T, uint32_t bit, uint32_t *__restrict__ flags) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < T; i += (long long)gridDim.x * blockDim.x)
    flags[idx[i]] |= bit;  // one function per launch: no two threads touch one group
}

__global__ void k_nonzero(const uint32_t *__restrict__ flags, long long n, uint32_t *__restrict__ out) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    out[i] = flags[i] != 0u;
}

__global__ void k_union_scatter(const uint32_t *__restrict__ flags, const uint32_t *__restrict__ pos,
                                const long long *__restrict__ keys, long long n, long long *__restrict__ keys_out,
                                uint32_t *__restrict__ flags_out, unsigned long long *__restrict__ n_out) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const uint32_t f = flags[i];
    if (f) {
      keys_out[pos[i]] = keys[i];
      flags_out[pos[i]] = f;
    }
    if (i == n - 1) *n_out = (unsigned long long)pos[i] + (f != 0u);
  }
}

}  // namespace

size_t trim_scratch_bytes(long long n) {
  size_t sort = 0, scan = 0;
  PINOT_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, sort, (const unsigned long long *)nullptr,
                                               (unsigned long long *)nullptr, (const uint32_t *)nullptr,
                                               (uint32_t *)nullptr, (int)n));
  scan = exclusive_sum_u32(nullptr, nullptr, n, nullptr, 0, nullptr);
  const size_t a8 = ((size_t)n * 8 + 255) / 256 * 256, a4 = ((size_t)n * 4 + 255) / 256 * 256;
  return 2 * a8 + 2 * a4 + std::max(sort, scan) + 256;
}

void launch_trim_select(const double *vals, const long long *counts, int avg, int asc, long long n, long long T,
                        uint32_t bit, uint32_t *flags, void *scratch, size_t scratch_bytes, hipStream_t stream) {
  if (n <= 0) return;
  const size_t a8 = ((size_t)n * 8 + 255) / 256 * 256, a4 = ((size_t)n * 4 + 255) / 256 * 256;
  uint8_t *p = static_cast<uint8_t *>(scratch);
  auto *k_in = reinterpret_cast<unsigned long long *>(p), *k_out = reinterpret_cast<unsigned long long *>(p + a8);
  auto *i_in = reinterpret_cast<uint32_t *>(p + 2 * a8), *i_out = reinterpret_cast<uint32_t *>(p + 2 * a8 + a4);
  void *tmp = p + 2 * a8 + 2 * a4;
  size_t tb = scratch_bytes - (2 * a8 + 2 * a4);
  const int grid = (int)std::min<long long>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_trim_keys, dim3(grid), dim3(256), 0, stream, vals, counts, avg, asc, n, k_in, i_in);
  PINOT_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tb, k_in, k_out, i_in, i_out, (int)n, 0, 64, stream));
  const long long t = std::min(T, n);
  hipLaunchKernelGGL(k_trim_mark, dim3((int)std::min<long long>((t + 255) / 256, 4096)), dim3(256), 0, stream, i_out, t,
                     bit, flags);
}

void launch_trim_union(const uint32_t *flags, const long long *keys, long long n, long long *keys_out,
                       uint32_t *flags_out, unsigned long long *n_out, void *scratch, size_t scratch_bytes,
                       hipStream_t stream) {
  if (n <= 0) return;
  const size_t a4 = ((size_t)n * 4 + 255) / 256 * 256;
  uint8_t *p = static_cast<uint8_t *>(scratch);
  auto *nz = reinterpret_cast<uint32_t *>(p), *pos = reinterpret_cast<uint32_t *>(p + a4);
  const int grid = (int)std::min<long long>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_nonzero, dim3(grid), dim3(256), 0, stream, flags, n, nz);
  exclusive_sum_u32(nz, pos, n, p + 2 * a4, scratch_bytes - 2 * a4, stream);
  hipLaunchKernelGGL(k_union_scatter, dim3(grid), dim3(256), 0, stream, flags, pos, keys, n, keys_out, flags_out, n_out);
}

__global__ void k_key_bitmap(const unsigned long long *__restrict__ counts, long long G, uint64_t *bits) {
  const long long nw = (G + 63) / 64;
  const int lane = threadIdx.x & 63;
  for (long long w = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < nw;
       w += ((long long)gridDim.x * blockDim.x) >> 6) {
    const long long k = w * 64 + lane;
    const uint64_t word = __ballot(k < G && counts[k] != 0);
    if (lane == 0) bits[w] = word;
  }
}

void launch_key_bitmap(const unsigned long long *counts, long long G, uint64_t *bits, hipStream_t stream) {
  if (G <= 0) return;
  const long long nw = (G + 63) / 64;
  const int grid = (int)std::min<long long>((nw * 64 + 255) / 256, 4096);
  hipLaunchKernelGGL(k_key_bitmap, dim3(grid), dim3(256), 0, stream, counts, G, bits);
}

void launch_group_final(const unsigned long long *counts, const long long *keys, long long n, const GroupFinalArgs &f,
                        hipStream_t stream) {
  if (n <= 0) return;
  const int grid = (int)std::min<long long>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_group_final, dim3(grid), dim3(256), 0, stream, counts, keys, n, f);
}

size_t admission_scratch_bytes(long long G) {
  size_t need = 0;
  PINOT_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, need, (const uint32_t *)nullptr, (uint32_t *)nullptr, (int)G));
  return ((size_t)G * 4 + 255) / 256 * 256 + need + 256;
}

void launch_admission_bitmaps(const uint32_t *first_doc, int S, long long G, const long long *upper, uint32_t *bitmaps,
                              long long words, void *scratch, size_t scratch_bytes, hipStream_t stream) {
  uint32_t *sorted = static_cast<uint32_t *>(scratch);
  const size_t sorted_b = ((size_t)G * 4 + 255) / 256 * 256;
  void *tmp = static_cast<uint8_t *>(scratch) + sorted_b;
  const int grid = (int)std::min<long long>((words + 255) / 256, 4096);
  for (int s = 0; s < S; s++) {
    const uint32_t *fd = first_doc + (size_t)s * G;
    const bool limited = upper[s] < G;
    if (limited) {
      size_t tb = scratch_bytes - sorted_b;
      PINOT_HIP(hipcub::DeviceRadixSort::SortKeys(tmp, tb, fd, sorted, (int)G, 0, 32, stream));
    }
    hipLaunchKernelGGL(k_admit_bitmap, dim3(grid), dim3(256), 0, stream, fd, G, limited ? sorted : nullptr,
                       limited ? upper[s] : G + 1, bitmaps + (size_t)s * words, words);
  }
}

void launch_narrow_u32(const uint32_t *in, long long n, uint8_t *out, hipStream_t stream) {
  if (n <= 0) return;
  const long long n4 = n / 4;
  const int grid = (int)std::min<long long>((n4 + 255) / 256, 8192);
  hipLaunchKernelGGL(k_narrow_u32, dim3(grid), dim3(256), 0, stream, in, n4, out);
}

void launch_widen_u8(const uint8_t *in, long long n, int32_t *out, hipStream_t stream) {
  if (n <= 0) return;
  const long long n4 = n / 4;  // n = G * 256: always a multiple of 4
  const int grid = (int)std::min<long long>((n4 + 255) / 256, 8192);
  hipLaunchKernelGGL(k_widen_u8, dim3(grid), dim3(256), 0, stream, in, n4, out);
}

__global__ void k_pad_counts(const uint32_t *__restrict__ in, long long n, uint32_t *__restrict__ out) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    out[i] = (in[i] + (kBucketRecs - 1)) & ~(uint32_t)(kBucketRecs - 1);
}

void launch_pad_counts(const uint32_t *in, long long n, uint32_t *out, hipStream_t stream) {
  if (n <= 0) return;
  const int grid = (int)std::min<long long>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_pad_counts, dim3(grid), dim3(256), 0, stream, in, n, out);
}

void launch_partition_starts(const uint32_t *offsets, const uint32_t *hist, int32_t P, int32_t nblk, uint32_t *pstart,
                             hipStream_t stream) {
  if (P <= 0) return;
  hipLaunchKernelGGL(k_partition_starts, dim3((P + 256) / 256), dim3(256), 0, stream, offsets, hist, P, nblk, pstart);
}

void launch_partition_split(const uint32_t *hist, const uint32_t *offsets, const uint32_t *pstart, int32_t P,
                            int32_t nblk, int32_t shift, int32_t split, const unsigned long long *runs,
                            unsigned long long *records, int nt_store, hipStream_t stream) {
  if (P <= 0 || split <= 0) return;
  const int Q = (P + (1 << split) - 1) >> split;
  hipLaunchKernelGGL(k_partition_split, dim3((unsigned)Q * (unsigned)nblk), dim3(kSplitBlock), 0, stream, hist, offsets, pstart,
                     P, nblk, shift, split, runs, records, nt_store);
}

void launch_gather_hll(const uint8_t *regs, const long long *keys, long long n, uint8_t *out, hipStream_t stream) {
  if (n <= 0) return;
  const int grid = (int)std::min<long long>((n * 16 + 255) / 256, 8192);
  hipLaunchKernelGGL(k_gather_hll, dim3(grid), dim3(256), 0, stream, regs, keys, n, out);
}

void launch_partition_reduce(const PartitionReduceArgs &a, hipStream_t stream) {
  if (a.P <= 0) return;
  if (a.skip_invalid)
    hipLaunchKernelGGL(k_partition_reduce<true>, dim3((unsigned)a.P), dim3(kReduceBlock), (size_t)a.lds_bytes, stream, a);
  else
    hipLaunchKernelGGL(k_partition_reduce<false>, dim3((unsigned)a.P), dim3(kReduceBlock), (size_t)a.lds_bytes, stream, a);
}

size_t exclusive_sum_u32(const uint32_t *in, uint32_t *out, long long n, void *tmp, size_t tmp_bytes,
                         hipStream_t stream) {
  size_t need = 0;
  PINOT_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, need, in, out, (int)n, stream));
  if (!tmp) return need;
  PINOT_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, in, out, (int)n, stream));
  return need;
}

size_t compact_keys_scratch_bytes(long long G) {
  const size_t flags = ((size_t)G * 4 + 255) / 256 * 256;
  return 2 * flags + exclusive_sum_u32(nullptr, nullptr, G, nullptr, 0, nullptr) + 256;
}

void launch_compact_keys_ordered(long long G, const unsigned long long *counts, long long *keys_out,
                                 unsigned long long *n_out, void *scratch, size_t scratch_bytes, hipStream_t stream) {
  if (G <= 0) return;
  const size_t flags_b = ((size_t)G * 4 + 255) / 256 * 256;
  uint32_t *flags = static_cast<uint32_t *>(scratch);
  uint32_t *pos = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(scratch) + flags_b);
  uint8_t *tmp = static_cast<uint8_t *>(scratch) + 2 * flags_b;
  const int grid = (int)std::min<long long>((G + 255) / 256, 4096);
  hipLaunchKernelGGL(k_key_flags, dim3(grid), dim3(256), 0, stream, G, counts, flags);
  exclusive_sum_u32(flags, pos, G, tmp, scratch_bytes - 2 * flags_b, stream);
  hipLaunchKernelGGL(k_key_scatter, dim3(grid), dim3(256), 0, stream, G, flags, pos, keys_out, n_out);
}

}  // namespace pinot
