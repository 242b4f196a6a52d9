// Fused group-by (K6 + K7 over the K1 filter): ONE launch per group-by query over every segment on the GPU.
// Restates DictionaryBasedGroupKeyGenerator (PC/query/aggregation/groupby/DictionaryBasedGroupKeyGenerator.java:195-302)
// and DefaultGroupByExecutor.process (PC/query/aggregation/groupby/DefaultGroupByExecutor.java:70-168) over the
// filter program of fused_common.h (PC = pinot-core/src/main/java/org/apache/pinot/core).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "fused_common.h"

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

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

// One aggregated value into accumulator `acc` at index k (global or LDS address space by pointer).
template <bool LDS>
__device__ __forceinline__ void agg_update(const GroupAggDev &ag, void *acc, long long k, uint32_t id) {
  switch (ag.acc_kind) {
    case 0:
      atomicAdd(static_cast<unsigned long long *>(acc) + k,
                (unsigned long long)(long long)static_cast<const int32_t *>(ag.dict)[id]);
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
      if (a.reserved2 == 0) {
        // all cursor claims first (inactive lanes add 0: no divergent branch around the LDS atomics, one
        // lgkmcnt wait), then the stores; the runs' lines combine in L2
        uint32_t pos[kGroupUnroll];
#pragma unroll
        for (int u = 0; u < kGroupUnroll; u++) pos[u] = atomicAdd(&plds[key[u] >> rshift], act[u] ? 1u : 0u);
#pragma unroll
        for (int u = 0; u < kGroupUnroll; u++)
          if (act[u]) a.emit[pos[u]] = rec[u];
      }
#pragma unroll
      for (int u = 0; u < kGroupUnroll; u++)
        if (act[u]) {
          if (a.reserved2 == 1) {  // debug.emit=1 (timing only, wrong results): sequential stores
            a.emit[doc[u]] = rec[u];
          } else if (a.reserved2 == 2) {  // debug.emit=2: LDS cursor only
            atomicAdd(&plds[key[u] >> a.shift], 1u);
          }
        }
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

// GB_COUNT / GB_EMIT with every needed column prefetched: one global-memory round trip per kGroupPfUnroll
// words instead of one per column (the per-doc reads are latency-bound).
constexpr int kGroupPfUnroll = 4;

template <int MODE>
__device__ __forceinline__ void group_chunk_pf(const GroupArgs &a, const GroupSegment &sg, int64_t ch, uint64_t mask,
                                               int lane, uint32_t *plds) {
  constexpr int C = kGroupPfCols, U = kGroupPfUnroll;
  const int nc = MODE == GB_COUNT ? a.n_gcols : a.pf_nc;
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
  const int rshift = a.shift + a.split;
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
        for (int u = 0; u < U; u++) {
          const uint32_t *p = reinterpret_cast<const uint32_t *>(fwd[c]) + (((uint64_t)doc[u] * (uint32_t)bits[c]) >> 5);
          lo[c][u] = p[0];
          hi[c][u] = p[1];
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
    if constexpr (MODE == GB_COUNT) {
#pragma unroll
      for (int u = 0; u < U; u++)
        if (act[u]) atomicAdd(&plds[key[u] >> a.shift], 1u);
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
}

// LDS accumulator identities (GB_LDS): counts 0, sums 0, min all-ones, max 0, HLL 0.
__device__ __forceinline__ void init_group_lds(const GroupArgs &a, const GroupSegment &sg, uint8_t *acc_lds, int tid) {
  uint32_t *w = reinterpret_cast<uint32_t *>(acc_lds);
  for (int i = tid; i < a.lds_acc_bytes / 4; i += kGroupBlock) w[i] = 0;
  __syncthreads();
  for (int g = 0; g < a.n_aggs; g++) {
    const GroupAggDev ag = load_const(a.aggs + sg.first_agg + g);
    if (ag.acc_kind == 2) {
      unsigned long long *m = reinterpret_cast<unsigned long long *>(acc_lds + ag.lds_off);
      for (long long i = tid; i < a.G; i += kGroupBlock) m[i] = ~0ull;
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void flush_group_lds(const GroupArgs &a, const GroupSegment &sg, uint8_t *acc_lds, int tid) {
  __syncthreads();
  const uint32_t *cnt = reinterpret_cast<const uint32_t *>(acc_lds);
  for (long long k = tid; k < a.G; k += kGroupBlock) {
    const uint32_t c = cnt[k];
    if (!c) continue;
    atomicAdd(a.counts + k, (unsigned long long)c);
    for (int g = 0; g < a.n_aggs; g++) {
      const GroupAggDev ag = load_const(a.aggs + sg.first_agg + g);
      const uint8_t *src = acc_lds + ag.lds_off;
      switch (ag.acc_kind) {
        case 0:
          atomicAdd(static_cast<unsigned long long *>(ag.acc) + k, reinterpret_cast<const unsigned long long *>(src)[k]);
          break;
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

template <int MODE, bool PF = false>
__global__ __launch_bounds__(kGroupBlock) void k_group_query(GroupArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = blockIdx.x / a.bps, b = blockIdx.x % a.bps;
  const int nblk = a.nsegs * a.bps;
  const GroupSegment sg = load_const(a.segs + g);
  const FusedStep *leaves = a.leaves + sg.first_leaf;
  uint8_t *stage = lds + wave * a.stage_bytes;
  uint8_t *acc_lds = lds + (size_t)kGroupWaves * a.stage_bytes;
  uint32_t *plds = reinterpret_cast<uint32_t *>(acc_lds);
  if constexpr (MODE == GB_LDS) init_group_lds(a, sg, acc_lds, tid);
  if constexpr (MODE == GB_COUNT) {
    for (int p = tid; p < a.P; p += kGroupBlock) plds[p] = 0;
    __syncthreads();
  }
  if constexpr (MODE == GB_EMIT) {
    if (a.split == 0) {
      for (int p = tid; p < a.P; p += kGroupBlock) plds[p] = a.offsets[(size_t)p * nblk + blockIdx.x];
    } else {  // coarse run (q, block) starts where run q starts + this block's share of q's earlier blocks
      const int F = 1 << a.split, Q = (a.P + F - 1) >> a.split;
      for (int q = tid; q < Q; q += kGroupBlock) {
        uint32_t c = a.pstart[q * F];
        for (int p = q * F; p < min(a.P, (q + 1) * F); p++) c += a.offsets[(size_t)p * nblk + blockIdx.x] - a.pstart[p];
        plds[q] = c;
      }
    }
    __syncthreads();
  }
  const int64_t nchunks = min((sg.nwords + 63) >> 6, sg.ch_end);
  unsigned long long matched = 0;
  for (int64_t ch = sg.ch_begin + (int64_t)b * kGroupWaves + wave; ch < nchunks; ch += (int64_t)a.bps * kGroupWaves) {
    uint64_t mask = chunk_word(sg.pre, sg.nwords, sg.num_docs, ch, lane);
    mask = eval_filter<true, 12>(leaves, sg.n_leaves, mask, ch * 64 + lane, sg.nwords, sg.num_docs, lane,
                             [&](int, const FusedStep &st) -> const uint8_t * {
                               stage_chunk_rt(st.fwd, st.bits, ch, stage, lane);
                               wait_stage();
                               return stage;
                             });
    matched += __popcll(mask);
    if (__any(mask != 0)) {
      if constexpr (PF) group_chunk_pf<MODE>(a, sg, ch, mask, lane, plds);
      else group_chunk<MODE>(a, sg, ch, mask, lane, acc_lds, plds);
    }
  }
  matched = wave_sum(matched);  // the EMIT pass re-reads what the COUNT pass already counted
  if (MODE != GB_EMIT && MODE != GB_VERIFY && MODE != GB_FIRST && lane == 0 && matched) atomicAdd(a.matched + g, matched);
  if constexpr (MODE == GB_LDS) flush_group_lds(a, sg, acc_lds, tid);
  if constexpr (MODE == GB_COUNT) {
    __syncthreads();
    for (int p = tid; p < a.P; p += kGroupBlock) a.hist[(size_t)p * nblk + blockIdx.x] = plds[p];
  }
}


}  // namespace

size_t group_query_lds_bytes(const GroupArgs &a) {
  size_t acc = 0;
  if (a.mode == GB_LDS) acc = (size_t)a.lds_acc_bytes;
  if (a.mode == GB_COUNT || a.mode == GB_EMIT) acc = (size_t)a.P * 4;
  return (size_t)kGroupWaves * a.stage_bytes + acc;
}

int group_query_blocks_per_cu(const GroupArgs &a) {
  int n = 0;
  const size_t lds = group_query_lds_bytes(a);
  hipError_t err = hipErrorInvalidValue;
  switch (a.mode) {
    case GB_GLOBAL: err = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_group_query<GB_GLOBAL>, kGroupBlock, lds); break;
    case GB_LDS: err = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_group_query<GB_LDS>, kGroupBlock, lds); break;
    case GB_COUNT: err = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_group_query<GB_COUNT>, kGroupBlock, lds); break;
    case GB_FIRST: err = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_group_query<GB_FIRST>, kGroupBlock, lds); break;
    default: err = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_group_query<GB_EMIT>, kGroupBlock, lds); break;
  }
  return (err != hipSuccess || n < 1) ? 1 : n;
}

void launch_group_query(const GroupArgs &a, hipStream_t stream) {
  if (a.nsegs <= 0 || a.bps <= 0) return;
  const dim3 grid((unsigned)(a.nsegs * a.bps)), block(kGroupBlock);
  const size_t lds = group_query_lds_bytes(a);
  switch (a.mode) {
    case GB_GLOBAL: hipLaunchKernelGGL(k_group_query<GB_GLOBAL>, grid, block, lds, stream, a); break;
    case GB_LDS: hipLaunchKernelGGL(k_group_query<GB_LDS>, grid, block, lds, stream, a); break;
    case GB_COUNT: hipLaunchKernelGGL(k_group_query<GB_COUNT>, grid, block, lds, stream, a); break;  // 2 columns: no gain
    case GB_EMIT:
      if (a.pf_nc > 0) hipLaunchKernelGGL((k_group_query<GB_EMIT, true>), grid, block, lds, stream, a);
      else hipLaunchKernelGGL(k_group_query<GB_EMIT>, grid, block, lds, stream, a);
      break;
    case GB_FIRST: hipLaunchKernelGGL(k_group_query<GB_FIRST>, grid, block, lds, stream, a); break;
    default: hipLaunchKernelGGL(k_group_query<GB_VERIFY>, grid, block, lds, stream, a); break;
  }
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
