// Device helpers shared by the HIP translation units of the segment executor (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace pinot {
namespace dev {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ uint64_t tail_mask(int64_t w, int64_t nwords, int32_t num_docs) {
  if (w != nwords - 1) return ~0ull;
  const int rem = num_docs - (int)(w * 64);
  return rem >= 64 ? ~0ull : ((1ull << rem) - 1ull);
}

// LDS-DMA (global_load_lds_dwordx4) operand address spaces
typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void glob_void_t;

// Loads through an explicitly global pointer: a pointer read from a descriptor is generic, and a generic (flat)
// load counts against lgkmcnt as well as vmcnt — every later LDS wait would then also wait for it.
template <typename T>
__device__ __forceinline__ T gload(const void *p) {
  return *reinterpret_cast<const __attribute__((address_space(1))) T *>(reinterpret_cast<uintptr_t>(p));
}

// Waits for this wave's outstanding global loads, LDS-DMA included (the staged chunk is then readable
// by the same wave; no other wave reads it).
__device__ __forceinline__ void wait_stage() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int o) {
  return (unsigned long long)__shfl_xor((long long)v, o, 64);
}

__device__ __forceinline__ unsigned long long combine(int kind, unsigned long long a, unsigned long long b) {
  switch (kind) {
    case SLOT_SUM_U64:
      return a + b;
    case SLOT_SUM_F64:
      return (unsigned long long)__double_as_longlong(__longlong_as_double((long long)a) +
                                                      __longlong_as_double((long long)b));
    case SLOT_MINMAX: {
      const uint32_t mn = min((uint32_t)a, (uint32_t)b), mx = max((uint32_t)(a >> 32), (uint32_t)(b >> 32));
      return ((unsigned long long)mx << 32) | mn;
    }
    default:
      return a;
  }
}

__device__ __forceinline__ unsigned long long slot_init(int kind) {
  return kind == SLOT_MINMAX ? 0x00000000FFFFFFFFull : 0ull;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += shfl_xor_u64(v, o);
  return v;
}

}  // namespace dev
}  // namespace pinot
