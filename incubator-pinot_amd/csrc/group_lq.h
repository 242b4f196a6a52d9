// Lane-owns-quarter column reads shared by the fused group-by kernels (fused_group.hip, group_ring.hip): lane l of a
// pass over 1024 docs owns the 16 consecutive docs 16l .. 16l + 15, i.e. the packed quarter qi, whose 16*B bits start
// at bit 16*B*qi of the MSB-first big-endian fixed-bit stream (PinotDataBitSet.readInt,
// PC/io/util/PinotDataBitSet.java:79-100). A wave's loads of one column are the pass's 128*B contiguous bytes.
#pragma once
#include <hip/hip_runtime.h>

#include "device.h"

namespace pinot {
namespace {
using namespace dev;

typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));

template <int B, int J, typename F>
__device__ __forceinline__ void decode_quarter_apply(const uint32_t (&D)[(B + 1) / 2 + 1], F &f) {
  constexpr int q = J * B, k = q >> 5, o = q & 31;
  constexpr uint32_t mask = (uint32_t)((1ull << B) - 1ull);
  if constexpr (o + B <= 32) f.template put<J>((D[k] >> (32 - o - B)) & mask);
  else f.template put<J>(__builtin_amdgcn_alignbit(D[k], D[k + 1], 64 - o - B) & mask);
  if constexpr (J + 1 < 16) decode_quarter_apply<B, J + 1>(D, f);
}

// Raw dwords of a lane's quarter: ceil(B/2) (+1 for odd B) from dword (qi * B) / 2, issued as up to three 16-B loads
// so that every column's loads of a quarter are in flight before the first decode waits.
__device__ __forceinline__ void load_raw_lq(const uint8_t *fwd, int bits, int64_t qi, uint32_t (&R)[12]) {
  const uint32_t *p = reinterpret_cast<const uint32_t *>(fwd) + ((qi * bits) >> 1);
  const int n = (bits + 1) / 2 + (bits & 1);
  const u32x4a x0 = gload<u32x4a>(p);
  R[0] = x0.x; R[1] = x0.y; R[2] = x0.z; R[3] = x0.w;
  if (n > 4) {  // uniform
    const u32x4a x1 = gload<u32x4a>(p + 4);
    R[4] = x1.x; R[5] = x1.y; R[6] = x1.z; R[7] = x1.w;
  }
  if (n > 8) {
    const u32x4a x2 = gload<u32x4a>(p + 8);
    R[8] = x2.x; R[9] = x2.y; R[10] = x2.z; R[11] = x2.w;
  }
}

struct IdOut {
  uint32_t (&id)[16];
  template <int J>
  __device__ __forceinline__ void put(uint32_t v) { id[J] = v; }
};

// The raw dwords pass through an empty volatile asm first: otherwise the compiler hoists the byte swaps and constant
// shifts of every width of the switch above it (all widths' values live at once).
template <int B>
__device__ __forceinline__ void decode_raw_lq_b(const uint32_t (&Rin)[12], int64_t qi, uint32_t (&id)[16]) {
  constexpr int N = (B + 1) / 2 + (B & 1);
  uint32_t R[N];
#pragma unroll
  for (int i = 0; i < N; i++) {
    R[i] = Rin[i];
    asm volatile("" : "+v"(R[i]));
  }
  uint32_t D[(B + 1) / 2 + 1];
  if constexpr (B & 1) {
    const bool odd = qi & 1;
#pragma unroll
    for (int i = 0; i + 1 < N; i++) D[i] = odd ? __builtin_amdgcn_alignbit(bswap32(R[i]), bswap32(R[i + 1]), 16) : bswap32(R[i]);
    D[N - 1] = bswap32(R[N - 1]);
  } else {
#pragma unroll
    for (int i = 0; i < N; i++) D[i] = bswap32(R[i]);
  }
  IdOut f{id};
  decode_quarter_apply<B, 0>(D, f);
}

// Decode a lane's 16 values and hand them to f inside the width's switch arm (only f's effects leave the switch).
template <typename F>
__device__ __forceinline__ void decode_raw_lq(const uint32_t (&R)[12], int bits, int64_t qi, F &&f) {
#define PINOT_RQ(B)                   \
  {                                   \
    uint32_t id[16];                  \
    decode_raw_lq_b<B>(R, qi, id);    \
    f(id);                            \
  }
  switch (bits) {  // widths up to kGroupLwMaxBits (the host routes wider columns through group_chunk_pf)
    case 1: PINOT_RQ(1); break;   case 2: PINOT_RQ(2); break;   case 3: PINOT_RQ(3); break;   case 4: PINOT_RQ(4); break;
    case 5: PINOT_RQ(5); break;   case 6: PINOT_RQ(6); break;   case 7: PINOT_RQ(7); break;   case 8: PINOT_RQ(8); break;
    case 9: PINOT_RQ(9); break;   case 10: PINOT_RQ(10); break; case 11: PINOT_RQ(11); break; case 12: PINOT_RQ(12); break;
    case 13: PINOT_RQ(13); break; case 14: PINOT_RQ(14); break; case 15: PINOT_RQ(15); break; case 16: PINOT_RQ(16); break;
    case 17: PINOT_RQ(17); break; case 18: PINOT_RQ(18); break; case 19: PINOT_RQ(19); break; case 20: PINOT_RQ(20); break;
    default: break;
  }
#undef PINOT_RQ
}

}  // namespace
}  // namespace pinot
