// Loopback collective's device step: the element-wise reduction over the ranks' buffers (all on this device).
// A plain HBM stream (n reads + 1 write per element), grid-stride, no atomics: the result is written once.
#include "collective.h"

namespace pinot {
namespace {

template <typename T, int OP>
__global__ void k_rank_reduce(RankPtrs in, int n, T *__restrict__ out, size_t count) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) {
    T acc = static_cast<const T *>(in.p[0])[i];
    for (int r = 1; r < n; r++) {
      const T x = static_cast<const T *>(in.p[r])[i];
      if (OP == 0) acc = acc + x;
      else if (OP == 1) acc = x < acc ? x : acc;
      else acc = x > acc ? x : acc;
    }
    out[i] = acc;
  }
}

template <typename T>
void launch_t(COp op, const RankPtrs &in, int n, void *out, size_t count, hipStream_t st) {
  const int block = 256;
  const size_t want = (count + block - 1) / block;
  const int grid = (int)(want < 2048 ? (want ? want : 1) : 2048);
  T *o = static_cast<T *>(out);
  if (op == COp::SUM) hipLaunchKernelGGL((k_rank_reduce<T, 0>), dim3(grid), dim3(block), 0, st, in, n, o, count);
  else if (op == COp::MIN) hipLaunchKernelGGL((k_rank_reduce<T, 1>), dim3(grid), dim3(block), 0, st, in, n, o, count);
  else hipLaunchKernelGGL((k_rank_reduce<T, 2>), dim3(grid), dim3(block), 0, st, in, n, o, count);
}

}  // namespace

void launch_rank_reduce(CType t, COp op, const RankPtrs &in, int n, void *out, size_t count, hipStream_t st) {
  switch (t) {
    case CType::I64: launch_t<long long>(op, in, n, out, count, st); break;
    case CType::U64: launch_t<unsigned long long>(op, in, n, out, count, st); break;
    case CType::F64: launch_t<double>(op, in, n, out, count, st); break;
    case CType::U8: launch_t<unsigned char>(op, in, n, out, count, st); break;
  }
}

}  // namespace pinot
