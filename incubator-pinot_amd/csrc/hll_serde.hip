// HyperLogLog.getBytes on the device for the groups a device-trimmed group-by keeps (pinot_gpu_group_by_top): the
// server's DataTable writer then copies each DISTINCTCOUNTHLL map value as pre-serialised bytes instead of fetching
// and packing the registers on the host (IntermediateResultsBlock.getDataTable -> ObjectSerDeUtils HYPER_LOG_LOG_SER_DE,
// pinot-core/src/main/java/org/apache/pinot/core/common/ObjectSerDeUtils.java:248-273).
//
// stream-lib 2.7.0 HyperLogLog.getBytes at log2m 8 (restated in datatable.cpp hll_bytes_at): big-endian int log2m (8),
// big-endian int registerSet.size * 4 (43 * 4), then the RegisterSet's 43 big-endian int words, register p in word
// p / 6 at bit 5 * (p % 6) (RegisterSet.set: LOG2_BITS_PER_WORD 6, REGISTER_SIZE 5; 256 registers -> 43 words).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

namespace pinot {
namespace {

constexpr int kHllWords = 45;  // 2 header ints + 43 register words = 180 bytes per group

// One thread per output int of a group's 180 bytes (groups' rows of 256 u8 registers in, 180-B rows out).
__global__ void k_hll_getbytes(const uint8_t *__restrict__ regs, long long n, uint32_t *__restrict__ out) {
  const long long total = n * kHllWords;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long g = i / kHllWords;
    const int w = (int)(i - g * kHllWords);
    uint32_t u;
    if (w == 0) {
      u = 8u;
    } else if (w == 1) {
      u = 43u * 4u;
    } else {
      const int word = w - 2, m = word < 42 ? 6 : 4;
      const uint8_t *r = regs + g * 256 + 6 * word;
      u = 0;
      for (int k = 0; k < m; k++) u |= (uint32_t)(r[k] & 0x1Fu) << (5 * k);
    }
    out[i] = __builtin_bswap32(u);
  }
}

}  // namespace

// regs: [n][256] u8 registers (device); out: [n][180] bytes (device, 4-byte aligned).
void launch_hll_getbytes(const uint8_t *regs, long long n, uint8_t *out, hipStream_t stream) {
  if (n <= 0) return;
  const long long total = n * kHllWords;
  const int grid = (int)std::min<long long>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(k_hll_getbytes, dim3(grid), dim3(256), 0, stream, regs, n, reinterpret_cast<uint32_t *>(out));
}

}  // namespace pinot
