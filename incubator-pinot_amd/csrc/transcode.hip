// Device transcode of raw numeric columns (transcode.h):
//   k_raw_keys      big-endian value bytes -> order-preserving u64 key (as segment_parse.cpp raw_value_key) + doc
//   radix sort      (key, doc) pairs over the key's 32 or 64 bits (hipcub)
//   k_new_value     1 where a sorted key differs from its predecessor; an inclusive scan numbers the distinct keys
//   k_scatter_ids   dictId of each doc (its sorted position's number - 1) and the distinct keys in order
//   k_pack_ids      the dictIds MSB-first at `bits` per value, one 32-bit window of the output per thread
#include "transcode.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "common.h"

namespace pinot {
namespace {

__global__ void k_raw_keys(const uint8_t *__restrict__ raw, uint64_t n, int w, int type, unsigned long long *__restrict__ keys,
                           uint32_t *__restrict__ docs) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint8_t *p = raw + i * (uint64_t)w;
    unsigned long long v = 0;
    for (int k = 0; k < w; k++) v = (v << 8) | p[k];
    unsigned long long key;
    if (type == PINOT_INT) {
      key = (unsigned long long)(uint32_t)v ^ 0x80000000ull;
    } else if (type == PINOT_LONG) {
      key = v ^ 0x8000000000000000ull;
    } else if (type == PINOT_FLOAT) {
      uint32_t b = (uint32_t)v;
      if ((b & 0x7F800000u) == 0x7F800000u && (b & 0x7FFFFFu)) b = 0x7FC00000u;  // floatToIntBits NaN
      key = (b & 0x80000000u) ? (unsigned long long)(~b) : (unsigned long long)(b | 0x80000000u);
    } else {
      if ((v & 0x7FF0000000000000ull) == 0x7FF0000000000000ull && (v & 0xFFFFFFFFFFFFFull)) v = 0x7FF8000000000000ull;
      key = (v & 0x8000000000000000ull) ? ~v : (v | 0x8000000000000000ull);
    }
    keys[i] = key;
    docs[i] = (uint32_t)i;
  }
}

__global__ void k_new_value(const unsigned long long *__restrict__ sk, uint64_t n, uint32_t *__restrict__ flag) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    flag[i] = (i == 0 || sk[i] != sk[i - 1]) ? 1u : 0u;
}

__global__ void k_scatter_ids(const unsigned long long *__restrict__ sk, const uint32_t *__restrict__ sdocs,
                              const uint32_t *__restrict__ flag, const uint32_t *__restrict__ num, uint64_t n,
                              uint32_t *__restrict__ ids, unsigned long long *__restrict__ uniq) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t id = num[i] - 1u;
    ids[sdocs[i]] = id;
    if (flag[i]) uniq[id] = sk[i];
  }
}

__global__ void k_pack_ids(const uint32_t *__restrict__ ids, uint64_t n, int bits, uint64_t out_bytes,
                           uint8_t *__restrict__ out) {
  const uint64_t words = (out_bytes + 3) / 4;
  for (uint64_t wd = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; wd < words; wd += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b0 = wd * 32;  // the window's first bit (bit 0 = the MSB of byte 0)
    const uint64_t j0 = b0 / (uint64_t)bits, j1 = std::min<uint64_t>(n - 1, (b0 + 31) / (uint64_t)bits);
    unsigned long long acc = 0;
    for (uint64_t j = j0; j <= j1; j++) {
      const long long end = (long long)(j * (uint64_t)bits + (uint64_t)bits) - (long long)b0;  // past the id's last bit
      const long long sh = 32 - end;
      const unsigned long long v = ids[j];
      acc |= sh >= 0 ? v << sh : v >> (-sh);
    }
    const uint32_t x = (uint32_t)acc;
    for (int k = 0; k < 4; k++)
      if (wd * 4 + k < out_bytes) out[wd * 4 + k] = (uint8_t)(x >> (24 - 8 * k));
  }
}

unsigned grid_for(uint64_t n) { return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 16384)); }

}  // namespace

namespace {
struct TranscodeSizes {
  size_t a8, a4, raw_b, tmp_b;
  size_t total() const { return raw_b + 3 * a8 + 5 * a4 + tmp_b + 256; }
};

TranscodeSizes transcode_sizes(uint64_t n, int w, hipStream_t stream) {
  TranscodeSizes z;
  z.a8 = (n * 8 + 255) / 256 * 256;
  z.a4 = (n * 4 + 255) / 256 * 256;
  z.raw_b = (n * (uint64_t)w + 255) / 256 * 256;
  size_t sort_b = 0, scan_b = 0;
  PINOT_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_b, (const unsigned long long *)nullptr,
                                               (unsigned long long *)nullptr, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                               (int)n, 0, w * 8, stream));
  PINOT_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, scan_b, (const uint32_t *)nullptr, (uint32_t *)nullptr, (int)n, stream));
  z.tmp_b = std::max(sort_b, scan_b);
  return z;
}
}  // namespace

size_t transcode_numeric_device_bytes(uint64_t n, int w, hipStream_t stream) {
  if (n == 0 || n >= (1ull << 31)) return 0;
  return transcode_sizes(n, w, stream).total();
}

void transcode_numeric_device(const uint8_t *raw, uint64_t n, int w, int data_type, hipStream_t stream,
                              std::vector<uint64_t> &uniq, std::vector<uint8_t> &fwd) {
  uniq.clear();
  fwd.clear();
  if (n == 0) return;
  require(n < (1ull << 31), PINOT_ERR_UNSUPPORTED, "device transcode over 2^31 docs");
  const TranscodeSizes z = transcode_sizes(n, w, stream);
  const size_t a8 = z.a8, a4 = z.a4, raw_b = z.raw_b;
  size_t sort_b = z.tmp_b, scan_b = z.tmp_b;
  DeviceBuffer buf(z.total());
  uint8_t *p = buf.get<uint8_t>();
  uint8_t *d_raw = p;
  auto *keys = reinterpret_cast<unsigned long long *>(p + raw_b);
  auto *skeys = reinterpret_cast<unsigned long long *>(p + raw_b + a8);
  auto *d_uniq = reinterpret_cast<unsigned long long *>(p + raw_b + 2 * a8);
  auto *docs = reinterpret_cast<uint32_t *>(p + raw_b + 3 * a8);
  auto *sdocs = reinterpret_cast<uint32_t *>(p + raw_b + 3 * a8 + a4);
  auto *flag = reinterpret_cast<uint32_t *>(p + raw_b + 3 * a8 + 2 * a4);
  auto *num = reinterpret_cast<uint32_t *>(p + raw_b + 3 * a8 + 3 * a4);
  auto *ids = reinterpret_cast<uint32_t *>(p + raw_b + 3 * a8 + 4 * a4);
  void *tmp = p + raw_b + 3 * a8 + 5 * a4;
  PINOT_HIP(hipMemcpyAsync(d_raw, raw, n * (uint64_t)w, hipMemcpyHostToDevice, stream));
  hipLaunchKernelGGL(k_raw_keys, dim3(grid_for(n)), dim3(256), 0, stream, d_raw, n, w, data_type, keys, docs);
  PINOT_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, sort_b, keys, skeys, docs, sdocs, (int)n, 0, w * 8, stream));
  hipLaunchKernelGGL(k_new_value, dim3(grid_for(n)), dim3(256), 0, stream, skeys, n, flag);
  PINOT_HIP(hipcub::DeviceScan::InclusiveSum(tmp, scan_b, flag, num, (int)n, stream));
  hipLaunchKernelGGL(k_scatter_ids, dim3(grid_for(n)), dim3(256), 0, stream, skeys, sdocs, flag, num, n, ids, d_uniq);
  PINOT_HIP(hipGetLastError());
  uint32_t card = 0;
  PINOT_HIP(hipMemcpyAsync(&card, num + (n - 1), 4, hipMemcpyDeviceToHost, stream));
  PINOT_HIP(hipStreamSynchronize(stream));
  require(card >= 1 && card <= n, PINOT_ERR_DEVICE, "device transcode: distinct count out of range");
  uniq.resize(card);
  PINOT_HIP(hipMemcpyAsync(uniq.data(), d_uniq, (size_t)card * 8, hipMemcpyDeviceToHost, stream));
  const int bits = num_bits_per_value(std::max<int64_t>((int64_t)card - 1, 0));
  const uint64_t out_bytes = (n * (uint64_t)bits + 7) / 8;
  auto *packed = reinterpret_cast<uint8_t *>(keys);  // the unsorted keys are dead: n * 8 >= the packed bytes
  hipLaunchKernelGGL(k_pack_ids, dim3(grid_for((out_bytes + 3) / 4)), dim3(256), 0, stream, ids, n, bits, out_bytes, packed);
  PINOT_HIP(hipGetLastError());
  fwd.resize(out_bytes);
  PINOT_HIP(hipMemcpyAsync(fwd.data(), packed, out_bytes, hipMemcpyDeviceToHost, stream));
  PINOT_HIP(hipStreamSynchronize(stream));
}

}  // namespace pinot
