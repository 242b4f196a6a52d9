// stream-lib 2.7.0 HyperLogLog(log2m = 8) + MurmurHash, host side.
//
// DistinctCountHLLAggregationFunction (PC/query/aggregation/function/DistinctCountHLLAggregationFunction.java:35-360,
// DEFAULT_LOG2M = 8) offers the boxed VALUE of every doc. The device never hashes: the host hashes every
// dictionary value once and uploads (register << 8 | rank) per dictId; the kernels only atomicMax ranks.
#include <cmath>
#include <cstdint>

#include "engine.h"

namespace pinot {

static constexpr uint32_t kM = 0x5bd1e995u;

// MurmurHash.hashLong(long): Integer values are widened (sign-extended) to long first.
uint32_t murmur_hash_long(int64_t data) {
  uint64_t d = static_cast<uint64_t>(data);
  uint32_t h = 0;
  uint32_t k = static_cast<uint32_t>(d) * kM;
  k ^= k >> 24;
  h ^= k * kM;
  k = static_cast<uint32_t>(d >> 32) * kM;
  k ^= k >> 24;
  h *= kM;
  h ^= k * kM;
  h ^= h >> 13;
  h *= kM;
  h ^= h >> 15;
  return h;
}

// MurmurHash.hash(byte[], length, seed = -1) for String values (String.getBytes()).
uint32_t murmur_hash_bytes(const uint8_t *data, int length) {
  uint32_t h = static_cast<uint32_t>(-1) ^ static_cast<uint32_t>(length);
  const int len4 = length >> 2;
  for (int i = 0; i < len4; i++) {
    const int i4 = i << 2;
    uint32_t k = static_cast<uint32_t>(static_cast<int32_t>(static_cast<int8_t>(data[i4 + 3])));
    k = (k << 8) | data[i4 + 2];
    k = (k << 8) | data[i4 + 1];
    k = (k << 8) | data[i4 + 0];
    k *= kM;
    k ^= k >> 24;
    k *= kM;
    h *= kM;
    h ^= k;
  }
  const int left = length - (len4 << 2);
  if (left != 0) {
    auto sb = [&](int i) { return static_cast<uint32_t>(static_cast<int32_t>(static_cast<int8_t>(data[i]))); };
    if (left >= 3) h ^= sb(length - 3) << 16;
    if (left >= 2) h ^= sb(length - 2) << 8;
    if (left >= 1) h ^= sb(length - 1);
    h *= kM;
  }
  h ^= h >> 13;
  h *= kM;
  h ^= h >> 15;
  return h;
}

// HyperLogLog.offerHashed: j = h >>> (32 - log2m); r = nlz((h << log2m) | (1 << (log2m - 1)) + 1) + 1
uint16_t hll_register_rank(uint32_t h) {
  const uint32_t j = h >> 24;
  const uint32_t w = (h << 8) | 129u;
  const uint32_t r = static_cast<uint32_t>(__builtin_clz(w)) + 1u;
  return static_cast<uint16_t>((j << 8) | r);
}

// HyperLogLog.cardinality() with Math.round (floor(x + 0.5); +inf -> Long.MAX_VALUE).
int64_t hll_cardinality(const uint8_t *regs) {
  const double m = 256.0;
  const double alpha_mm = (0.7213 / (1.0 + 1.079 / m)) * m * m;
  double sum = 0.0, zeros = 0.0;
  for (int j = 0; j < 256; j++) {
    sum += 1.0 / static_cast<double>(1u << regs[j]);
    if (regs[j] == 0) zeros += 1.0;
  }
  const double estimate = alpha_mm * (1.0 / sum);
  double x = estimate;
  if (estimate <= 2.5 * m) x = zeros > 0 ? m * std::log(m / zeros) : INFINITY;
  if (std::isinf(x)) return INT64_MAX;
  return static_cast<int64_t>(std::floor(x + 0.5));
}

namespace {
// Linear counting m * log(m / zeros) for zeros = 1 .. 256: the same std::log evaluations, made once (a 1 M-group
// result would otherwise spend milliseconds in log on the host).
struct LinearCounting {
  double v[257];
  LinearCounting() {
    v[0] = INFINITY;
    for (int z = 1; z <= 256; z++) v[z] = 256.0 * std::log(256.0 / (double)z);
  }
};
const LinearCounting kLinearCounting;
}  // namespace

const double *hll_linear_counting_table() { return kLinearCounting.v; }
double hll_alpha_mm() {
  const double m = 256.0;
  return (0.7213 / (1.0 + 1.079 / m)) * m * m;
}

int64_t hll_cardinality_from_sum(unsigned long long sum_fixed32, uint32_t zeros) {
  const double m = 256.0;
  const double alpha_mm = (0.7213 / (1.0 + 1.079 / m)) * m * m;
  const double sum = std::ldexp((double)sum_fixed32, -32);  // exact: the register loop's double sum
  const double estimate = alpha_mm * (1.0 / sum);
  double x = estimate;
  if (estimate <= 2.5 * m) x = zeros <= 256 ? kLinearCounting.v[zeros] : m * std::log(m / (double)zeros);
  if (std::isinf(x)) return INT64_MAX;
  return static_cast<int64_t>(std::floor(x + 0.5));
}

}  // namespace pinot
