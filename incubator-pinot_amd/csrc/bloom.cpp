// Bloom filters and partition functions of the segment pruners (bloom.h has the references).
#include "bloom.h"

#include <climits>
#include <cmath>
#include <cstring>

#include "engine.h"

namespace pinot {

namespace {
inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}
inline uint64_t le64(const uint8_t *p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
  return v;
}
uint32_t be32(const uint8_t *p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }
uint64_t be64(const uint8_t *p) { return ((uint64_t)be32(p) << 32) | be32(p + 4); }
void put_be32(std::vector<uint8_t> &o, uint32_t v) {
  for (int s = 24; s >= 0; s -= 8) o.push_back((uint8_t)(v >> s));
}
void put_be64(std::vector<uint8_t> &o, uint64_t v) {
  put_be32(o, (uint32_t)(v >> 32));
  put_be32(o, (uint32_t)v);
}
constexpr uint64_t kLongMax = 0x7FFFFFFFFFFFFFFFull;
}  // namespace

void murmur3_x64_128(const uint8_t *data, size_t len, uint64_t &out1, uint64_t &out2) {
  const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
  uint64_t h1 = 0, h2 = 0;
  const size_t nblocks = len / 16;
  for (size_t i = 0; i < nblocks; i++) {
    uint64_t k1 = le64(data + 16 * i), k2 = le64(data + 16 * i + 8);
    k1 *= c1;
    k1 = rotl64(k1, 31);
    k1 *= c2;
    h1 ^= k1;
    h1 = rotl64(h1, 27);
    h1 += h2;
    h1 = h1 * 5 + 0x52dce729;
    k2 *= c2;
    k2 = rotl64(k2, 33);
    k2 *= c1;
    h2 ^= k2;
    h2 = rotl64(h2, 31);
    h2 += h1;
    h2 = h2 * 5 + 0x38495ab5;
  }
  const uint8_t *tail = data + 16 * nblocks;
  uint64_t k1 = 0, k2 = 0;
  const size_t rem = len & 15;
  for (size_t i = rem; i > 8; i--) k2 ^= (uint64_t)tail[i - 1] << (8 * (i - 9));
  if (rem > 8) {
    k2 *= c2;
    k2 = rotl64(k2, 33);
    k2 *= c1;
    h2 ^= k2;
  }
  for (size_t i = rem < 8 ? rem : 8; i > 0; i--) k1 ^= (uint64_t)tail[i - 1] << (8 * (i - 1));
  if (rem > 0) {
    k1 *= c1;
    k1 = rotl64(k1, 31);
    k1 *= c2;
    h1 ^= k1;
  }
  h1 ^= (uint64_t)len;
  h2 ^= (uint64_t)len;
  h1 += h2;
  h2 += h1;
  h1 = fmix64(h1);
  h2 = fmix64(h2);
  h1 += h2;
  h2 += h1;
  out1 = h1;
  out2 = h2;
}

// BloomFilterStrategies.MURMUR128_MITZ_32 / MURMUR128_MITZ_64 (mightContain / put walk the same bit indexes).
template <typename F>
static bool walk_bits(const BloomFilter &b, const std::string &s, F &&f) {
  uint64_t h1, h2;
  murmur3_x64_128(reinterpret_cast<const uint8_t *>(s.data()), s.size(), h1, h2);
  const uint64_t bit_size = (uint64_t)b.words.size() * 64;
  if (b.strategy == 0) {
    const int32_t a = (int32_t)(uint32_t)h1, c = (int32_t)(uint32_t)(h1 >> 32);
    for (int i = 1; i <= b.num_hash_functions; i++) {
      int32_t combined = (int32_t)((uint32_t)a + (uint32_t)i * (uint32_t)c);
      if (combined < 0) combined = ~combined;
      if (!f((uint64_t)combined % bit_size)) return false;
    }
    return true;
  }
  uint64_t combined = h1;
  for (int i = 0; i < b.num_hash_functions; i++) {
    if (!f((combined & kLongMax) % bit_size)) return false;
    combined += h2;
  }
  return true;
}

bool BloomFilter::might_contain(const std::string &utf8) const {
  if (words.empty()) return true;
  return walk_bits(*this, utf8, [&](uint64_t i) { return ((words[i >> 6] >> (i & 63)) & 1ull) != 0; });
}

void BloomFilter::put(const std::string &utf8) {
  if (words.empty()) return;
  walk_bits(*this, utf8, [&](uint64_t i) {
    words[i >> 6] |= 1ull << (i & 63);
    return true;
  });
}

std::vector<uint8_t> BloomFilter::serialize() const {
  std::vector<uint8_t> o;
  put_be32(o, 1);  // BloomFilterType.GUAVA_ON_HEAP
  put_be32(o, 1);  // GuavaOnHeapBloomFilter.VERSION
  o.push_back((uint8_t)strategy);
  o.push_back((uint8_t)num_hash_functions);
  put_be32(o, (uint32_t)words.size());
  for (uint64_t w : words) put_be64(o, w);
  return o;
}

BloomFilter parse_bloom_filter(const uint8_t *p, size_t len, const std::string &column) {
  auto bad = [&](const std::string &why) { return Error(PINOT_ERR_BAD_ARG, column + ": bloom filter: " + why); };
  if (len < 14) throw bad("truncated header");
  if (be32(p) != 1) throw bad("type " + std::to_string(be32(p)) + " (only GUAVA_ON_HEAP = 1)");
  if (be32(p + 4) != 1) throw bad("version " + std::to_string(be32(p + 4)));
  BloomFilter b;
  b.strategy = p[8];
  if (b.strategy > 1) throw bad("strategy ordinal " + std::to_string(b.strategy));
  b.num_hash_functions = p[9];
  if (b.num_hash_functions < 1) throw bad("no hash functions");
  const int32_t n = (int32_t)be32(p + 10);
  if (n < 1 || (uint64_t)n * 8 != len - 14) throw bad("bit array length");
  b.words.resize((size_t)n);
  for (int32_t i = 0; i < n; i++) b.words[(size_t)i] = be64(p + 14 + 8 * (size_t)i);
  return b;
}

long long bloom_compute_num_bits(long long cardinality, double p) {
  return (long long)std::ceil((cardinality * std::log(p)) / std::log(1.0 / std::pow(2.0, std::log(2.0))));
}

int bloom_compute_num_hash_functions(long long cardinality, long long num_bits) {
  return (int)std::max(1.0, std::floor(((double)num_bits / cardinality) * std::log(2.0) + 0.5));  // Math.round
}

BloomFilter create_bloom_filter(int64_t cardinality) {
  constexpr long long kMbInBits = 8388608;   // BloomFilterCreator.MB_IN_BITS
  constexpr double kDefaultFpp = 0.05;       // DEFAULT_MAX_FALSE_POS_PROBABILITY
  const long long card = std::max<long long>(cardinality, 0);
  double fpp = kDefaultFpp;                  // BloomFilterUtil.computeMaxFalsePositiveProbabilityForNumBits
  if (card > 0 && bloom_compute_num_bits(card, kDefaultFpp) > kMbInBits) {
    const int k = bloom_compute_num_hash_functions(card, kMbInBits);
    fpp = std::pow(1.0 - std::exp(-1.0 * k / ((double)kMbInBits / card)), k);
  }
  // com.google.common.hash.BloomFilter.create(funnel, expectedInsertions, fpp)
  const long long n = card == 0 ? 1 : card;
  const long long num_bits = (long long)(-n * std::log(fpp) / (std::log(2.0) * std::log(2.0)));
  BloomFilter b;
  b.strategy = 1;
  b.num_hash_functions = std::max(1, (int)std::floor((double)num_bits / n * std::log(2.0) + 0.5));
  b.words.assign((size_t)((num_bits + 63) / 64), 0ull);
  return b;
}

PartitionFunctionKind partition_function_of(const std::string &name) {
  std::string l;
  for (char ch : name) l.push_back((char)std::tolower((unsigned char)ch));
  if (l == "modulo") return PF_MODULO;
  if (l == "murmur") return PF_MURMUR;
  if (l == "bytearray") return PF_BYTE_ARRAY;
  if (l == "hashcode") return PF_HASH_CODE;
  throw Error(PINOT_ERR_BAD_ARG, "No enum constant for: " + name);
}

int32_t kafka_murmur2(const uint8_t *data, size_t length) {
  const uint32_t m = 0x5bd1e995u;
  const int r = 24;
  uint32_t h = 0x9747b28cu ^ (uint32_t)length;
  const size_t length4 = length / 4;
  for (size_t i = 0; i < length4; i++) {
    const size_t i4 = i * 4;
    uint32_t k = (uint32_t)data[i4] + ((uint32_t)data[i4 + 1] << 8) + ((uint32_t)data[i4 + 2] << 16) +
                 ((uint32_t)data[i4 + 3] << 24);
    k *= m;
    k ^= k >> r;
    k *= m;
    h *= m;
    h ^= k;
  }
  const size_t t = length & ~(size_t)3;
  switch (length % 4) {
    case 3: h ^= (uint32_t)data[t + 2] << 16; [[fallthrough]];
    case 2: h ^= (uint32_t)data[t + 1] << 8; [[fallthrough]];
    case 1:
      h ^= (uint32_t)data[t];
      h *= m;
  }
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return (int32_t)h;
}

int32_t java_hash_code(const TypedValue &v) {
  switch (v.data_type) {
    case PINOT_INT: return (int32_t)v.i;
    case PINOT_LONG: return (int32_t)(uint32_t)((uint64_t)v.i ^ ((uint64_t)v.i >> 32));
    case PINOT_FLOAT: {  // Float.floatToIntBits: NaN canonical
      const float f = (float)v.d;
      uint32_t u;
      std::memcpy(&u, &f, 4);
      if (std::isnan(f)) u = 0x7fc00000u;
      return (int32_t)u;
    }
    case PINOT_DOUBLE: {  // Double.doubleToLongBits: NaN canonical
      uint64_t u;
      std::memcpy(&u, &v.d, 8);
      if (std::isnan(v.d)) u = 0x7ff8000000000000ull;
      return (int32_t)(uint32_t)(u ^ (u >> 32));
    }
    default: {  // String.hashCode over UTF-16 code units
      uint32_t h = 0;
      const std::string &s = v.s;
      for (size_t i = 0; i < s.size();) {
        const uint8_t c0 = (uint8_t)s[i];
        uint32_t cp;
        int n;
        if (c0 < 0x80) cp = c0, n = 1;
        else if ((c0 >> 5) == 6) cp = c0 & 0x1F, n = 2;
        else if ((c0 >> 4) == 14) cp = c0 & 0x0F, n = 3;
        else cp = c0 & 0x07, n = 4;
        for (int k = 1; k < n && i + (size_t)k < s.size(); k++) cp = (cp << 6) | ((uint8_t)s[i + (size_t)k] & 0x3F);
        i += (size_t)n;
        if (cp >= 0x10000) {
          cp -= 0x10000;
          h = 31 * h + (0xD800 + (cp >> 10));
          h = 31 * h + (0xDC00 + (cp & 0x3FF));
        } else {
          h = 31 * h + cp;
        }
      }
      return (int32_t)h;
    }
  }
}

int32_t partition_of(PartitionFunctionKind f, int32_t n, const TypedValue &v) {
  switch (f) {
    case PF_MODULO: {  // Integer values (or the String's Integer.parseInt), Java %: may be negative
      int64_t x;
      if (v.data_type == PINOT_INT) x = v.i;
      else if (v.data_type == PINOT_STRING) x = java_parse_integer(v.s, INT32_MIN, INT32_MAX);
      else throw Error(PINOT_ERR_BAD_QUERY, "Illegal argument for partitioning, expected Integer");
      return (int32_t)((int32_t)x % n);
    }
    case PF_MURMUR:
      return (int32_t)(((uint32_t)kafka_murmur2(reinterpret_cast<const uint8_t *>(v.s.data()), v.s.size()) & 0x7fffffffu) %
                       (uint32_t)n);
    case PF_BYTE_ARRAY: {  // abs(Arrays.hashCode(toString().getBytes())) % n, abs(MIN_VALUE) -> 0
      uint32_t h = 1;
      for (char ch : v.s) h = 31 * h + (uint32_t)(int32_t)(int8_t)ch;
      const int32_t x = (int32_t)h;
      const int32_t a = x == INT32_MIN ? 0 : (x < 0 ? -x : x);
      return a % n;
    }
    case PF_HASH_CODE: {  // Math.abs(hashCode()) % n: abs(MIN_VALUE) stays negative
      const int32_t x = java_hash_code(v);
      const int32_t a = x == INT32_MIN ? INT32_MIN : (x < 0 ? -x : x);
      return a % n;
    }
    default: return -1;
  }
}

}  // namespace pinot
