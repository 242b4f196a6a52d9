// Segment-pruning metadata beyond min / max: per-column bloom filters (the ColumnValueSegmentPruner's EQUALITY test,
// PC/query/pruner/ColumnValueSegmentPruner.java:140-144) and partition metadata (PartitionSegmentPruner,
// PC/query/pruner/PartitionSegmentPruner.java:73-111). PC = pinot-core/src/main/java/org/apache/pinot/core.
//
// Bloom filter: Pinot's GuavaOnHeapBloomFilter (PC/bloom/GuavaOnHeapBloomFilter.java) over
// com.google.common.hash.BloomFilter (guava 20.0, pom.xml:317-320; not in the container, restated from its published
// algorithm): Funnels.stringFunnel(UTF-8) of value.toString(), Hashing.murmur3_128() (MurmurHash3_x64_128, seed 0),
// strategy MURMUR128_MITZ_64 (ordinal 1; MITZ_32, ordinal 0, read too). File = BE int BloomFilterType (GUAVA_ON_HEAP
// = 1), BE int version (1) (BloomFilterCreator.java:57-64), then Guava's writeTo: byte strategy ordinal, byte
// numHashFunctions, BE int word count, BE longs. Sizing: BloomFilterCreator.java:48-53 + BloomFilterUtil.java (pinned
// by BloomFilterCreatorTest's known answers) + BloomFilter.create's optimalNumOfBits / optimalNumOfHashFunctions.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace pinot {

struct BloomFilter {
  int strategy = 1;                // 0 MURMUR128_MITZ_32, 1 MURMUR128_MITZ_64
  int num_hash_functions = 0;
  std::vector<uint64_t> words;     // LockFreeBitArray data (bit i of word i >> 6, 1L << i)

  bool empty() const { return words.empty(); }
  bool might_contain(const std::string &utf8) const;
  void put(const std::string &utf8);
  std::vector<uint8_t> serialize() const;  // the .bloom file (Pinot header + Guava writeTo)
};

// MurmurHash3_x64_128 (seed 0): the two 64-bit halves (Guava's HashCode bytes are h1 then h2, little-endian).
void murmur3_x64_128(const uint8_t *data, size_t len, uint64_t &h1, uint64_t &h2);

// BloomFilterReader(PinotDataBuffer) (PC/segment/index/readers/BloomFilterReader.java:36-50); throws BAD_ARG on a
// malformed file.
BloomFilter parse_bloom_filter(const uint8_t *bytes, size_t len, const std::string &column);
// BloomFilterCreator(indexDir, column, cardinality): maxFalsePosProbability for a 1 MB (8388608-bit) cap, then
// BloomFilter.create(stringFunnel, cardinality, fpp).
BloomFilter create_bloom_filter(int64_t cardinality);
long long bloom_compute_num_bits(long long cardinality, double max_false_pos_probability);  // BloomFilterUtil
int bloom_compute_num_hash_functions(long long cardinality, long long num_bits);

// PartitionFunctionFactory (PC/data/partition/PartitionFunctionFactory.java): Modulo, Murmur, ByteArray, HashCode
// (case-insensitive names). getPartition of a typed value given as (data type, Java toString, int64 / double value).
enum PartitionFunctionKind { PF_NONE = 0, PF_MODULO, PF_MURMUR, PF_BYTE_ARRAY, PF_HASH_CODE };
PartitionFunctionKind partition_function_of(const std::string &name);  // throws BAD_ARG for an unknown name
struct TypedValue {
  int data_type = 0;     // pinot_data_type
  int64_t i = 0;         // INT / LONG
  double d = 0;          // FLOAT (exact float value) / DOUBLE
  std::string s;         // the value's Java toString (STRING: the value)
};
int32_t partition_of(PartitionFunctionKind f, int32_t num_partitions, const TypedValue &v);
// Kafka's murmur2 as MurmurPartitionFunction copies it (seed 0x9747b28c).
int32_t kafka_murmur2(const uint8_t *data, size_t len);
// Java hashCode of the boxed value (Integer / Long / Float / Double / String over UTF-16 code units).
int32_t java_hash_code(const TypedValue &v);

}  // namespace pinot
