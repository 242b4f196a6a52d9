// Raw (no-dictionary) numeric columns transcoded to the dictionary-encoded form on the device at registration
// (segment.cpp): the host path (segment_parse.cpp transcode_raw) sorts and deduplicates on the CPU, 2-6 s per 32 M-doc
// LONG column. The reference reads such columns raw (PhysicalColumnIndexContainer.java:101-106 picks the
// FixedByteChunkSingleValueReader); this engine serves them through the dictionary plans, so the transcode is a cold
// cost paid once per segment load — here a radix sort of (value key, doc) pairs in HBM, bit-identical to the host's.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace pinot {

// The distinct order-preserving keys of n big-endian values of w bytes (PINOT_INT / LONG / FLOAT / DOUBLE, keyed as
// segment_parse.cpp's raw_value_key does) ascending in uniq, and the docs' dictIds packed MSB-first at
// num_bits_per_value(card - 1) bits in fwd (FixedBitIntReaderWriter, the host pack_ids bytes).
void transcode_numeric_device(const uint8_t *raw, uint64_t n, int w, int data_type, hipStream_t stream,
                              std::vector<uint64_t> &uniq, std::vector<uint8_t> &fwd);
// HBM the device transcode of n values of w bytes allocates (its scratch buffer, hipcub's temporaries included).
size_t transcode_numeric_device_bytes(uint64_t n, int w, hipStream_t stream);

}  // namespace pinot
