// Host half of segment registration: every check on the caller's column bytes, with no device involved.
// register_column (segment.cpp) runs parse_column and only then uploads; pinot_segment_validate runs it alone.
// This file and planner.cpp are what the sanitizer build (Makefile `fuzz`, tests/fuzz/fuzz_host.cpp) exercises
// with malformed descriptors: a bad byte must come back as PINOT_ERR_BAD_ARG, never as a fault.
//
// Readers restated (PC = pinot-core/src/main/java/org/apache/pinot/core):
//   dictionaries   PC/segment/index/readers/{Int,Long,Float,Double,String}Dictionary.java (BE values, padded strings)
//   sorted index   PC/segment/index/readers/SortedIndexReaderImpl.java:34-39 (2 BE ints per dictId)
//   inverted index PC/segment/index/readers/BitmapInvertedIndexReader.java:92-119 (BE offsets + portable roaring)
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>

#include "engine.h"

namespace pinot {

// ---------------------------------------------------------------- Java Double.toString / Float.toString
// The digits are the shortest decimal that reads back as the same double (float), the closest such if several,
// and when one digit suffices the closest of the 1- and 2-digit ones (Double.toString javadoc, JDK 19+ wording:
// Double.MIN_VALUE -> 4.9E-324, Float.MIN_VALUE -> 1.4E-45). Layout:
// plain decimal with at least one fraction digit for 1e-3 <= |v| < 1e7, else d.dddE<exp>
// (DoubleDictionary.getStringValue -> Double.toString, PC/segment/index/readers/DoubleDictionary.java:73-75).
static std::string java_layout(bool neg, const std::string &digits, int exp10) {
  std::string out = neg ? "-" : "";
  if (exp10 >= -3 && exp10 < 7) {
    if (exp10 >= 0) {
      std::string ip = digits.substr(0, std::min<size_t>(digits.size(), (size_t)exp10 + 1));
      while ((int)ip.size() < exp10 + 1) ip += '0';
      std::string fp = (int)digits.size() > exp10 + 1 ? digits.substr(exp10 + 1) : "0";
      out += ip + "." + fp;
    } else {
      out += "0." + std::string((size_t)(-exp10 - 1), '0') + digits;
    }
  } else {
    out += digits.substr(0, 1) + "." + (digits.size() > 1 ? digits.substr(1) : "0") + "E" + std::to_string(exp10);
  }
  return out;
}

// Shortest digits of a finite positive v: for p = 1, 2, ... the correctly rounded p-digit decimal D x 10^q, or, when
// that one misses v's rounding interval (asymmetric at powers of two), its neighbour D -/+ 1 in the last place
// if that one reads back as v. Returns the digits without trailing zeros and the exponent of the first digit.
template <typename T>
static void shortest_digits(T v, int max_p, std::string &digits, int &exp10) {
  auto reads_back = [&](unsigned long long d, int q) {
    char b[48];
    snprintf(b, sizeof(b), "%llue%d", d, q);
    if constexpr (sizeof(T) == 4) return strtof(b, nullptr) == v;
    else return strtod(b, nullptr) == v;
  };
  char buf[64];
  for (int p = 1; p <= max_p; p++) {
    snprintf(buf, sizeof(buf), "%.*e", p - 1, (double)v);
    unsigned long long d = 0;
    const char *c = buf;
    for (; *c && *c != 'e'; c++)
      if (*c >= '0' && *c <= '9') d = d * 10 + (unsigned long long)(*c - '0');
    const int e = atoi(c + 1), q = e - (p - 1);
    unsigned long long pick = 0;
    int pq = q;
    if (reads_back(d, q)) pick = d;
    else if (d > 1 && reads_back(d - 1, q)) pick = d - 1;
    else if (reads_back(d + 1, q)) pick = d + 1;
    if (pick && p == 1) {  // one digit suffices: the javadoc then takes the closest of the 1- and 2-digit decimals
      snprintf(buf, sizeof(buf), "%.1e", (double)v);
      const unsigned long long d2 = (unsigned long long)(buf[0] - '0') * 10 + (unsigned long long)(buf[2] - '0');
      const int q2 = atoi(buf + 4) - 1;
      if (reads_back(d2, q2)) {
        pick = d2;
        pq = q2;
      }
    }
    if (pick || p == max_p) {
      if (!pick) pick = d;
      digits = std::to_string(pick);
      exp10 = pq + (int)digits.size() - 1;
      while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
      return;
    }
  }
}

std::string java_double_to_string(double v) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) return v > 0 ? "Infinity" : "-Infinity";
  if (v == 0) return std::signbit(v) ? "-0.0" : "0.0";
  std::string digits;
  int e10;
  shortest_digits<double>(std::fabs(v), 17, digits, e10);
  return java_layout(v < 0, digits, e10);
}

std::string java_float_to_string(float v) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) return v > 0 ? "Infinity" : "-Infinity";
  if (v == 0) return std::signbit(v) ? "-0.0" : "0.0";
  std::string digits;
  int e10;
  shortest_digits<float>(std::fabs(v), 9, digits, e10);
  return java_layout(v < 0, digits, e10);
}

std::string ColumnData::string_value(int32_t id) const {
  switch (data_type) {
    case PINOT_INT:
    case PINOT_LONG:
      return std::to_string(dict_int[id]);
    case PINOT_FLOAT:  // FloatDictionary.getStringValue -> Float.toString
      return java_float_to_string(static_cast<float>(dict_dbl[id]));
    case PINOT_DOUBLE:
      return java_double_to_string(dict_dbl[id]);
    default:
      return dict_str[id];
  }
}

double ColumnData::double_value(int32_t id) const {
  switch (data_type) {
    case PINOT_INT:
    case PINOT_LONG:
      return static_cast<double>(dict_int[id]);
    case PINOT_FLOAT:
    case PINOT_DOUBLE:
      return dict_dbl[id];
    default:
      return std::stod(dict_str[id]);
  }
}

// ---------------------------------------------------------------- dictionaries
static void decode_dictionary(ColumnData &c, const pinot_column_desc &d) {
  const uint8_t *p = d.dictionary;
  const int64_t card = c.card;
  auto need = [&](uint64_t w, const char *what) {
    require(card == 0 || (p != nullptr && d.dictionary_len / w >= (uint64_t)card), PINOT_ERR_BAD_ARG,
            c.name + ": " + what + " dictionary too short");
  };
  switch (c.data_type) {
    case PINOT_INT:
      need(4, "INT");
      c.dict_int.resize(card);
      for (int64_t i = 0; i < card; i++) c.dict_int[i] = static_cast<int32_t>(load_be32(p + 4 * i));
      break;
    case PINOT_LONG:
      need(8, "LONG");
      c.dict_int.resize(card);
      for (int64_t i = 0; i < card; i++) c.dict_int[i] = static_cast<int64_t>(load_be64(p + 8 * i));
      break;
    case PINOT_FLOAT:
      need(4, "FLOAT");
      c.dict_dbl.resize(card);
      for (int64_t i = 0; i < card; i++) {
        uint32_t u = load_be32(p + 4 * i);
        float f;
        memcpy(&f, &u, 4);
        c.dict_dbl[i] = static_cast<double>(f);
      }
      break;
    case PINOT_DOUBLE:
      need(8, "DOUBLE");
      c.dict_dbl.resize(card);
      for (int64_t i = 0; i < card; i++) {
        uint64_t u = load_be64(p + 8 * i);
        memcpy(&c.dict_dbl[i], &u, 8);
      }
      break;
    case PINOT_STRING: {
      const int w = d.string_width;
      require(w >= 1 && w <= (1 << 20), PINOT_ERR_BAD_ARG, c.name + ": STRING dictionary width");
      need((uint64_t)w, "STRING");
      c.dict_str.resize(card);
      for (int64_t i = 0; i < card; i++) {
        const char *s = reinterpret_cast<const char *>(p + (size_t)i * w);
        size_t n = 0;  // getUnpaddedString: stop at the first padding byte (FixedByteValueReaderWriter.java:56-68)
        while (n < (size_t)w && (uint8_t)s[n] != (uint8_t)c.string_pad) n++;
        c.dict_str[i].assign(s, n);
      }
      break;
    }
    default:
      throw Error(PINOT_ERR_BAD_ARG, c.name + ": unknown data type");
  }
  if (d.dictionary_len) c.dict_be.assign(d.dictionary, d.dictionary + d.dictionary_len);
}

// ---------------------------------------------------------------- portable roaring
// RoaringBitmap 0.8.0 RoaringArray.deserialize: the container directory the device binary-searches. Every
// property the kernels rely on is checked here: keys strictly ascending (binary search), array values strictly
// ascending (binary search), runs inside their 65536-doc key (the LDS tile k_roaring_expand ORs them into),
// payloads inside the blob.
static void parse_roaring(const uint8_t *blob, size_t len, uint64_t base, std::vector<RoaringContainer> &out,
                          const std::string &col) {
  auto u16 = [&](size_t o) -> uint32_t {
    require(o <= len && len - o >= 2, PINOT_ERR_BAD_ARG, col + ": truncated roaring bitmap");
    return (uint32_t)blob[o] | ((uint32_t)blob[o + 1] << 8);
  };
  auto u32 = [&](size_t o) -> uint32_t { return u16(o) | (u16(o + 2) << 16); };
  const uint32_t cookie = u32(0);
  size_t pos = 4;
  uint32_t n;
  const uint8_t *runs = nullptr;
  bool has_offsets;
  if (cookie == 12346u) {  // SERIAL_COOKIE_NO_RUNCONTAINER
    n = u32(4);
    pos = 8;
    has_offsets = true;
  } else if ((cookie & 0xFFFFu) == 12347u) {  // SERIAL_COOKIE
    n = (cookie >> 16) + 1;
    require(len - pos >= (n + 7) / 8, PINOT_ERR_BAD_ARG, col + ": truncated roaring run bitmap");
    runs = blob + pos;
    pos += (n + 7) / 8;
    has_offsets = n >= 4;  // NO_OFFSET_THRESHOLD
  } else {
    throw Error(PINOT_ERR_BAD_ARG, col + ": bad roaring cookie");
  }
  require(n <= 65536, PINOT_ERR_BAD_ARG, col + ": roaring container count > 65536");
  const size_t kc = pos;
  pos += 4 * (size_t)n;
  const size_t offs = pos;
  if (has_offsets) pos += 4 * (size_t)n;
  require(pos <= len, PINOT_ERR_BAD_ARG, col + ": truncated roaring header");
  int64_t prev_key = -1;
  for (uint32_t i = 0; i < n; i++) {
    RoaringContainer c{};
    c.key = (uint16_t)u16(kc + 4 * i);
    require((int64_t)c.key > prev_key, PINOT_ERR_BAD_ARG, col + ": roaring keys not ascending");
    prev_key = c.key;
    const uint32_t card = u16(kc + 4 * i + 2) + 1;
    const bool is_run = runs && ((runs[i / 8] >> (i % 8)) & 1);
    const size_t start = has_offsets ? u32(offs + 4 * i) : pos;
    size_t size;
    if (is_run) {
      const uint32_t nruns = u16(start);
      c.type = 2;
      c.cardinality = nruns;
      c.payload_offset = base + start + 2;
      size = 2 + 4 * (size_t)nruns;
    } else if (card > 4096) {  // DEFAULT_MAX_SIZE: bitmap container
      c.type = 1;
      c.cardinality = card;
      c.payload_offset = base + start;
      size = 8192;
    } else {
      c.type = 0;
      c.cardinality = card;
      c.payload_offset = base + start;
      size = 2 * (size_t)card;
    }
    require(start <= len && len - start >= size, PINOT_ERR_BAD_ARG, col + ": roaring container out of bounds");
    if (c.type == 0) {
      for (uint32_t k = 1; k < card; k++)
        require(u16(start + 2 * k) > u16(start + 2 * (k - 1)), PINOT_ERR_BAD_ARG,
                col + ": roaring array container not strictly ascending");
    } else if (c.type == 2) {
      for (uint32_t k = 0; k < c.cardinality; k++)
        require(u16(start + 2 + 4 * k) + u16(start + 4 + 4 * k) <= 0xFFFFu, PINOT_ERR_BAD_ARG,
                col + ": roaring run leaves its container");
    }
    pos = start + size;
    out.push_back(c);
  }
}

// ---------------------------------------------------------------- one column
void parse_column(ColumnData &c, const pinot_column_desc &d, int32_t num_docs, ParsedIndexes &out) {
  require(d.name != nullptr, PINOT_ERR_BAD_ARG, "column without name");
  c.name = d.name;
  c.data_type = d.data_type;
  require(d.cardinality >= 0, PINOT_ERR_BAD_ARG, c.name + ": negative cardinality");
  c.card = d.cardinality;
  c.bits = d.bits_per_value;
  c.is_sorted = d.is_sorted != 0;
  c.has_inverted = d.has_inverted_index != 0 || c.is_sorted;
  c.string_width = d.string_width;
  require(d.padding_byte >= 0 && d.padding_byte <= 255, PINOT_ERR_BAD_ARG, c.name + ": padding byte out of range");
  c.string_pad = d.padding_byte;
  c.num_docs = num_docs;
  require(c.card >= 1 || num_docs == 0, PINOT_ERR_BAD_ARG, c.name + ": empty dictionary");
  require(c.bits >= 1 && c.bits <= 32, PINOT_ERR_BAD_ARG, c.name + ": bits out of range");
  // The reader takes the width from the segment metadata (column.<c>.bitsPerElement, ColumnMetadata.java:98 ->
  // FixedBitSingleValueReader, PhysicalColumnIndexContainer.java:99); the creator writes
  // getNumBitsPerValue(card - 1) (SegmentColumnarIndexCreator.java:404), so any wider width still decodes.
  require(c.bits >= num_bits_per_value(std::max<int64_t>(c.card - 1, 0)), PINOT_ERR_BAD_ARG,
          c.name + ": bits_per_value < getNumBitsPerValue(cardinality - 1)");
  decode_dictionary(c, d);
  require((d.min_value == nullptr) == (d.max_value == nullptr), PINOT_ERR_BAD_ARG,
          c.name + ": minValue without maxValue (or the reverse)");
  if (d.min_value) {
    c.has_minmax = true;
    c.min_value = d.min_value;
    c.max_value = d.max_value;
  }
  parse_pruning_metadata(c, d);

  const int64_t n = num_docs;
  c.fwd_bytes = (uint64_t)((n * c.bits + 7) / 8);
  out.sorted_starts.clear();
  out.containers.clear();
  if (d.multi_value) {
    parse_multi_value(c, d, num_docs);
  } else if (c.is_sorted) {
    require(d.sorted_index && d.sorted_index_len / 8 >= (uint64_t)c.card, PINOT_ERR_BAD_ARG,
            c.name + ": sorted index must hold 2 ints per dictId");
    c.sorted_start.resize(c.card);
    c.sorted_end.resize(c.card);
    out.sorted_starts.resize((size_t)c.card + 1);
    for (int32_t i = 0; i < c.card; i++) {
      c.sorted_start[i] = static_cast<int32_t>(load_be32(d.sorted_index + 8 * i));
      c.sorted_end[i] = static_cast<int32_t>(load_be32(d.sorted_index + 8 * i + 4));
      out.sorted_starts[i] = c.sorted_start[i];
    }
    out.sorted_starts[c.card] = (int32_t)n;
    // the ranges tile [0, numDocs) in dictId order (k_sorted_to_fwd writes doc positions from them)
    for (int32_t i = 0; i < c.card; i++) {
      const int64_t s = c.sorted_start[i], e = c.sorted_end[i];
      require(s == (i == 0 ? 0 : (int64_t)c.sorted_end[i - 1] + 1) && e >= s - 1 && e < n, PINOT_ERR_BAD_ARG,
              c.name + ": sorted index ranges must tile the docs");
    }
    require(c.card == 0 || (int64_t)c.sorted_end[c.card - 1] == n - 1, PINOT_ERR_BAD_ARG,
            c.name + ": sorted index ranges must tile the docs");
  } else {
    require(d.forward_index && d.forward_index_len >= c.fwd_bytes, PINOT_ERR_BAD_ARG,
            c.name + ": forward index shorter than ceil(N*b/8) (FixedBitIntReaderWriter.java:31-36)");
  }
  if (!c.is_sorted && c.has_inverted) {
    require(d.inverted_index && d.inverted_index_len / 4 >= (uint64_t)c.card + 1, PINOT_ERR_BAD_ARG,
            c.name + ": inverted index header");
    require(d.inverted_index_len < (1ull << 32), PINOT_ERR_UNSUPPORTED, c.name + ": inverted index beyond 4 GiB");
    c.inv_dir.assign((size_t)c.card + 1, 0);
    c.inv_bytes.assign(c.card, 0);
    for (int32_t i = 0; i < c.card; i++) {
      const uint32_t o0 = load_be32(d.inverted_index + 4 * i), o1 = load_be32(d.inverted_index + 4 * (i + 1));
      require(o0 <= o1 && o1 <= d.inverted_index_len, PINOT_ERR_BAD_ARG, c.name + ": inverted index offsets");
      c.inv_dir[i] = (int32_t)out.containers.size();
      c.inv_bytes[i] = o1 - o0;
      parse_roaring(d.inverted_index + o0, o1 - o0, o0, out.containers, c.name);
    }
    c.inv_dir[c.card] = (int32_t)out.containers.size();
  }
}

// ---------------------------------------------------------------- multi-value forward index
// FixedBitMultiValueReader (PC/io/reader/impl/v1/FixedBitMultiValueReader.java:60-74): CHUNK OFFSET (BE int per
// chunk of numRowsPerChunk = (int) ceil((float) 2048 / (numValues / numRows)) rows: the entry index of the chunk's
// first row), BITMAP (one bit per entry, MSB first as PinotDataBitSet reads it: set = the entry starts a row), RAW
// DATA (the entries' dictIds at bits_per_value, FixedBitIntReaderWriter). The row starts become a CSR offset array.
void parse_multi_value(ColumnData &c, const pinot_column_desc &d, int32_t num_docs) {
  require(!c.is_sorted, PINOT_ERR_BAD_ARG, c.name + ": a multi-value column cannot be sorted");
  require(d.encoding == PINOT_ENCODING_DICTIONARY, PINOT_ERR_UNSUPPORTED, c.name + ": raw multi-value columns");
  const int64_t rows = num_docs, values = d.total_number_of_entries;
  require(values >= rows && values < ((int64_t)1 << 32) - 1, PINOT_ERR_BAD_ARG,
          c.name + ": totalNumberOfEntries must be >= numDocs (every row holds a value) and < 2^32");
  c.mv = true;
  c.num_values = values;
  c.mv_offsets_host.assign((size_t)rows + 1, 0);
  c.fwd_bytes = (uint64_t)((values * c.bits + 7) / 8);
  if (rows == 0) {
    c.mv_raw_offset = 0;
    return;
  }
  const int64_t per_row = values / rows;  // Java int division
  const float q = 2048.0f / (float)per_row;
  const int64_t rows_per_chunk = std::max<int64_t>(1, (int64_t)std::ceil((double)q));
  const int64_t num_chunks = (rows + rows_per_chunk - 1) / rows_per_chunk;
  const uint64_t off_bytes = (uint64_t)num_chunks * 4, bitmap_bytes = (uint64_t)((values + 7) / 8);
  require(d.forward_index && d.forward_index_len >= off_bytes + bitmap_bytes + c.fwd_bytes, PINOT_ERR_BAD_ARG,
          c.name + ": multi-value forward index shorter than its chunk offsets + bitmap + packed entries");
  const uint8_t *bitmap = d.forward_index + off_bytes;
  int64_t row = 0, longest = 0;
  for (uint64_t byte = 0; byte < bitmap_bytes; byte++) {
    uint8_t b = bitmap[byte];
    while (b) {
      const int k = __builtin_clz((uint32_t)b) - 24;  // MSB first: bit 7 of the byte is entry 8 * byte
      const int64_t entry = (int64_t)byte * 8 + k;
      b &= (uint8_t)~(0x80u >> k);
      if (entry >= values) break;
      require(row < rows, PINOT_ERR_BAD_ARG, c.name + ": more row starts than rows");
      require(row > 0 || entry == 0, PINOT_ERR_BAD_ARG, c.name + ": the first entry must start a row");
      c.mv_offsets_host[(size_t)row++] = (uint32_t)entry;
    }
  }
  require(row == rows, PINOT_ERR_BAD_ARG, c.name + ": fewer row starts than rows");
  c.mv_offsets_host[(size_t)rows] = (uint32_t)values;
  for (int64_t r = 0; r < rows; r++)
    longest = std::max<int64_t>(longest, (int64_t)c.mv_offsets_host[(size_t)r + 1] - c.mv_offsets_host[(size_t)r]);
  c.max_mv = (int32_t)longest;
  require(d.max_number_of_multi_values <= 0 || longest <= d.max_number_of_multi_values, PINOT_ERR_BAD_ARG,
          c.name + ": a row longer than maxNumberOfMultiValues");
  for (int64_t k = 0; k < num_chunks; k++)  // each chunk offset is its first row's start (getIntArray reads them)
    require((int64_t)load_be32(d.forward_index + 4 * k) == (int64_t)c.mv_offsets_host[(size_t)(k * rows_per_chunk)],
            PINOT_ERR_BAD_ARG, c.name + ": chunk offset " + std::to_string(k) + " disagrees with the bitmap");
  c.mv_raw_offset = off_bytes + bitmap_bytes;
}

// ---------------------------------------------------------------- pruning metadata
// Bloom filter: the .bloom bytes (BloomFilterReader), or built from the dictionary values' toString as
// BloomFilterHandler does at load (BloomFilterHandler.java:107-116: creator.add(dictionaryReader.get(i)) for every
// dictId; Dictionary.getStringValue is that toString for every type). Partition metadata as ColumnMetadata reads it
// (ColumnMetadata.java:184-194).
// The dictionary and pruning metadata of a dictionary-encoded column, nothing else (no forward or inverted index):
// the stateless pruning call builds bloom filters / partition lists from it (pruner.cpp prune_segment_desc).
void parse_dictionary_only(ColumnData &c, const pinot_column_desc &d) {
  require(d.name != nullptr, PINOT_ERR_BAD_ARG, "column without name");
  c.name = d.name;
  c.data_type = d.data_type;
  require(d.cardinality >= 0, PINOT_ERR_BAD_ARG, c.name + ": negative cardinality");
  c.card = d.cardinality;
  c.string_width = d.string_width;
  require(d.padding_byte >= 0 && d.padding_byte <= 255, PINOT_ERR_BAD_ARG, c.name + ": padding byte out of range");
  c.string_pad = d.padding_byte;
  decode_dictionary(c, d);
  parse_pruning_metadata(c, d);
}

void parse_pruning_metadata(ColumnData &c, const pinot_column_desc &d) {
  require(!(d.bloom_filter && d.create_bloom_filter), PINOT_ERR_BAD_ARG,
          c.name + ": bloom filter bytes and create_bloom_filter together");
  if (d.bloom_filter) {
    c.bloom = parse_bloom_filter(d.bloom_filter, d.bloom_filter_len, c.name);
  } else if (d.create_bloom_filter) {
    c.bloom = create_bloom_filter(c.card);
    for (int32_t i = 0; i < c.card; i++) c.bloom.put(c.string_value(i));
  }
  if (d.partition_function) {
    c.partition_fn = partition_function_of(d.partition_function);
    require(d.num_partitions > 0, PINOT_ERR_BAD_ARG, c.name + ": Number of partitions must be > 0");
    c.num_partitions = d.num_partitions;
    if (d.num_partition_values == -1) {  // the partitions of every dictionary value, as the creator records them
      for (int32_t i = 0; i < c.card; i++) {
        TypedValue v;
        v.data_type = c.data_type;
        if (c.data_type == PINOT_INT || c.data_type == PINOT_LONG) v.i = c.dict_int[(size_t)i];
        else if (c.data_type != PINOT_STRING) v.d = c.dict_dbl[(size_t)i];
        v.s = c.string_value(i);
        try {
          c.partitions.push_back(partition_of((PartitionFunctionKind)c.partition_fn, c.num_partitions, v));
        } catch (const Error &e) {
          throw Error(PINOT_ERR_BAD_ARG, c.name + ": " + e.what());
        }
      }
    } else {
      require(d.num_partition_values >= 0 && (d.num_partition_values == 0 || d.partition_values), PINOT_ERR_BAD_ARG,
              c.name + ": partition values");
      c.partitions.assign(d.partition_values, d.partition_values + d.num_partition_values);
    }
    std::sort(c.partitions.begin(), c.partitions.end());
    c.partitions.erase(std::unique(c.partitions.begin(), c.partitions.end()), c.partitions.end());
  } else {
    require(d.num_partition_values == 0, PINOT_ERR_BAD_ARG, c.name + ": partition values without a partition function");
  }
}

// ---------------------------------------------------------------- raw (no-dictionary) columns
// FixedByteChunkSingleValueReader values (PC/io/reader/impl/v1/FixedByteChunkSingleValueReader.java) become the
// dictionary form the device path reads: the distinct values sorted as the segment creator sorts a dictionary
// (Arrays.sort on the primitives: Integer / Long order, Float / Double.compare order), each doc's dictId packed at
// getNumBitsPerValue(card - 1) bits, MSB first (FixedBitIntReaderWriter).
namespace {

// fn(t) for t in [0, T) on T threads (registration is a cold path: plain threads, no pool)
void run_threads(size_t T, const std::function<void(size_t)> &fn) {
  if (T <= 1) {
    fn(0);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(T - 1);
  for (size_t t = 1; t < T; t++) th.emplace_back(fn, t);
  fn(0);
  for (auto &x : th) x.join();
}

size_t transcode_threads(uint64_t n, size_t requested) {
  if (requested) return requested;
  const size_t hw = std::max<size_t>(1, std::thread::hardware_concurrency());
  return (size_t)std::max<uint64_t>(1, std::min<uint64_t>({n >> 20, 16, hw}));
}

// Chunk t of T over [0, n) with boundaries on multiples of `align`.
void chunk_of(uint64_t n, size_t T, size_t t, uint64_t align, uint64_t &lo, uint64_t &hi) {
  auto at = [&](size_t k) { return k >= T ? n : std::min<uint64_t>(n, (n * k / T) / align * align); };
  lo = at(t);
  hi = at(t + 1);
}

// The distinct values of v in ascending order: chunks sorted and deduplicated in parallel, then merged pairwise
// (each round's merges in parallel).
template <class V>
std::vector<V> sorted_unique(std::vector<V> v, size_t T) {
  const uint64_t n = v.size();
  if (T > n / 2) T = std::max<size_t>(1, (size_t)(n / 2));
  std::vector<std::vector<V>> parts(T);
  run_threads(T, [&](size_t t) {
    uint64_t lo, hi;
    chunk_of(n, T, t, 1, lo, hi);
    std::vector<V> &p = parts[t];
    p.assign(std::make_move_iterator(v.begin() + lo), std::make_move_iterator(v.begin() + hi));
    std::sort(p.begin(), p.end());
    p.erase(std::unique(p.begin(), p.end()), p.end());
  });
  v.clear();
  v.shrink_to_fit();
  while (parts.size() > 1) {
    std::vector<std::vector<V>> next((parts.size() + 1) / 2);
    run_threads(next.size(), [&](size_t k) {
      if (2 * k + 1 == parts.size()) {
        next[k] = std::move(parts[2 * k]);
        return;
      }
      std::vector<V> &a = parts[2 * k], &b = parts[2 * k + 1], &o = next[k];
      o.reserve(a.size() + b.size());
      std::merge(std::make_move_iterator(a.begin()), std::make_move_iterator(a.end()),
                 std::make_move_iterator(b.begin()), std::make_move_iterator(b.end()), std::back_inserter(o));
      o.erase(std::unique(o.begin(), o.end()), o.end());
      std::vector<V>().swap(a);
      std::vector<V>().swap(b);
    });
    parts = std::move(next);
  }
  return parts.empty() ? std::vector<V>() : std::move(parts[0]);
}

// dictIds packed MSB-first at `bits` per value (FixedBitIntReaderWriter), chunks of 8-doc multiples in parallel
// (each chunk owns whole bytes)
void pack_ids(const std::vector<uint32_t> &ids, int bits, std::vector<uint8_t> &fwd, size_t T = 1) {
  const uint64_t n = ids.size();
  fwd.assign((size_t)((n * (uint64_t)bits + 7) / 8), 0);
  run_threads(T, [&](size_t t) {
    uint64_t lo, hi;
    chunk_of(n, T, t, 8, lo, hi);
    uint64_t acc = 0;  // pending bits, right-aligned
    int have = 0;
    size_t out = (size_t)(lo * (uint64_t)bits / 8);
    for (uint64_t i = lo; i < hi; i++) {
      acc = (acc << bits) | ids[i];
      have += bits;
      while (have >= 8) {
        have -= 8;
        fwd[out++] = (uint8_t)(acc >> have);
      }
      acc &= have ? ((1ull << have) - 1) : 0;
    }
    if (have) fwd[out] = (uint8_t)(acc << (8 - have));
  });
}

void finish_transcoded(const pinot_column_desc &d, TranscodedColumn &out) {
  out.desc.name = d.name;
  out.desc.data_type = d.data_type;
  out.desc.encoding = PINOT_ENCODING_DICTIONARY;
  out.desc.dictionary = out.dictionary.data();
  out.desc.dictionary_len = out.dictionary.size();
  out.desc.forward_index = out.forward_index.data();
  out.desc.forward_index_len = out.forward_index.size();
  out.desc.min_value = d.min_value;
  out.desc.max_value = d.max_value;
  out.desc.num_partitions = d.num_partitions;
  out.desc.partition_function = d.partition_function;
  out.desc.partition_values = d.partition_values;
  out.desc.num_partition_values = d.num_partition_values;
}

// A raw STRING column (VarByteChunkSingleValueReader.getString per doc, given flat: N + 1 BE offsets then bytes) as
// a dictionary column: the distinct values sorted in byte order (== code-point order, the order the dictionary
// predicate evaluators binary-search in), zero-padded to the longest; the raw-value evaluators' equals / compareTo
// on the values then give the same docs as the dictionary evaluators on the ids. A value holding a NUL byte would
// end at the padding: rejected.
bool transcode_raw_string(const pinot_column_desc &d, int32_t num_docs, TranscodedColumn &out, size_t T) {
  const std::string name = d.name ? d.name : "";
  const uint64_t n = (uint64_t)std::max(num_docs, 0);
  const uint64_t hdr = (n + 1) * 4;
  require(d.forward_index && d.forward_index_len >= hdr, PINOT_ERR_BAD_ARG,
          name + ": raw STRING forward index shorter than its numDocs + 1 offsets");
  const uint8_t *data = d.forward_index + hdr;
  const uint64_t data_len = d.forward_index_len - hdr;
  std::vector<std::string> vals(n);
  uint64_t prev = load_be32(d.forward_index);
  require(prev == 0, PINOT_ERR_BAD_ARG, name + ": raw STRING offsets must start at 0");
  for (uint64_t i = 0; i < n; i++) {
    const uint64_t e = load_be32(d.forward_index + 4 * (i + 1));
    require(e >= prev && e <= data_len, PINOT_ERR_BAD_ARG, name + ": raw STRING offsets not ascending within the bytes");
    vals[i].assign(reinterpret_cast<const char *>(data + prev), e - prev);
    require(vals[i].find('\0') == std::string::npos, PINOT_ERR_UNSUPPORTED,
            name + ": raw STRING value with a NUL byte (the dictionary's padding byte)");
    prev = e;
  }
  const std::vector<std::string> uniq = sorted_unique(vals, T);
  require(uniq.size() < (1ull << 31), PINOT_ERR_UNSUPPORTED, name + ": more than 2^31 distinct values");
  size_t width = 0;
  for (const auto &u : uniq) width = std::max(width, u.size());
  require(width < (size_t)INT32_MAX, PINOT_ERR_UNSUPPORTED, name + ": value too long");
  const int64_t card = (int64_t)uniq.size();
  out.dictionary.assign((size_t)card * width, 0);
  for (int64_t j = 0; j < card; j++) memcpy(out.dictionary.data() + (size_t)j * width, uniq[j].data(), uniq[j].size());
  std::vector<uint32_t> ids(n);
  run_threads(T, [&](size_t t) {
    uint64_t lo, hi;
    chunk_of(n, T, t, 1, lo, hi);
    for (uint64_t i = lo; i < hi; i++)
      ids[i] = (uint32_t)(std::lower_bound(uniq.begin(), uniq.end(), vals[i]) - uniq.begin());
  });
  const int bits = num_bits_per_value(std::max<int64_t>(card - 1, 0));
  pack_ids(ids, bits, out.forward_index, T);
  out.desc = pinot_column_desc{};
  out.desc.cardinality = (int32_t)card;
  out.desc.bits_per_value = bits;
  out.desc.string_width = (int32_t)width;
  out.desc.padding_byte = 0;
  finish_transcoded(d, out);
  return true;
}

}  // namespace

bool transcode_raw(const pinot_column_desc &d, int32_t num_docs, TranscodedColumn &out) {
  return transcode_raw_threads(d, num_docs, out, 0);
}

int raw_numeric_width(const pinot_column_desc &d, int32_t num_docs) {
  if (d.encoding == PINOT_ENCODING_DICTIONARY) return 0;
  const std::string name = d.name ? d.name : "";
  require(d.encoding == PINOT_ENCODING_RAW, PINOT_ERR_BAD_ARG, name + ": unknown column encoding");
  require(!d.multi_value, PINOT_ERR_UNSUPPORTED, name + ": raw multi-value columns are not served");
  require(!d.bloom_filter && !d.create_bloom_filter, PINOT_ERR_UNSUPPORTED,
          name + ": bloom filters are not supported for no-dictionary columns");  // BloomFilterHandler.java:117-118
  if (d.data_type == PINOT_STRING) return 0;
  require(d.data_type >= PINOT_INT && d.data_type <= PINOT_DOUBLE, PINOT_ERR_BAD_ARG, name + ": data type");
  const int w = (d.data_type == PINOT_INT || d.data_type == PINOT_FLOAT) ? 4 : 8;
  const uint64_t n = (uint64_t)std::max(num_docs, 0);
  require(d.forward_index && d.forward_index_len >= n * (uint64_t)w, PINOT_ERR_BAD_ARG,
          name + ": raw forward index shorter than numDocs values");
  return w;
}

void transcoded_numeric_finish(const pinot_column_desc &d, const uint64_t *uniq, int64_t card, TranscodedColumn &out) {
  const std::string name = d.name ? d.name : "";
  require(card < (1ll << 31), PINOT_ERR_UNSUPPORTED, name + ": more than 2^31 distinct values");
  const int w = (d.data_type == PINOT_INT || d.data_type == PINOT_FLOAT) ? 4 : 8;
  out.dictionary.resize((size_t)card * w);
  for (int64_t j = 0; j < card; j++) {  // invert the key back to the BE value bytes
    uint64_t k = uniq[j], v;
    switch (d.data_type) {
      case PINOT_INT: v = (k ^ 0x80000000ull) & 0xFFFFFFFFull; break;
      case PINOT_LONG: v = k ^ 0x8000000000000000ull; break;
      case PINOT_FLOAT: v = (k & 0x80000000ull) ? (k & 0x7FFFFFFFull) : (~k & 0xFFFFFFFFull); break;
      default: v = (k & 0x8000000000000000ull) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k; break;
    }
    for (int b = 0; b < w; b++) out.dictionary[(size_t)j * w + b] = (uint8_t)(v >> (8 * (w - 1 - b)));
  }
  out.desc = pinot_column_desc{};
  out.desc.cardinality = (int32_t)card;
  out.desc.bits_per_value = num_bits_per_value(std::max<int64_t>(card - 1, 0));
  finish_transcoded(d, out);
}

bool transcode_raw_threads(const pinot_column_desc &d, int32_t num_docs, TranscodedColumn &out, size_t threads) {
  if (d.encoding == PINOT_ENCODING_DICTIONARY) return false;
  const size_t T = transcode_threads((uint64_t)std::max(num_docs, 0), threads);
  const int w = raw_numeric_width(d, num_docs);
  if (d.data_type == PINOT_STRING) return transcode_raw_string(d, num_docs, out, T);
  const uint64_t n = (uint64_t)std::max(num_docs, 0);
  // sort keys: order-preserving u64 images of the values (sign flip for ints, IEEE total order for floats with
  // NaN canonicalised, as Double.compare orders them); transcode.hip's k_raw_keys forms the same keys
  auto key = [&](uint64_t i) -> uint64_t {
    const uint8_t *p = d.forward_index + i * w;
    uint64_t v = 0;
    for (int k = 0; k < w; k++) v = (v << 8) | p[k];
    switch (d.data_type) {
      case PINOT_INT: return (uint64_t)(uint32_t)v ^ 0x80000000ull;
      case PINOT_LONG: return v ^ 0x8000000000000000ull;
      case PINOT_FLOAT: {
        uint32_t b = (uint32_t)v;
        if ((b & 0x7F800000u) == 0x7F800000u && (b & 0x7FFFFFu)) b = 0x7FC00000u;  // floatToIntBits NaN
        return (b & 0x80000000u) ? (uint64_t)(~b) : (uint64_t)(b | 0x80000000u);
      }
      default: {
        if ((v & 0x7FF0000000000000ull) == 0x7FF0000000000000ull && (v & 0xFFFFFFFFFFFFFull)) v = 0x7FF8000000000000ull;
        return (v & 0x8000000000000000ull) ? ~v : (v | 0x8000000000000000ull);
      }
    }
  };
  std::vector<uint64_t> keys(n);
  run_threads(T, [&](size_t t) {
    uint64_t lo, hi;
    chunk_of(n, T, t, 1, lo, hi);
    for (uint64_t i = lo; i < hi; i++) keys[i] = key(i);
  });
  const std::vector<uint64_t> uniq = sorted_unique(keys, T);
  const int64_t card = (int64_t)uniq.size();
  require(card < (1ll << 31), PINOT_ERR_UNSUPPORTED, std::string(d.name ? d.name : "") + ": more than 2^31 distinct values");
  const int bits = num_bits_per_value(std::max<int64_t>(card - 1, 0));
  std::vector<uint32_t> ids(n);
  run_threads(T, [&](size_t t) {
    uint64_t lo, hi;
    chunk_of(n, T, t, 1, lo, hi);
    for (uint64_t i = lo; i < hi; i++)
      ids[i] = (uint32_t)(std::lower_bound(uniq.begin(), uniq.end(), keys[i]) - uniq.begin());
  });
  pack_ids(ids, bits, out.forward_index, T);
  transcoded_numeric_finish(d, uniq.data(), card, out);
  return true;
}

void validate_segment(const pinot_segment_desc &d) {
  require(d.num_docs >= 0, PINOT_ERR_BAD_ARG, "num_docs < 0");
  require(d.num_columns >= 0 && (d.num_columns == 0 || d.columns), PINOT_ERR_BAD_ARG, "columns");
  std::vector<std::string> names;
  for (int i = 0; i < d.num_columns; i++) {
    ColumnData c;
    ParsedIndexes idx;
    TranscodedColumn tc;
    parse_column(c, transcode_raw(d.columns[i], d.num_docs, tc) ? tc.desc : d.columns[i], d.num_docs, idx);
    for (const std::string &nm : names) require(nm != c.name, PINOT_ERR_BAD_ARG, "duplicate column " + c.name);
    names.push_back(c.name);
  }
}

}  // namespace pinot
