// Segment registration: Pinot column buffers (big-endian, as PinotDataBuffer holds them) -> HBM.
//
// Mirrors what ImmutableSegmentLoader.load + PhysicalColumnIndexContainer wire up per column
// (PC/indexsegment/immutable/ImmutableSegmentLoader.java:59-153,
//  PC/segment/index/column/PhysicalColumnIndexContainer.java:63-121):
//   sorted column   -> SortedIndexReaderImpl (2 BE ints per dictId, SortedIndexReaderImpl.java:34-39)
//   unsorted column -> FixedBitSingleValueReader over the packed stream (FixedBitSingleValueReader.java:36-51)
//   + optional BitmapInvertedIndexReader (offsets + portable roaring, BitmapInvertedIndexReader.java:92-119)
//   + dictionary (IntDictionary / LongDictionary / ... / StringDictionary)
// The packed forward index is uploaded byte-for-byte; sorted columns additionally get a packed
// forward index synthesised on the device so aggregation/group-by kernels see one layout.
#include <algorithm>
#include <atomic>
#include <cstring>

#include "engine.h"
#include "transcode.h"

namespace pinot {

uint64_t next_segment_uid() {
  static std::atomic<uint64_t> n{0};
  return ++n;
}

static void upload(DeviceBuffer &buf, const void *src, size_t bytes, size_t alloc_bytes, hipStream_t s) {
  buf.alloc(alloc_bytes);
  if (alloc_bytes > bytes) PINOT_HIP(hipMemsetAsync(buf.get<uint8_t>() + bytes, 0, alloc_bytes - bytes, s));
  if (bytes) PINOT_HIP(hipMemcpyAsync(buf.get(), src, bytes, hipMemcpyHostToDevice, s));
}

// Forward-index allocations are padded by one full 64-word staging chunk (64 * 8 * 32 B) plus a DMA
// piece, so the last chunk's global_load_lds pieces never leave the allocation.
static size_t padded(size_t bytes) { return ((bytes + 255) / 256) * 256 + 16384 + 1024; }

// Detects value(id) = base + step * id over the whole (sorted) INT/LONG dictionary.
static void detect_affine(ColumnData &c) {
  c.affine = false;
  if ((c.data_type != PINOT_INT && c.data_type != PINOT_LONG) || c.dict_int.empty()) return;
  const int64_t base = c.dict_int[0];
  const int64_t step = c.dict_int.size() > 1 ? c.dict_int[1] - c.dict_int[0] : 0;
  for (size_t i = 0; i < c.dict_int.size(); i++)
    if (c.dict_int[i] != base + step * (int64_t)i) return;
  c.affine = true;
  c.affine_base = base;
  c.affine_step = step;
}

static void upload_dictionary(Engine &e, ColumnData &c) {
  detect_affine(c);
  const int64_t card = c.card;
  if (c.data_type == PINOT_INT) {
    std::vector<int32_t> v(card);
    for (int64_t i = 0; i < card; i++) v[i] = static_cast<int32_t>(c.dict_int[i]);
    upload(c.dict_dev, v.data(), card * 4, std::max<size_t>(card * 4, 16), e.stream);
    PINOT_HIP(hipStreamSynchronize(e.stream));
  } else if (c.data_type == PINOT_LONG) {
    upload(c.dict_dev, c.dict_int.data(), card * 8, std::max<size_t>(card * 8, 16), e.stream);
  } else if (c.data_type == PINOT_FLOAT || c.data_type == PINOT_DOUBLE) {
    upload(c.dict_dev, c.dict_dbl.data(), card * 8, std::max<size_t>(card * 8, 16), e.stream);
  }
}

// A raw (no-dictionary) column as a dictionary column: numeric ones on the device (transcode.hip), STRING on the host;
// the bytes are the host path's either way (tests/test_gpu_raw.py compares them).
bool transcode_column(Engine &e, const pinot_column_desc &d, int32_t num_docs, TranscodedColumn &tc) {
  const int w = raw_numeric_width(d, num_docs);
  if (!w || !e.raw_device) return transcode_raw(d, num_docs, tc);
  {  // the device transcode's scratch (~n (w + 44) B) must leave room in HBM: else the host path (counted)
    const size_t need = transcode_numeric_device_bytes((uint64_t)std::max(num_docs, 0), w, e.stream);
    size_t free_b = 0, total_b = 0;
    PINOT_HIP(hipMemGetInfo(&free_b, &total_b));
    if ((double)need > 0.5 * (double)free_b) {
      e.raw_host_fallbacks++;
      return transcode_raw(d, num_docs, tc);
    }
  }
  std::vector<uint64_t> uniq;
  transcode_numeric_device(d.forward_index, (uint64_t)std::max(num_docs, 0), w, d.data_type, e.stream, uniq,
                           tc.forward_index);
  transcoded_numeric_finish(d, uniq.data(), (int64_t)uniq.size(), tc);
  e.raw_device_columns++;
  return true;
}

static void register_column(Engine &e, SegmentData &seg, const pinot_column_desc &d_in) {
  TranscodedColumn tc;
  const bool raw = transcode_column(e, d_in, seg.num_docs, tc);  // no-dictionary column: one-time transcoding
  const pinot_column_desc &d = raw ? tc.desc : d_in;
  auto cp = std::make_unique<ColumnData>();
  ColumnData &c = *cp;
  ParsedIndexes idx;
  parse_column(c, d, seg.num_docs, idx);  // every check on the caller's bytes (segment_parse.cpp)
  c.raw = raw;
  require(seg.by_name.find(c.name) == seg.by_name.end(), PINOT_ERR_BAD_ARG, "duplicate column " + c.name);
  upload_dictionary(e, c);
  if (c.is_sorted) {
    DeviceBuffer dstarts;
    upload(dstarts, idx.sorted_starts.data(), idx.sorted_starts.size() * 4, idx.sorted_starts.size() * 4, e.stream);
    c.fwd.alloc(padded(c.fwd_bytes));
    PINOT_HIP(hipMemsetAsync(c.fwd.get(), 0, c.fwd.size(), e.stream));
    launch_sorted_to_fwd(dstarts.get<int32_t>(), c.card, c.bits, (int32_t)seg.num_docs, c.fwd.get<uint8_t>(), e.stream);
    PINOT_HIP(hipGetLastError());
    PINOT_HIP(hipStreamSynchronize(e.stream));
  } else if (c.mv) {  // the packed entries, and the CSR row starts
    upload(c.fwd, c.fwd_bytes ? d.forward_index + c.mv_raw_offset : nullptr, c.fwd_bytes, padded(c.fwd_bytes), e.stream);
    upload(c.mv_offsets, c.mv_offsets_host.data(), c.mv_offsets_host.size() * 4, c.mv_offsets_host.size() * 4 + 16,
           e.stream);
    PINOT_HIP(hipStreamSynchronize(e.stream));
  } else {
    upload(c.fwd, d.forward_index, c.fwd_bytes, padded(c.fwd_bytes), e.stream);
  }
  if (!c.is_sorted && c.has_inverted) {
    const std::vector<RoaringContainer> &conts = idx.containers;
    c.inv_keys.resize(conts.size());
    for (size_t i = 0; i < conts.size(); i++) c.inv_keys[i] = conts[i].key;
    upload(c.inv_payload, d.inverted_index, d.inverted_index_len, padded(d.inverted_index_len), e.stream);
    upload(c.inv_containers, conts.data(), conts.size() * sizeof(RoaringContainer),
           std::max<size_t>(conts.size() * sizeof(RoaringContainer), 16), e.stream);
    upload(c.inv_dir_dev, c.inv_dir.data(), c.inv_dir.size() * 4, c.inv_dir.size() * 4, e.stream);
    PINOT_HIP(hipStreamSynchronize(e.stream));
  }
  seg.device_bytes += c.fwd.size() + c.dict_dev.size() + c.inv_payload.size() + c.inv_containers.size() +
                      c.inv_dir_dev.size() + c.mv_offsets.size();
  seg.by_name[c.name] = (int)seg.cols.size();
  seg.cols.push_back(std::move(cp));
}

std::unique_ptr<SegmentData> register_segment(Engine &e, const pinot_segment_desc &d) {
  require(d.num_docs >= 0, PINOT_ERR_BAD_ARG, "num_docs < 0");
  require(d.num_columns >= 0 && (d.num_columns == 0 || d.columns), PINOT_ERR_BAD_ARG, "columns");
  auto seg = std::make_unique<SegmentData>();
  seg->uid = next_segment_uid();
  seg->name = d.name ? d.name : "";
  seg->num_docs = d.num_docs;
  for (int i = 0; i < d.num_columns; i++) register_column(e, *seg, d.columns[i]);
  PINOT_HIP(hipStreamSynchronize(e.stream));
  return seg;
}

// ---------------------------------------------------------------- synthetic sorted / inverted columns
// Host-built Pinot-format buffers (the same bytes a segment file would hold), registered through the
// normal descriptor path: SORTED = value v on docs [v*N/card, (v+1)*N/card); INVERTED = the HBM
// generator's values (restated below) with a fixed-bit forward index and a bitmap inverted index
// (OffHeapBitmapInvertedIndexCreator layout: (card+1) BE int offsets + portable roaring, array / bitmap
// containers, no runs).
namespace {

uint64_t splitmix64_host(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void put_be32(std::vector<uint8_t> &b, size_t off, uint32_t v) {
  b[off] = (uint8_t)(v >> 24);
  b[off + 1] = (uint8_t)(v >> 16);
  b[off + 2] = (uint8_t)(v >> 8);
  b[off + 3] = (uint8_t)v;
}

void append_le16(std::vector<uint8_t> &b, uint32_t v) {
  b.push_back((uint8_t)v);
  b.push_back((uint8_t)(v >> 8));
}

void append_le32(std::vector<uint8_t> &b, uint32_t v) {
  append_le16(b, v & 0xFFFFu);
  append_le16(b, v >> 16);
}

// Portable roaring serialisation of ascending doc ids (cookie 12346: no run containers).
void serialize_roaring(const int32_t *docs, size_t n, std::vector<uint8_t> &out) {
  std::vector<std::pair<uint32_t, std::pair<size_t, size_t>>> conts;  // key, [begin, end)
  for (size_t i = 0; i < n;) {
    const uint32_t key = (uint32_t)docs[i] >> 16;
    size_t j = i;
    while (j < n && ((uint32_t)docs[j] >> 16) == key) j++;
    conts.push_back({key, {i, j}});
    i = j;
  }
  const size_t base = out.size();
  append_le32(out, 12346u);
  append_le32(out, (uint32_t)conts.size());
  for (auto &c : conts) {
    append_le16(out, c.first);
    append_le16(out, (uint32_t)(c.second.second - c.second.first - 1));
  }
  const size_t offs = out.size();
  out.resize(out.size() + 4 * conts.size());
  for (size_t k = 0; k < conts.size(); k++) {
    const uint32_t rel = (uint32_t)(out.size() - base);
    for (int q = 0; q < 4; q++) out[offs + 4 * k + q] = (uint8_t)(rel >> (8 * q));
    const size_t b = conts[k].second.first, e = conts[k].second.second;
    if (e - b > 4096) {
      uint64_t words[1024] = {0};
      for (size_t i = b; i < e; i++) {
        const uint32_t lo = (uint32_t)docs[i] & 0xFFFFu;
        words[lo >> 6] |= 1ull << (lo & 63);
      }
      for (int w = 0; w < 1024; w++) {
        append_le32(out, (uint32_t)words[w]);
        append_le32(out, (uint32_t)(words[w] >> 32));
      }
    } else {
      for (size_t i = b; i < e; i++) append_le16(out, (uint32_t)docs[i] & 0xFFFFu);
    }
  }
}

}  // namespace

std::unique_ptr<SegmentData> register_synthetic(Engine &e, const char *name, int32_t num_docs, int32_t ncols,
                                                const char *const *names, const int32_t *cards, uint64_t seed,
                                                const int32_t *kinds) {
  require(num_docs > 0 && ncols > 0 && names && cards, PINOT_ERR_BAD_ARG, "synthetic segment arguments");
  auto seg = std::make_unique<SegmentData>();
  seg->uid = next_segment_uid();
  seg->name = name ? name : "synthetic";
  seg->num_docs = num_docs;
  for (int i = 0; i < ncols; i++) {
    const int kind = kinds ? kinds[i] : PINOT_SYNTH_RANDOM;
    if (kind != PINOT_SYNTH_RANDOM) {
      require(kind == PINOT_SYNTH_SORTED || kind == PINOT_SYNTH_INVERTED, PINOT_ERR_BAD_ARG, "synthetic column kind");
      const int32_t card = cards[i];
      require(card >= 1 && card <= num_docs, PINOT_ERR_BAD_ARG, "synthetic cardinality must be in [1, num_docs]");
      const int bits = num_bits_per_value(card - 1);
      std::vector<uint8_t> dict((size_t)card * 4), sorted, fwd, inv;
      for (int32_t k = 0; k < card; k++) put_be32(dict, 4 * (size_t)k, (uint32_t)k);
      pinot_column_desc d{};
      d.name = names[i];
      d.data_type = PINOT_INT;
      d.cardinality = card;
      d.bits_per_value = bits;
      d.dictionary = dict.data();
      d.dictionary_len = dict.size();
      if (kind == PINOT_SYNTH_SORTED) {
        sorted.resize((size_t)card * 8);
        for (int32_t v = 0; v < card; v++) {
          put_be32(sorted, 8 * (size_t)v, (uint32_t)((int64_t)v * num_docs / card));
          put_be32(sorted, 8 * (size_t)v + 4, (uint32_t)((int64_t)(v + 1) * num_docs / card - 1));
        }
        d.is_sorted = 1;
        d.sorted_index = sorted.data();
        d.sorted_index_len = sorted.size();
      } else {
        const uint64_t cseed = seed ^ ((uint64_t)(i + 1) * 0xD1B54A32D192ED03ull);
        std::vector<int32_t> vals(num_docs);
        for (int64_t doc = 0; doc < num_docs; doc++)  // k_synth_column's value(d)
          vals[doc] = doc < card ? (int32_t)doc
                                 : (int32_t)(splitmix64_host(cseed ^ ((uint64_t)doc * 0x9E3779B97F4A7C15ull)) % (uint64_t)card);
        fwd.assign(((size_t)num_docs * bits + 7) / 8 + 8, 0);
        {  // PinotDataBitSet: MSB-first, big-endian, no padding between values
          uint64_t acc = 0;
          int nb = 0;
          size_t o = 0;
          for (int64_t doc = 0; doc < num_docs; doc++) {
            acc = (acc << bits) | (uint32_t)vals[doc];
            nb += bits;
            while (nb >= 8) {
              fwd[o++] = (uint8_t)(acc >> (nb - 8));
              nb -= 8;
            }
            acc &= (1ull << nb) - 1ull;
          }
          if (nb) fwd[o] = (uint8_t)(acc << (8 - nb));
        }
        // counting sort of docs by value -> ascending doc lists per dictId
        std::vector<int64_t> start((size_t)card + 1, 0);
        for (int32_t v : vals) start[v + 1]++;
        for (int32_t v = 0; v < card; v++) start[v + 1] += start[v];
        std::vector<int32_t> order(num_docs);
        {
          std::vector<int64_t> cur(start.begin(), start.end() - 1);
          for (int64_t doc = 0; doc < num_docs; doc++) order[cur[vals[doc]]++] = (int32_t)doc;
        }
        inv.assign(4 * ((size_t)card + 1), 0);
        inv.reserve(inv.size() + (size_t)num_docs * 2 + (size_t)card * 64 + ((size_t)num_docs >> 16) * card * 8);
        for (int32_t v = 0; v < card; v++) {
          put_be32(inv, 4 * (size_t)v, (uint32_t)inv.size());
          serialize_roaring(order.data() + start[v], (size_t)(start[v + 1] - start[v]), inv);
        }
        put_be32(inv, 4 * (size_t)card, (uint32_t)inv.size());
        require(inv.size() < UINT32_MAX, PINOT_ERR_UNSUPPORTED, "synthetic inverted index beyond 4 GiB");
        d.forward_index = fwd.data();
        d.forward_index_len = fwd.size();
        d.has_inverted_index = 1;
        d.inverted_index = inv.data();
        d.inverted_index_len = inv.size();
      }
      register_column(e, *seg, d);
      continue;
    }
    auto cp = std::make_unique<ColumnData>();
    ColumnData &c = *cp;
    c.name = names[i];
    c.data_type = PINOT_INT;
    c.card = cards[i];
    require(c.card >= 1 && c.card <= num_docs, PINOT_ERR_BAD_ARG, "synthetic cardinality must be in [1, num_docs]");
    c.bits = num_bits_per_value(c.card - 1);
    c.num_docs = num_docs;
    c.dict_int.resize(c.card);
    for (int32_t k = 0; k < c.card; k++) c.dict_int[k] = k;
    upload_dictionary(e, c);
    c.fwd_bytes = (uint64_t)(((int64_t)num_docs * c.bits + 7) / 8);
    c.fwd.alloc(padded(c.fwd_bytes));
    PINOT_HIP(hipMemsetAsync(c.fwd.get(), 0, c.fwd.size(), e.stream));
    const uint64_t cseed = seed ^ ((uint64_t)(i + 1) * 0xD1B54A32D192ED03ull);
    launch_synth_column(cseed, c.card, c.bits, num_docs, c.fwd.get<uint8_t>(), e.stream);
    PINOT_HIP(hipGetLastError());
    seg->device_bytes += c.fwd.size() + c.dict_dev.size();
    seg->by_name[c.name] = (int)seg->cols.size();
    seg->cols.push_back(std::move(cp));
  }
  PINOT_HIP(hipStreamSynchronize(e.stream));
  return seg;
}

void ensure_hll_lut(Engine &e, ColumnData &c) {
  if (c.hll_lut.size()) return;
  std::vector<uint16_t> lut(c.card);
  for (int32_t i = 0; i < c.card; i++) {
    uint32_t h;
    switch (c.data_type) {
      case PINOT_INT:
      case PINOT_LONG:
        h = murmur_hash_long(c.dict_int[i]);
        break;
      case PINOT_DOUBLE: {
        int64_t bits;
        memcpy(&bits, &c.dict_dbl[i], 8);
        h = murmur_hash_long(bits);  // hashLong(Double.doubleToRawLongBits)
        break;
      }
      case PINOT_FLOAT: {
        float f = static_cast<float>(c.dict_dbl[i]);
        int32_t bits;
        memcpy(&bits, &f, 4);
        h = murmur_hash_long(bits);  // hashLong(Float.floatToRawIntBits), sign-extended
        break;
      }
      default:
        h = murmur_hash_bytes(reinterpret_cast<const uint8_t *>(c.dict_str[i].data()), (int)c.dict_str[i].size());
    }
    lut[i] = hll_register_rank(h);
  }
  upload(c.hll_lut, lut.data(), lut.size() * 2, std::max<size_t>(lut.size() * 2, 16), e.stream);
  PINOT_HIP(hipStreamSynchronize(e.stream));
}

}  // namespace pinot
