// Pinot segment directories -> pinot_segment_desc (host only; registration then uploads what it describes).
//
// Restates the parts of the reference's loader this path needs (PC = pinot-core/src/main/java/org/apache/pinot/core):
//   layout         SegmentDirectoryPaths.findSegmentDirectory: <indexDir>/v3 when it exists, else <indexDir>
//                  (PC/segment/store/SegmentDirectoryPaths.java:41-56)
//   metadata       metadata.properties, Apache Commons PropertiesConfiguration syntax; SegmentMetadataImpl.init /
//                  ColumnMetadata.fromPropertiesConfiguration (PC/segment/index/SegmentMetadataImpl.java:219-260,
//                  PC/segment/index/ColumnMetadata.java:87-116); keys from V1Constants (PC/segment/creator/impl/
//                  V1Constants.java:54-146)
//   v1 / v2        FilePerIndexDirectory: <col>.dict, <col>.sv.unsorted.fwd | <col>.sv.sorted.fwd, <col>.bitmap.inv
//                  (PC/segment/store/FilePerIndexDirectory.java:148-168, SegmentMetadataImpl.java:498-527)
//   v3             SingleFileIndexDirectory: columns.psf + index_map ("<col>.<index>.startOffset|size = n"); each
//                  entry starts with the 8-byte magic 0xdeadbeefdeafbead, counted in its size
//                  (PC/segment/store/SingleFileIndexDirectory.java:62-320)
// Files are memory-mapped read-only. Columns this executor does not serve (multi-value, raw / no-dictionary,
// BYTES) are skipped and named by pinot_gpu_segment_dir_info; queries naming them fail as unknown columns. Raw
// (no-dictionary) INT / LONG / FLOAT / DOUBLE columns are read from their chunked .sv.raw.fwd index.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <map>
#include <set>

#include "engine.h"

namespace pinot {

namespace {

constexpr uint64_t kV3Magic = 0xdeadbeefdeafbeadull;

bool is_dir(const std::string &p) {
  struct stat st;
  return stat(p.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}
bool is_file(const std::string &p) {
  struct stat st;
  return stat(p.c_str(), &st) == 0 && S_ISREG(st.st_mode);
}

std::string read_text(const std::string &path) {
  const int fd = open(path.c_str(), O_RDONLY);
  require(fd >= 0, PINOT_ERR_BAD_ARG, "cannot open " + path);
  std::string out;
  char buf[65536];
  for (;;) {
    const ssize_t n = read(fd, buf, sizeof(buf));
    if (n <= 0) break;
    out.append(buf, (size_t)n);
  }
  close(fd);
  return out;
}

// Commons-Configuration-1.x properties: '#'/'!' comments, key and value split at the first unescaped '=', ':'
// or whitespace, trailing-backslash continuation, Java escapes (\\, \t, \n, \r, \f, \uXXXX) in keys and values.
std::string unescape_properties(const std::string &s) {
  std::string o;
  for (size_t i = 0; i < s.size(); i++) {
    if (s[i] != '\\' || i + 1 == s.size()) {
      o += s[i];
      continue;
    }
    const char c = s[++i];
    switch (c) {
      case 't': o += '\t'; break;
      case 'n': o += '\n'; break;
      case 'r': o += '\r'; break;
      case 'f': o += '\f'; break;
      case 'u': {
        require(i + 4 < s.size(), PINOT_ERR_BAD_ARG, "metadata.properties: bad \\u escape");
        const unsigned long cp = strtoul(s.substr(i + 1, 4).c_str(), nullptr, 16);
        i += 4;
        if (cp < 0x80) {
          o += (char)cp;
        } else if (cp < 0x800) {
          o += (char)(0xC0 | (cp >> 6));
          o += (char)(0x80 | (cp & 0x3F));
        } else {
          o += (char)(0xE0 | (cp >> 12));
          o += (char)(0x80 | ((cp >> 6) & 0x3F));
          o += (char)(0x80 | (cp & 0x3F));
        }
        break;
      }
      default: o += c;  // \\ \= \: \, \# and any other char stand for themselves
    }
  }
  return o;
}

std::string trim(const std::string &s) {
  size_t a = 0, b = s.size();
  while (a < b && (s[a] == ' ' || s[a] == '\t' || s[a] == '\f')) a++;
  while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t' || s[b - 1] == '\f' || s[b - 1] == '\r')) b--;
  return s.substr(a, b - a);
}

std::map<std::string, std::string> parse_properties(const std::string &text) {
  std::map<std::string, std::string> kv;
  std::vector<std::string> lines;
  std::string cur;  // a line ending in an odd number of backslashes continues on the next (leading blanks dropped)
  size_t i = 0;
  while (i < text.size()) {
    const size_t e = std::min(text.find('\n', i), text.size());
    std::string line = text.substr(i, e - i);
    i = e + 1;
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (!cur.empty()) line = trim(line);
    size_t nbs = 0;
    while (nbs < line.size() && line[line.size() - 1 - nbs] == '\\') nbs++;
    if (nbs % 2 == 1) {
      cur += line.substr(0, line.size() - 1);
      continue;
    }
    lines.push_back(cur + line);
    cur.clear();
  }
  if (!cur.empty()) lines.push_back(cur);
  for (const std::string &raw : lines) {
    const std::string line = trim(raw);
    if (line.empty() || line[0] == '#' || line[0] == '!') continue;
    size_t sep = std::string::npos;
    for (size_t i = 0; i < line.size(); i++) {
      if (line[i] == '\\') {
        i++;
        continue;
      }
      if (line[i] == '=' || line[i] == ':' || line[i] == ' ' || line[i] == '\t') {
        sep = i;
        break;
      }
    }
    std::string key = sep == std::string::npos ? line : line.substr(0, sep);
    std::string value = sep == std::string::npos ? "" : trim(line.substr(sep + 1));
    if (sep != std::string::npos && (line[sep] == ' ' || line[sep] == '\t') && !value.empty() &&
        (value[0] == '=' || value[0] == ':'))
      value = trim(value.substr(1));
    kv[unescape_properties(trim(key))] = value;  // values unescaped per use (lists split on unescaped ',')
  }
  return kv;
}

// getList: split on unescaped ',' (Commons list delimiter), each element trimmed and unescaped; empty -> none
std::vector<std::string> prop_list(const std::map<std::string, std::string> &kv, const std::string &key) {
  std::vector<std::string> out;
  auto it = kv.find(key);
  if (it == kv.end()) return out;
  const std::string &v = it->second;
  std::string cur;
  for (size_t i = 0; i <= v.size(); i++) {
    if (i == v.size() || v[i] == ',') {
      const std::string t = trim(unescape_properties(cur));
      if (!t.empty()) out.push_back(t);
      cur.clear();
    } else {
      if (v[i] == '\\' && i + 1 < v.size()) cur += v[i++];
      cur += v[i];
    }
  }
  return out;
}

std::string prop(const std::map<std::string, std::string> &kv, const std::string &key, const char *dflt = nullptr) {
  auto it = kv.find(key);
  if (it == kv.end()) {
    require(dflt != nullptr, PINOT_ERR_BAD_ARG, "metadata.properties: missing " + key);
    return dflt;
  }
  return unescape_properties(it->second);
}

int64_t prop_int(const std::map<std::string, std::string> &kv, const std::string &key, const char *dflt = nullptr) {
  const std::string v = prop(kv, key, dflt);
  char *end = nullptr;
  errno = 0;
  const long long x = strtoll(v.c_str(), &end, 10);
  require(errno == 0 && end && *end == 0 && !v.empty(), PINOT_ERR_BAD_ARG, "metadata.properties: " + key + " = " + v);
  return x;
}

bool prop_bool(const std::map<std::string, std::string> &kv, const std::string &key, bool dflt) {
  auto it = kv.find(key);
  if (it == kv.end()) return dflt;
  std::string v = trim(unescape_properties(it->second));
  std::transform(v.begin(), v.end(), v.begin(), ::tolower);
  return v == "true" || v == "on" || v == "yes";
}

int data_type_of(std::string t) {
  std::transform(t.begin(), t.end(), t.begin(), ::toupper);
  if (t == "INT") return PINOT_INT;
  if (t == "LONG") return PINOT_LONG;
  if (t == "FLOAT") return PINOT_FLOAT;
  if (t == "DOUBLE") return PINOT_DOUBLE;
  if (t == "STRING") return PINOT_STRING;
  return -1;  // BYTES, BOOLEAN, ...: not served here
}

}  // namespace

MappedFile::MappedFile(const std::string &path) {
  const int fd = open(path.c_str(), O_RDONLY);
  require(fd >= 0, PINOT_ERR_BAD_ARG, "cannot open " + path);
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    throw Error(PINOT_ERR_BAD_ARG, "cannot stat " + path);
  }
  size = (size_t)st.st_size;
  if (size) {
    void *m = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) {
      close(fd);
      throw Error(PINOT_ERR_BAD_ARG, "cannot map " + path);
    }
    data = static_cast<const uint8_t *>(m);
  }
  close(fd);
}

MappedFile::~MappedFile() {
  if (data) munmap(const_cast<uint8_t *>(data), size);
}

// Raw Snappy block (no framing), as org.xerial.snappy.Snappy.uncompress reads it: varint32 length, then literal
// (tag & 3 == 0) and back-reference copy elements (1, 2 or 4 offset bytes).
void snappy_uncompress(const uint8_t *p, uint64_t n, std::vector<uint8_t> &out, const std::string &what) {
  uint64_t i = 0, len = 0;
  for (int shift = 0;; shift += 7) {
    require(i < n && shift <= 28, PINOT_ERR_BAD_ARG, what + ": bad Snappy length");
    const uint8_t b = p[i++];
    len |= (uint64_t)(b & 0x7F) << shift;
    if (!(b & 0x80)) break;
  }
  const size_t base = out.size();
  out.reserve(base + len);
  while (i < n) {
    const uint8_t tag = p[i++];
    uint64_t l, off = 0;
    switch (tag & 3) {
      case 0: {
        l = (uint64_t)(tag >> 2) + 1;
        if (l > 60) {
          const int nb = (int)l - 60;
          require(i + nb <= n, PINOT_ERR_BAD_ARG, what + ": truncated Snappy literal");
          l = 0;
          for (int k = 0; k < nb; k++) l |= (uint64_t)p[i + k] << (8 * k);
          l += 1;
          i += nb;
        }
        require(l <= n - i && out.size() - base + l <= len, PINOT_ERR_BAD_ARG, what + ": Snappy literal overruns");
        out.insert(out.end(), p + i, p + i + l);
        i += l;
        continue;
      }
      case 1:
        require(i < n, PINOT_ERR_BAD_ARG, what + ": truncated Snappy copy");
        l = 4 + ((tag >> 2) & 7);
        off = ((uint64_t)(tag >> 5) << 8) | p[i++];
        break;
      case 2:
        require(i + 2 <= n, PINOT_ERR_BAD_ARG, what + ": truncated Snappy copy");
        l = 1 + (tag >> 2);
        off = (uint64_t)p[i] | ((uint64_t)p[i + 1] << 8);
        i += 2;
        break;
      default:
        require(i + 4 <= n, PINOT_ERR_BAD_ARG, what + ": truncated Snappy copy");
        l = 1 + (tag >> 2);
        off = (uint64_t)p[i] | ((uint64_t)p[i + 1] << 8) | ((uint64_t)p[i + 2] << 16) | ((uint64_t)p[i + 3] << 24);
        i += 4;
        break;
    }
    const uint64_t have = out.size() - base;
    require(off >= 1 && off <= have && have + l <= len, PINOT_ERR_BAD_ARG, what + ": bad Snappy copy");
    for (uint64_t k = 0; k < l; k++) out.push_back(out[out.size() - off]);  // overlapping copies repeat bytes
  }
  require(out.size() - base == len, PINOT_ERR_BAD_ARG, what + ": Snappy length mismatch");
}

// FixedByteChunkSingleValueReader (PC/io/reader/impl/v1/BaseChunkSingleValueReader.java:57-96, :120-147): header
// ints version, numChunks, numDocsPerChunk, lengthOfLongestEntry [, v2+: totalDocs, compressionType, dataHeaderStart],
// then numChunks absolute chunk offsets; chunks PASS_THROUGH (0) or SNAPPY (1; version 1 is always Snappy).
// Returns the docs' values back to back, big-endian, entry_size bytes each.
std::vector<uint8_t> read_raw_chunks(const uint8_t *b, uint64_t n, int64_t num_docs, int entry_size,
                                     const std::string &what) {
  auto be32 = [&](uint64_t off) -> int64_t {
    require(off + 4 <= n, PINOT_ERR_BAD_ARG, what + ": raw forward index header truncated");
    return (int32_t)(((uint32_t)b[off] << 24) | ((uint32_t)b[off + 1] << 16) | ((uint32_t)b[off + 2] << 8) | b[off + 3]);
  };
  const int64_t version = be32(0), num_chunks = be32(4), per_chunk = be32(8), longest = be32(12);
  require(version >= 1 && version <= 2, PINOT_ERR_UNSUPPORTED, what + ": raw forward index version");
  require(longest == entry_size, PINOT_ERR_BAD_ARG, what + ": raw entry size differs from the data type's");
  require(num_chunks >= 0 && per_chunk >= 1 && num_chunks * per_chunk >= num_docs, PINOT_ERR_BAD_ARG,
          what + ": raw chunk layout does not cover the docs");
  int64_t compression = 1, header_start = 16;
  if (version > 1) {
    compression = be32(20);
    header_start = be32(24);
  }
  require(compression == 0 || compression == 1, PINOT_ERR_UNSUPPORTED, what + ": chunk compression type");
  std::vector<uint8_t> values;
  values.reserve((size_t)num_docs * entry_size);
  for (int64_t c = 0; c < num_chunks; c++) {
    const int64_t start = be32((uint64_t)header_start + 4 * c);
    const int64_t end = c + 1 < num_chunks ? be32((uint64_t)header_start + 4 * (c + 1)) : (int64_t)n;
    require(start >= header_start + 4 * num_chunks && start <= end && (uint64_t)end <= n, PINOT_ERR_BAD_ARG,
            what + ": chunk offsets");
    if (compression == 0) values.insert(values.end(), b + start, b + end);
    else snappy_uncompress(b + start, (uint64_t)(end - start), values, what);
  }
  require(values.size() >= (size_t)num_docs * entry_size, PINOT_ERR_BAD_ARG, what + ": raw chunks hold too few docs");
  values.resize((size_t)num_docs * entry_size);
  return values;
}

// VarByteChunkSingleValueWriter file (header as read_raw_chunks; each chunk, decompressed, = numDocsPerChunk int
// offsets from the chunk start, then the values' bytes): per doc the bytes VarByteChunkSingleValueReader.getBytes
// returns (VarByteChunkSingleValueReader.java:58-115: length = next offset - offset; the chunk's end for its last
// row or when the next offset is 0, the filler of a partial chunk), flattened as the C-ABI's raw STRING form:
// numDocs + 1 BE offsets, then the bytes.
std::vector<uint8_t> read_var_byte_chunks(const uint8_t *b, uint64_t n, int64_t num_docs, const std::string &what) {
  auto be32 = [&](const uint8_t *p, uint64_t len, uint64_t off) -> int64_t {
    require(off + 4 <= len, PINOT_ERR_BAD_ARG, what + ": var-byte chunk truncated");
    return (int32_t)(((uint32_t)p[off] << 24) | ((uint32_t)p[off + 1] << 16) | ((uint32_t)p[off + 2] << 8) | p[off + 3]);
  };
  const int64_t version = be32(b, n, 0), num_chunks = be32(b, n, 4), per_chunk = be32(b, n, 8);
  require(version >= 1 && version <= 2, PINOT_ERR_UNSUPPORTED, what + ": raw forward index version");
  require(num_chunks >= 0 && per_chunk >= 1 && num_chunks * per_chunk >= num_docs && per_chunk < (1 << 26),
          PINOT_ERR_BAD_ARG, what + ": var-byte chunk layout does not cover the docs");
  int64_t compression = 1, header_start = 16;
  if (version > 1) {
    compression = be32(b, n, 20);
    header_start = be32(b, n, 24);
  }
  require(compression == 0 || compression == 1, PINOT_ERR_UNSUPPORTED, what + ": chunk compression type");
  std::vector<uint8_t> offs((size_t)(num_docs + 1) * 4), bytes;
  auto put_be32 = [&](int64_t i, uint64_t v) {
    require(v < (1ull << 31), PINOT_ERR_UNSUPPORTED, what + ": raw STRING column over 2 GB");
    for (int k = 0; k < 4; k++) offs[(size_t)i * 4 + k] = (uint8_t)(v >> (24 - 8 * k));
  };
  put_be32(0, 0);
  int64_t doc = 0;
  std::vector<uint8_t> chunk;
  for (int64_t c = 0; c < num_chunks && doc < num_docs; c++) {
    const int64_t start = be32(b, n, (uint64_t)header_start + 4 * c);
    const int64_t end = c + 1 < num_chunks ? be32(b, n, (uint64_t)header_start + 4 * (c + 1)) : (int64_t)n;
    require(start >= header_start + 4 * num_chunks && start <= end && (uint64_t)end <= n, PINOT_ERR_BAD_ARG,
            what + ": chunk offsets");
    chunk.clear();
    if (compression == 0) chunk.assign(b + start, b + end);
    else snappy_uncompress(b + start, (uint64_t)(end - start), chunk, what);
    const uint64_t limit = chunk.size();
    require(limit >= (uint64_t)per_chunk * 4, PINOT_ERR_BAD_ARG, what + ": var-byte chunk shorter than its offsets");
    for (int64_t r = 0; r < per_chunk && doc < num_docs; r++, doc++) {
      const int64_t o = be32(chunk.data(), limit, 4 * (uint64_t)r);
      int64_t e = (int64_t)limit;
      if (r + 1 < per_chunk) {
        e = be32(chunk.data(), limit, 4 * (uint64_t)(r + 1));
        if (e == 0) e = (int64_t)limit;
      }
      require(o >= per_chunk * 4 && o <= e && (uint64_t)e <= limit, PINOT_ERR_BAD_ARG, what + ": var-byte row offsets");
      bytes.insert(bytes.end(), chunk.begin() + o, chunk.begin() + e);
      put_be32(doc + 1, bytes.size());
    }
  }
  require(doc == num_docs, PINOT_ERR_BAD_ARG, what + ": var-byte chunks hold too few docs");
  offs.insert(offs.end(), bytes.begin(), bytes.end());
  return offs;
}

bool read_segment_identity(const std::string &index_dir, std::string &name, int64_t &crc) {
  require(is_dir(index_dir), PINOT_ERR_BAD_ARG, "not a segment directory: " + index_dir);
  const std::string v3 = index_dir + "/v3";
  const std::string dir = is_dir(v3) ? v3 : index_dir;
  const std::string meta_path = is_file(dir + "/metadata.properties") ? dir + "/metadata.properties"
                                                                      : index_dir + "/metadata.properties";
  const auto kv = parse_properties(read_text(meta_path));
  name = prop(kv, "segment.name", "");
  // SegmentDirectoryPaths.findCreationMetaFile: v3/creation.meta, else the index directory's
  std::string cm = dir + "/creation.meta";
  if (!is_file(cm)) cm = index_dir + "/creation.meta";
  if (!is_file(cm)) return false;
  MappedFile f(cm);
  require(f.size >= 8, PINOT_ERR_BAD_ARG, "creation.meta shorter than its CRC");
  uint64_t v = 0;
  for (int k = 0; k < 8; k++) v = (v << 8) | f.data[k];  // DataInputStream.readLong (big-endian)
  crc = (int64_t)v;
  return true;
}

void read_star_tree(const std::string &dir, const std::map<std::string, std::string> &kv, SegmentDirData &out);

void read_segment_dir(const std::string &index_dir, SegmentDirData &out) {
  require(is_dir(index_dir), PINOT_ERR_BAD_ARG, "not a segment directory: " + index_dir);
  const std::string v3 = index_dir + "/v3";
  const std::string dir = is_dir(v3) ? v3 : index_dir;
  const std::string meta_path = is_file(dir + "/metadata.properties") ? dir + "/metadata.properties"
                                                                      : index_dir + "/metadata.properties";
  const auto kv = parse_properties(read_text(meta_path));
  const std::string version = prop(kv, "segment.index.version", "v1");
  const bool single_file = version == "v3";
  require(version == "v1" || version == "v2" || version == "v3", PINOT_ERR_UNSUPPORTED, "segment version " + version);
  require(!single_file || dir == v3, PINOT_ERR_BAD_ARG, "v3 segment without a v3/ directory: " + index_dir);
  out.name = prop(kv, "segment.name", "");
  out.time_column = prop(kv, "segment.time.column.name", "");
  const int64_t total = prop_int(kv, "segment.total.docs", nullptr);
  require(total >= 0 && total < INT32_MAX, PINOT_ERR_BAD_ARG, "segment.total.docs out of range");
  out.num_docs = (int32_t)total;
  // padding: segment key, else the legacy '%' (ColumnMetadata.java:111-115)
  int pad = '%';
  if (kv.count("segment.padding.character")) {
    const std::string p = unescape_properties(prop(kv, "segment.padding.character"));  // unescapeJava of the value
    require(!p.empty(), PINOT_ERR_BAD_ARG, "empty segment.padding.character");
    pad = (uint8_t)p[0];
  }

  // physical columns in the order SegmentMetadataImpl adds them (dimensions, metrics, time, date-time)
  std::vector<std::string> names;
  std::set<std::string> seen;
  for (const char *key : {"segment.dimension.column.names", "segment.metric.column.names", "segment.time.column.name",
                          "segment.datetime.column.names"})
    for (const std::string &c : prop_list(kv, key))
      if (seen.insert(c).second) names.push_back(c);

  // v3: index_map entries -> (offset, size) of each (column, index) inside columns.psf
  std::map<std::string, std::pair<uint64_t, uint64_t>> entries;
  const MappedFile *psf = nullptr;
  if (single_file) {
    const auto im = parse_properties(read_text(dir + "/index_map"));
    std::map<std::string, std::pair<int64_t, int64_t>> raw;
    for (const auto &e : im) {
      const size_t last = e.first.rfind('.');
      require(last != std::string::npos && last > 0, PINOT_ERR_BAD_ARG, "index_map key " + e.first);
      const std::string what = e.first.substr(last + 1), idx = e.first.substr(0, last);
      auto &slot = raw.emplace(idx, std::make_pair((int64_t)-1, (int64_t)-1)).first->second;
      const int64_t v = prop_int(im, e.first);
      if (what == "startOffset") slot.first = v;
      else if (what == "size") slot.second = v;
      else throw Error(PINOT_ERR_BAD_ARG, "index_map key " + e.first);
    }
    out.files.emplace_back(new MappedFile(dir + "/columns.psf"));
    psf = out.files.back().get();
    for (const auto &r : raw) {
      const int64_t off = r.second.first, size = r.second.second;
      require(off >= 0 && size >= 8 && (uint64_t)off <= psf->size && (uint64_t)size <= psf->size - (uint64_t)off,
              PINOT_ERR_BAD_ARG, "index_map entry " + r.first + " outside columns.psf");
      uint64_t magic = 0;
      for (int i = 0; i < 8; i++) magic = (magic << 8) | psf->data[off + i];
      require(magic == kV3Magic, PINOT_ERR_BAD_ARG, "columns.psf: missing magic marker for " + r.first);
      entries[r.first] = {(uint64_t)off + 8, (uint64_t)size - 8};
    }
  }
  auto index_bytes = [&](const std::string &col, const char *index, const std::string &v1_file, const uint8_t **p,
                         uint64_t *n) -> bool {
    if (single_file) {
      auto it = entries.find(col + "." + index);
      if (it == entries.end()) return false;
      *p = psf->data + it->second.first;
      *n = it->second.second;
      return true;
    }
    const std::string path = dir + "/" + v1_file;
    if (!is_file(path)) return false;
    out.files.emplace_back(new MappedFile(path));
    *p = out.files.back()->data;
    *n = out.files.back()->size;
    return true;
  };

  out.column_names.reserve(names.size());
  for (const std::string &c : names) {
    const std::string k = "column." + c + ".";
    const int dt = data_type_of(prop(kv, k + "dataType"));
    const bool single = prop_bool(kv, k + "isSingleValues", true), dict = prop_bool(kv, k + "hasDictionary", true);
    if (dt < 0 || (!single && !dict)) {
      out.skipped.push_back(c);
      continue;
    }
    out.column_names.push_back(c);
    pinot_column_desc d{};
    d.data_type = dt;
    if (kv.count(k + "minValue") && kv.count(k + "maxValue")) {  // ColumnMetadata.java:155-156
      out.strings.push_back(unescape_properties(prop(kv, k + "minValue")));
      d.min_value = out.strings.back().c_str();
      out.strings.push_back(unescape_properties(prop(kv, k + "maxValue")));
      d.max_value = out.strings.back().c_str();
    }
    if (kv.count(k + "partitionFunction")) {  // ColumnMetadata.java:184-194
      out.strings.push_back(prop(kv, k + "partitionFunction"));
      d.partition_function = out.strings.back().c_str();
      const int64_t np = prop_int(kv, k + "numPartitions");
      require(np > 0 && np < INT32_MAX, PINOT_ERR_BAD_ARG, c + ": numPartitions out of range");
      d.num_partitions = (int32_t)np;
      std::vector<int32_t> parts;  // ColumnPartitionMetadata.extractPartitions: "n" or "[start end]" ranges
      for (const std::string &pv : prop_list(kv, k + "partitionValues")) {
        require(!pv.empty(), PINOT_ERR_BAD_ARG, c + ": empty partition value");
        if (pv[0] == '[') {
          const size_t sp = pv.find(' ');
          require(sp != std::string::npos && pv.back() == ']', PINOT_ERR_BAD_ARG, c + ": partition range " + pv);
          const int64_t a = java_parse_integer(pv.substr(1, sp - 1), INT32_MIN, INT32_MAX);
          const int64_t b = java_parse_integer(pv.substr(sp + 1, pv.size() - sp - 2), INT32_MIN, INT32_MAX);
          require(b - a < (int64_t)1 << 20, PINOT_ERR_BAD_ARG, c + ": partition range too wide " + pv);
          for (int64_t x = a; x <= b; x++) parts.push_back((int32_t)x);
        } else {
          parts.push_back((int32_t)java_parse_integer(pv, INT32_MIN, INT32_MAX));
        }
      }
      out.ints.push_back(std::move(parts));
      d.partition_values = out.ints.back().data();
      d.num_partition_values = (int32_t)out.ints.back().size();
    }
    if (!dict) {  // a raw (no-dictionary) fixed-width column: decompressed here, transcoded at registration
      const uint8_t *fp = nullptr;
      uint64_t fn = 0;
      require(index_bytes(c, "forward_index", c + ".sv.raw.fwd", &fp, &fn), PINOT_ERR_BAD_ARG,
              c + ": no raw forward index");
      if (dt == PINOT_STRING) {
        out.owned.push_back(read_var_byte_chunks(fp, fn, out.num_docs, c));
      } else {
        const int w = (dt == PINOT_INT || dt == PINOT_FLOAT) ? 4 : 8;
        out.owned.push_back(read_raw_chunks(fp, fn, out.num_docs, w, c));
      }
      d.encoding = PINOT_ENCODING_RAW;
      d.forward_index = out.owned.back().data();
      d.forward_index_len = out.owned.back().size();
      out.cols.push_back(d);
      continue;
    }
    const int64_t card = prop_int(kv, k + "cardinality"), bits = prop_int(kv, k + "bitsPerElement");
    const int64_t width = prop_int(kv, k + "lengthOfEachEntry", "0");
    require(card >= 0 && card < INT32_MAX && bits >= 0 && bits <= 64 && width >= 0 && width < INT32_MAX,
            PINOT_ERR_BAD_ARG, c + ": column metadata out of range");
    d.cardinality = (int32_t)card;
    d.bits_per_value = (int32_t)bits;
    d.string_width = (int32_t)width;
    d.padding_byte = dt == PINOT_STRING ? pad : 0;
    d.is_sorted = prop_bool(kv, k + "isSorted", false) ? 1 : 0;
    require(index_bytes(c, "dictionary", c + ".dict", &d.dictionary, &d.dictionary_len), PINOT_ERR_BAD_ARG,
            c + ": no dictionary");
    // a bloom filter the loader built (BloomFilterHandler; v1 <col>.bloom, v3 index type bloom_filter)
    index_bytes(c, "bloom_filter", c + ".bloom", &d.bloom_filter, &d.bloom_filter_len);
    const uint8_t *fp = nullptr;
    uint64_t fn = 0;
    if (!single) {  // FixedBitMultiValueWriter file (<col>.mv.fwd, V1Constants.java:61)
      d.multi_value = 1;
      d.is_sorted = 0;
      const int64_t entries = prop_int(kv, k + "totalNumberOfEntries");
      const int64_t maxmv = prop_int(kv, k + "maxNumberOfMultiValues", "0");
      require(entries >= 0 && maxmv >= 0 && maxmv < INT32_MAX, PINOT_ERR_BAD_ARG, c + ": multi-value metadata out of range");
      d.total_number_of_entries = entries;
      d.max_number_of_multi_values = (int32_t)maxmv;
    }
    require(index_bytes(c, "forward_index",
                        c + (!single ? ".mv.fwd" : d.is_sorted ? ".sv.sorted.fwd" : ".sv.unsorted.fwd"), &fp, &fn),
            PINOT_ERR_BAD_ARG, c + ": no forward index");
    if (d.is_sorted) {
      d.sorted_index = fp;
      d.sorted_index_len = fn;
    } else {
      d.forward_index = fp;
      d.forward_index_len = fn;
      // the bitmap index is used when the segment holds one (hasInvertedIndex with no file: none was built)
      if (prop_bool(kv, k + "hasInvertedIndex", false) &&
          index_bytes(c, "inverted_index", c + ".bitmap.inv", &d.inverted_index, &d.inverted_index_len))
        d.has_inverted_index = 1;
    }
    out.cols.push_back(d);
  }
  for (size_t i = 0; i < out.cols.size(); i++) out.cols[i].name = out.column_names[i].c_str();
  read_star_tree(dir, kv, out);
}

// Star-tree v2 files (StarTreeLoaderUtils.java:60-110, StarTreeIndexMapUtils.java): star_tree_index (the combined
// tree + forward indexes) located by star_tree_index_map ("<tree>.<column>.<STAR_TREE|FORWARD_INDEX>.<OFFSET|SIZE>",
// the tree's column "null"), described by metadata.properties' startree.v2.* keys (StarTreeV2Metadata: total.docs,
// split.order, function.column.pairs). Dimension forward indexes are fixed-bit at the segment column's bits;
// the pair columns are FixedByteChunk raw indexes (LONG for count, DOUBLE otherwise). Only the first tree is read.
void read_star_tree(const std::string &dir, const std::map<std::string, std::string> &kv, SegmentDirData &out) {
  if (!kv.count("startree.v2.count") || prop_int(kv, "startree.v2.count") < 1) return;
  const std::string pre = "startree.v2.0.";
  const int64_t ndocs = prop_int(kv, pre + "total.docs");
  require(ndocs >= 1 && ndocs < INT32_MAX, PINOT_ERR_BAD_ARG, "star-tree total.docs out of range");
  const std::string idx_path = dir + "/star_tree_index", map_path = dir + "/star_tree_index_map";
  require(is_file(idx_path) && is_file(map_path), PINOT_ERR_BAD_ARG, "star-tree index files missing in " + dir);
  out.files.emplace_back(new MappedFile(idx_path));
  const MappedFile &f = *out.files.back();
  const auto imap = parse_properties(read_text(map_path));
  auto range = [&](const std::string &col, const std::string &type, const uint8_t **p, uint64_t *n) {
    const std::string k = "0." + col + "." + type + ".";
    require(imap.count(k + "OFFSET") && imap.count(k + "SIZE"), PINOT_ERR_BAD_ARG, "star-tree index map lacks " + k);
    const int64_t o = prop_int(imap, k + "OFFSET"), sz = prop_int(imap, k + "SIZE");
    require(o >= 0 && sz >= 0 && (uint64_t)(o + sz) <= f.size, PINOT_ERR_BAD_ARG, "star-tree " + k + " outside star_tree_index");
    *p = f.data + o;
    *n = (uint64_t)sz;
  };
  range("null", "STAR_TREE", &out.star_tree, &out.star_tree_len);
  out.star_num_docs = (int32_t)ndocs;
  for (const std::string &dim : prop_list(kv, pre + "split.order")) {
    size_t ci = 0;
    while (ci < out.column_names.size() && out.column_names[ci] != dim) ci++;
    require(ci < out.column_names.size(), PINOT_ERR_BAD_ARG, "star-tree dimension " + dim + " is not a served column");
    pinot_column_desc d = out.cols[ci];  // the segment column: its dictionary, its bits
    d.is_sorted = 0;
    d.has_inverted_index = 0;
    d.inverted_index = nullptr;
    d.inverted_index_len = 0;
    d.sorted_index = nullptr;
    d.sorted_index_len = 0;
    d.bloom_filter = nullptr;
    d.bloom_filter_len = 0;
    d.create_bloom_filter = 0;
    d.min_value = d.max_value = nullptr;
    d.partition_function = nullptr;
    d.num_partitions = 0;
    d.partition_values = nullptr;
    d.num_partition_values = 0;
    range(dim, "FORWARD_INDEX", &d.forward_index, &d.forward_index_len);
    out.star_names.push_back(dim);
    out.star_cols.push_back(d);
  }
  for (const std::string &pair : prop_list(kv, pre + "function.column.pairs")) {
    if (pair.rfind("distinctCountHLL__", 0) == 0) {
      // DistinctCountHLLValueAggregator's BYTES values (HyperLogLog.getBytes) in a var-byte raw index: handed over
      // in the C-ABI's raw STRING layout (offsets + bytes); attach decodes the registers
      const uint8_t *p = nullptr;
      uint64_t n = 0;
      range(pair, "FORWARD_INDEX", &p, &n);
      out.owned.push_back(read_var_byte_chunks(p, n, ndocs, "star-tree " + pair));
      pinot_column_desc d{};
      d.data_type = PINOT_STRING;
      d.encoding = PINOT_ENCODING_RAW;
      d.forward_index = out.owned.back().data();
      d.forward_index_len = out.owned.back().size();
      out.star_names.push_back(pair);
      out.star_cols.push_back(d);
      continue;
    }
    if (pair.rfind("avg__", 0) == 0) {
      // AvgValueAggregator's BYTES values (AvgPair.toBytes: double sum, long count, big-endian, 16 B) in a var-byte
      // raw index, split into the C-ABI's two raw columns "<pair>.sum" (DOUBLE) and "<pair>.count" (LONG)
      const uint8_t *p = nullptr;
      uint64_t n = 0;
      range(pair, "FORWARD_INDEX", &p, &n);
      const std::vector<uint8_t> vb = read_var_byte_chunks(p, n, ndocs, "star-tree " + pair);
      const uint8_t *body = vb.data() + (size_t)(ndocs + 1) * 4;
      std::vector<uint8_t> sums((size_t)ndocs * 8), counts((size_t)ndocs * 8);
      for (int64_t i = 0; i < ndocs; i++) {
        auto at = [&](int64_t k) {
          const uint8_t *q = vb.data() + 4 * k;
          return ((uint64_t)q[0] << 24) | ((uint64_t)q[1] << 16) | ((uint64_t)q[2] << 8) | q[3];
        };
        const uint64_t o = at(i), e = at(i + 1);
        require(e - o == 16, PINOT_ERR_BAD_ARG, "star-tree " + pair + ": AvgPair value is not 16 bytes");
        memcpy(&sums[(size_t)i * 8], body + o, 8);
        memcpy(&counts[(size_t)i * 8], body + o + 8, 8);
      }
      const std::string part[2] = {pair + ".sum", pair + ".count"};
      for (int k = 0; k < 2; k++) {
        pinot_column_desc d{};
        d.data_type = k == 0 ? PINOT_DOUBLE : PINOT_LONG;
        d.encoding = PINOT_ENCODING_RAW;
        out.owned.push_back(k == 0 ? std::move(sums) : std::move(counts));
        d.forward_index = out.owned.back().data();
        d.forward_index_len = out.owned.back().size();
        out.star_names.push_back(part[k]);
        out.star_cols.push_back(d);
      }
      continue;
    }
    pinot_column_desc d{};
    d.data_type = pair.rfind("count__", 0) == 0 ? PINOT_LONG : PINOT_DOUBLE;
    d.encoding = PINOT_ENCODING_RAW;
    const uint8_t *p = nullptr;
    uint64_t n = 0;
    range(pair, "FORWARD_INDEX", &p, &n);
    out.owned.push_back(read_raw_chunks(p, n, ndocs, 8, "star-tree " + pair));
    d.forward_index = out.owned.back().data();
    d.forward_index_len = out.owned.back().size();
    out.star_names.push_back(pair);
    out.star_cols.push_back(d);
  }
  for (size_t i = 0; i < out.star_cols.size(); i++) out.star_cols[i].name = out.star_names[i].c_str();
  out.has_star = true;
}

pinot_segment_desc SegmentDirData::star_desc() const {
  pinot_segment_desc d{};
  d.name = name.c_str();
  d.num_docs = star_num_docs;
  d.num_columns = (int32_t)star_cols.size();
  d.columns = star_cols.data();
  return d;
}

pinot_segment_desc SegmentDirData::desc() const {
  pinot_segment_desc d{};
  d.name = name.c_str();
  d.num_docs = num_docs;
  d.num_columns = (int32_t)cols.size();
  d.columns = cols.data();
  return d;
}

}  // namespace pinot
