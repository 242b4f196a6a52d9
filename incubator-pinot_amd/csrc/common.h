// Internal shared definitions of the MI355X Pinot segment executor.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <stdexcept>
#include <string>
#include <mutex>
#include <vector>

#include "pinot_gpu.h"

namespace pinot {

// Exception type carried up to the C-ABI, where it becomes a pinot_status + last_error.
struct Error : std::runtime_error {
  pinot_status status;
  Error(pinot_status s, const std::string &m) : std::runtime_error(m), status(s) {}
};

#define PINOT_HIP(expr)                                                                       \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess) {                                                                   \
      throw ::pinot::Error(_e == hipErrorOutOfMemory ? PINOT_ERR_OOM : PINOT_ERR_DEVICE,      \
                           std::string(#expr) + ": " + hipGetErrorString(_e));                \
    }                                                                                         \
  } while (0)

inline void require(bool ok, pinot_status s, const std::string &msg) {
  if (!ok) throw Error(s, msg);
}

// Grow-only / owning device allocation.
class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  explicit DeviceBuffer(size_t bytes) { alloc(bytes); }
  ~DeviceBuffer() { reset(); }
  DeviceBuffer(const DeviceBuffer &) = delete;
  DeviceBuffer &operator=(const DeviceBuffer &) = delete;
  DeviceBuffer(DeviceBuffer &&o) noexcept : p_(o.p_), n_(o.n_), gen_(o.gen_ + 1) { o.p_ = nullptr; o.n_ = 0; o.gen_++; }
  DeviceBuffer &operator=(DeviceBuffer &&o) noexcept {
    if (this != &o) { reset(); p_ = o.p_; n_ = o.n_; gen_ += o.gen_ + 1; o.p_ = nullptr; o.n_ = 0; o.gen_++; }
    return *this;
  }
  void alloc(size_t bytes) {
    reset();
    gen_++;
    if (bytes == 0) return;
    PINOT_HIP(hipMalloc(&p_, bytes));
    n_ = bytes;
  }
  // Bumped by every (re)allocation: contents cached by address are stale once it changes.
  uint64_t generation() const { return gen_; }
  // Ensure capacity >= bytes (contents not preserved).
  void reserve(size_t bytes) {
    if (bytes > n_) alloc(bytes + bytes / 4);
  }
  void reset() {
    if (p_) (void)hipFree(p_);
    p_ = nullptr;
    n_ = 0;
  }
  template <typename T = void> T *get() const { return static_cast<T *>(p_); }
  size_t size() const { return n_; }

 private:
  void *p_ = nullptr;
  size_t n_ = 0;
  uint64_t gen_ = 0;
};

// Grow-only pinned host buffer (async H2D / D2H staging of the per-query tables and results).
class PinnedBuffer {
 public:
  PinnedBuffer() = default;
  ~PinnedBuffer() { reset(); }
  PinnedBuffer(const PinnedBuffer &) = delete;
  PinnedBuffer &operator=(const PinnedBuffer &) = delete;
  void reserve(size_t bytes) {
    if (bytes <= n_) return;
    reset();
    const size_t want = bytes + bytes / 4;
    PINOT_HIP(hipHostMalloc(&p_, want, hipHostMallocDefault));
    n_ = want;
  }
  void reset() {
    if (p_) (void)hipHostFree(p_);
    p_ = nullptr;
    n_ = 0;
  }
  template <typename T = void> T *get() const { return static_cast<T *>(p_); }

 private:
  void *p_ = nullptr;
  size_t n_ = 0;
};

// Pinned host memory the device writes directly (zero-copy results of the fused query kernel).
class MappedBuffer {
 public:
  MappedBuffer() = default;
  ~MappedBuffer() { reset(); }
  MappedBuffer(const MappedBuffer &) = delete;
  MappedBuffer &operator=(const MappedBuffer &) = delete;
  void reserve(size_t bytes) {
    if (bytes <= n_) return;
    reset();
    const size_t want = bytes + bytes / 4;
    PINOT_HIP(hipHostMalloc(&p_, want, hipHostMallocMapped | hipHostMallocCoherent));
    PINOT_HIP(hipHostGetDevicePointer(&d_, p_, 0));
    n_ = want;
  }
  void reset() {
    if (p_) (void)hipHostFree(p_);
    p_ = d_ = nullptr;
    n_ = 0;
  }
  template <typename T = void> T *host() const { return static_cast<T *>(p_); }
  template <typename T = void> T *device() const { return static_cast<T *>(d_); }

 private:
  void *p_ = nullptr, *d_ = nullptr;
  size_t n_ = 0;
};

// Pinned host blocks are slow to get and to give back (hipHostMalloc / hipHostFree: milliseconds for the result
// arrays of a 1M-group query, and the free waits for the device), so freed blocks are kept for reuse: one free list
// per power-of-two size class, at most kPinnedCacheBytes held in all.
struct PinnedCache {
  static constexpr size_t kPinnedCacheBytes = size_t(4) << 30;
  std::mutex mu;
  std::vector<void *> lists[64];
  size_t held = 0;
  static PinnedCache &get() {
    static PinnedCache *c = new PinnedCache();  // never destroyed: blocks may be returned during static teardown
    return *c;
  }
  static int size_class(size_t bytes) { return 64 - __builtin_clzll((unsigned long long)(bytes - 1)); }
  void *take(size_t bytes) {  // a block of 2^size_class(bytes) bytes, or nullptr
    std::lock_guard<std::mutex> lk(mu);
    auto &l = lists[size_class(bytes)];
    if (l.empty()) return nullptr;
    void *p = l.back();
    l.pop_back();
    held -= size_t(1) << size_class(bytes);
    return p;
  }
  bool give(void *p, size_t bytes) {
    std::lock_guard<std::mutex> lk(mu);
    const size_t sz = size_t(1) << size_class(bytes);
    if (held + sz > kPinnedCacheBytes) return false;
    lists[size_class(bytes)].push_back(p);
    held += sz;
    return true;
  }
};

// Allocator of the large host result arrays: >= 1 MiB blocks are pinned (hipHostMalloc, rounded up to their size class
// and cached by PinnedCache), so the device's final per-group arrays are copied straight into them (no staging
// buffer, no host fill); smaller blocks — and any block when pinning fails, e.g. without a GPU — come from malloc. A
// 64-byte header records which (and the pinned block's size).
template <typename T>
struct PinnedAllocator {
  using value_type = T;
  PinnedAllocator() = default;
  template <typename U>
  PinnedAllocator(const PinnedAllocator<U> &) {}
  T *allocate(size_t n) {
    size_t bytes = n * sizeof(T) + 64;
    void *p = nullptr;
    uint32_t tag = 0;
    if (bytes >= (1u << 20)) {
      bytes = size_t(1) << PinnedCache::size_class(bytes);
      p = PinnedCache::get().take(bytes);
      if (p || hipHostMalloc(&p, bytes, hipHostMallocDefault) == hipSuccess) tag = 1;
    }
    if (!tag) {
      (void)hipGetLastError();
      p = std::malloc(bytes);
      if (!p) throw std::bad_alloc();
    }
    static_cast<uint32_t *>(p)[0] = tag;
    reinterpret_cast<uint64_t *>(p)[1] = bytes;
    return reinterpret_cast<T *>(static_cast<uint8_t *>(p) + 64);
  }
  void deallocate(T *q, size_t) {
    if (!q) return;
    void *p = reinterpret_cast<uint8_t *>(q) - 64;
    if (static_cast<uint32_t *>(p)[0] == 1) {
      if (!PinnedCache::get().give(p, reinterpret_cast<uint64_t *>(p)[1])) (void)hipHostFree(p);
    } else {
      std::free(p);
    }
  }
  template <typename U>
  bool operator==(const PinnedAllocator<U> &) const { return true; }
  template <typename U>
  bool operator!=(const PinnedAllocator<U> &) const { return false; }
};
template <typename T>
using HostVec = std::vector<T, PinnedAllocator<T>>;

inline uint32_t load_be32(const uint8_t *p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | uint32_t(p[3]);
}
inline uint64_t load_be64(const uint8_t *p) {
  return (uint64_t(load_be32(p)) << 32) | load_be32(p + 4);
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// PinotDataBitSet.getNumBitsPerValue (PinotDataBitSet.java:60-71)
inline int num_bits_per_value(int64_t max_value) {
  if (max_value <= 1) return 1;
  int b = 0;
  while (max_value > 0) { b++; max_value >>= 1; }
  return b;
}

}  // namespace pinot
