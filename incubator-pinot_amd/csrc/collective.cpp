// Collectives of the multi-GPU server: RCCL over xGMI, and the one-device loopback that runs the same merge protocol
// with K ranks on one GPU (collective.h).
#include "collective.h"

#include <chrono>
#include <map>

namespace pinot {

#define PINOT_NCCL(expr)                                                                                 \
  do {                                                                                                   \
    ncclResult_t _r = (expr);                                                                            \
    if (_r != ncclSuccess) throw Error(PINOT_ERR_DEVICE, std::string(#expr) + ": " + ncclGetErrorString(_r)); \
  } while (0)

size_t ctype_size(CType t) { return t == CType::U8 ? 1 : 8; }

std::vector<const void *> Hub::exchange(int rank, const void *mine) {
  std::unique_lock<std::mutex> lk(mu_);
  require(!broken_, PINOT_ERR_DEVICE, "server communicator is broken (a rank failed to arrive earlier)");
  const uint64_t g = gen_;
  slots_[g & 1][rank] = mine;
  if (++arrived_ == n_) {
    arrived_ = 0;
    gen_++;
    cv_.notify_all();
  } else {
    const bool ok = cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms_), [&] { return gen_ != g || broken_; });
    if (!ok || gen_ == g) {
      broken_ = true;
      cv_.notify_all();
      throw Error(PINOT_ERR_DEVICE, "server communicator: a peer rank did not arrive within " +
                                        std::to_string(timeout_ms_) + " ms");
    }
  }
  return slots_[g & 1];
}

std::shared_ptr<Hub> loopback_hub(const uint8_t *id, int nranks, int timeout_ms, int device) {
  static std::mutex mu;
  static std::map<std::string, std::weak_ptr<Hub>> hubs;
  std::lock_guard<std::mutex> lk(mu);
  const std::string key(reinterpret_cast<const char *>(id), 128);
  auto it = hubs.find(key);
  if (it != hubs.end())
    if (auto h = it->second.lock()) {
      require(h->size() == nranks, PINOT_ERR_BAD_ARG, "loopback communicator: ranks disagree on nranks");
      require(h->device == device, PINOT_ERR_BAD_ARG, "loopback communicator: every rank must use the same device");
      return h;
    }
  for (auto i = hubs.begin(); i != hubs.end();) i = i->second.expired() ? hubs.erase(i) : std::next(i);
  auto h = std::make_shared<Hub>(nranks, timeout_ms);
  h->device = device;
  hubs[key] = h;
  return h;
}

std::vector<std::vector<uint8_t>> Collective::all_gather_host(const std::vector<uint8_t> &mine, hipStream_t st) {
  if (nranks_ == 1) return {mine};
  // one fixed-size round carries every rank's size and, when it fits, its payload (the control messages of an
  // aggregation or a group-by phase do): a second round only for payloads beyond the inline room. Every rank knows
  // every size after the first round, so all take the second one together.
  constexpr size_t kInline = 4096;
  std::vector<uint8_t> block(kInline, 0), first(kInline * (size_t)nranks_);
  const int64_t sz = (int64_t)mine.size();
  memcpy(block.data(), &sz, 8);
  if (!mine.empty() && mine.size() <= kInline - 8) memcpy(block.data() + 8, mine.data(), mine.size());
  all_gather_fixed_host(block.data(), kInline, first.data(), st);
  std::vector<int64_t> sizes(nranks_);
  int64_t mx = 0;
  for (int r = 0; r < nranks_; r++) {
    memcpy(&sizes[r], first.data() + (size_t)r * kInline, 8);
    require(sizes[r] >= 0, PINOT_ERR_DEVICE, "server communicator: bad control payload size");
    mx = std::max(mx, sizes[r]);
  }
  std::vector<std::vector<uint8_t>> out(nranks_);
  if (mx == 0) return out;
  if (mx <= (int64_t)(kInline - 8)) {
    for (int r = 0; r < nranks_; r++) {
      const auto at = first.begin() + (size_t)r * kInline + 8;
      out[r].assign(at, at + sizes[r]);
    }
    return out;
  }
  std::vector<uint8_t> padded(mx, 0), all((size_t)mx * nranks_);
  if (!mine.empty()) memcpy(padded.data(), mine.data(), mine.size());
  all_gather_fixed_host(padded.data(), (size_t)mx, all.data(), st);
  for (int r = 0; r < nranks_; r++) {
    require(sizes[r] >= 0 && sizes[r] <= mx, PINOT_ERR_DEVICE, "server communicator: bad control payload size");
    out[r].assign(all.begin() + (size_t)r * mx, all.begin() + (size_t)r * mx + sizes[r]);
  }
  return out;
}

namespace {

void hub_all_gather(Hub &hub, int rank, int n, const void *mine, size_t bytes, uint8_t *out) {
  auto ptrs = hub.exchange(rank, mine);
  for (int r = 0; r < n; r++) memcpy(out + (size_t)r * bytes, ptrs[r], bytes);
  hub.exchange(rank, nullptr);  // every rank has copied: the publishers' buffers may go
}

ncclDataType_t nccl_type(CType t) {
  switch (t) {
    case CType::I64: return ncclInt64;
    case CType::U64: return ncclUint64;
    case CType::F64: return ncclFloat64;
    default: return ncclUint8;
  }
}
ncclRedOp_t nccl_op(COp op) { return op == COp::SUM ? ncclSum : op == COp::MIN ? ncclMin : ncclMax; }

class RcclCollective : public Collective {
 public:
  RcclCollective(ncclComm_t comm, int rank, int nranks, std::shared_ptr<Hub> hub)
      : Collective(rank, nranks), comm_(comm), hub_(std::move(hub)) {}
  ~RcclCollective() override {
    if (comm_) (void)ncclCommDestroy(comm_);
  }
  const char *kind() const override { return "rccl"; }
  void group_start() override { PINOT_NCCL(ncclGroupStart()); }
  void group_end() override { PINOT_NCCL(ncclGroupEnd()); }
  void all_reduce(void *buf, size_t count, CType t, COp op, hipStream_t st) override {
    if (nranks_ == 1 || count == 0) return;
    PINOT_NCCL(ncclAllReduce(buf, buf, count, nccl_type(t), nccl_op(op), comm_, st));
  }
  void reduce_scatter(void *buf, size_t recvcount, CType t, COp op, hipStream_t st) override {
    if (nranks_ == 1 || recvcount == 0) return;
    uint8_t *b = static_cast<uint8_t *>(buf);
    PINOT_NCCL(ncclReduceScatter(b, b + (size_t)rank_ * recvcount * ctype_size(t), recvcount, nccl_type(t), nccl_op(op),
                                 comm_, st));
  }
  void gather(const void *send, size_t bytes, void *recv, const std::vector<size_t> &offsets, int root,
              hipStream_t st) override {
    uint8_t *rv = static_cast<uint8_t *>(recv);
    if (rank_ == root && bytes && rv + offsets[rank_] != send)
      PINOT_HIP(hipMemcpyAsync(rv + offsets[rank_], send, bytes, hipMemcpyDeviceToDevice, st));
    if (nranks_ == 1) return;
    PINOT_NCCL(ncclGroupStart());
    if (rank_ == root) {
      for (int r = 0; r < nranks_; r++) {
        const size_t n = offsets[r + 1] - offsets[r];
        if (r != root && n) PINOT_NCCL(ncclRecv(rv + offsets[r], n, ncclUint8, r, comm_, st));
      }
    } else if (bytes) {
      PINOT_NCCL(ncclSend(send, bytes, ncclUint8, root, comm_, st));
    }
    PINOT_NCCL(ncclGroupEnd());
  }

 protected:
  void all_gather_fixed_host(const void *mine, size_t bytes, uint8_t *out, hipStream_t st) override {
    if (hub_) {
      hub_all_gather(*hub_, rank_, nranks_, mine, bytes, out);
      return;
    }
    const size_t total = bytes * nranks_;
    stage_.reserve(total + 64);
    pinned_.reserve(total + 64);
    uint8_t *d = stage_.get<uint8_t>(), *h = pinned_.get<uint8_t>();
    memcpy(h + (size_t)rank_ * bytes, mine, bytes);
    PINOT_HIP(hipMemcpyAsync(d + (size_t)rank_ * bytes, h + (size_t)rank_ * bytes, bytes, hipMemcpyHostToDevice, st));
    PINOT_NCCL(ncclAllGather(d + (size_t)rank_ * bytes, d, bytes, ncclUint8, comm_, st));
    PINOT_HIP(hipMemcpyAsync(h, d, total, hipMemcpyDeviceToHost, st));
    PINOT_HIP(hipStreamSynchronize(st));
    memcpy(out, h, total);
  }

 private:
  ncclComm_t comm_;
  std::shared_ptr<Hub> hub_;
  DeviceBuffer stage_;
  PinnedBuffer pinned_;
};

class LoopbackCollective : public Collective {
 public:
  LoopbackCollective(std::shared_ptr<Hub> hub, int rank, int device)
      : Collective(rank, hub->size()), hub_(std::move(hub)) {
    require(nranks_ <= kMaxLoopbackRanks, PINOT_ERR_BAD_ARG, "loopback communicator: at most 16 ranks");
    PINOT_HIP(hipSetDevice(device));
    PINOT_HIP(hipEventCreateWithFlags(&ready_, hipEventDisableTiming));
    PINOT_HIP(hipEventCreateWithFlags(&done_, hipEventDisableTiming));
  }
  ~LoopbackCollective() override {
    if (ready_) (void)hipEventDestroy(ready_);
    if (done_) (void)hipEventDestroy(done_);
  }
  const char *kind() const override { return "loopback"; }
  void all_reduce(void *buf, size_t count, CType t, COp op, hipStream_t st) override {
    reduce_into(buf, 0, count, t, op, st);
  }
  void reduce_scatter(void *buf, size_t recvcount, CType t, COp op, hipStream_t st) override {
    reduce_into(buf, (size_t)rank_ * recvcount * ctype_size(t), recvcount, t, op, st);
  }
  void gather(const void *send, size_t bytes, void *recv, const std::vector<size_t> &offsets, int root,
              hipStream_t st) override {
    uint8_t *rv = static_cast<uint8_t *>(recv);
    if (nranks_ == 1) {
      if (bytes && rv + offsets[0] != send) PINOT_HIP(hipMemcpyAsync(rv + offsets[0], send, bytes, hipMemcpyDeviceToDevice, st));
      return;
    }
    auto all = arrive(send, st);
    if (rank_ == root)
      for (int r = 0; r < nranks_; r++) {
        const size_t n = offsets[r + 1] - offsets[r];
        if (n && rv + offsets[r] != all[r].buf)
          PINOT_HIP(hipMemcpyAsync(rv + offsets[r], all[r].buf, n, hipMemcpyDeviceToDevice, st));
      }
    depart(st);
  }

 protected:
  void all_gather_fixed_host(const void *mine, size_t bytes, uint8_t *out, hipStream_t) override {
    hub_all_gather(*hub_, rank_, nranks_, mine, bytes, out);
  }

 private:
  struct Pub {
    const void *buf;
    hipEvent_t ev;
  };
  // every rank's buffer, once every rank's earlier stream work on it is ordered before this rank's next step
  std::vector<Pub> arrive(const void *buf, hipStream_t st) {
    PINOT_HIP(hipEventRecord(ready_, st));
    pub_ready_ = Pub{buf, ready_};
    auto ptrs = hub_->exchange(rank_, &pub_ready_);
    std::vector<Pub> all(nranks_);
    for (int r = 0; r < nranks_; r++) all[r] = *static_cast<const Pub *>(ptrs[r]);
    for (int r = 0; r < nranks_; r++)
      if (r != rank_) PINOT_HIP(hipStreamWaitEvent(st, all[r].ev, 0));
    return all;
  }
  // no rank touches its buffers again before every rank's reads of them are done
  void depart(hipStream_t st) {
    PINOT_HIP(hipEventRecord(done_, st));
    pub_done_ = Pub{nullptr, done_};
    auto ptrs = hub_->exchange(rank_, &pub_done_);
    for (int r = 0; r < nranks_; r++)
      if (r != rank_) PINOT_HIP(hipStreamWaitEvent(st, static_cast<const Pub *>(ptrs[r])->ev, 0));
  }
  void reduce_into(void *buf, size_t byte_off, size_t count, CType t, COp op, hipStream_t st) {
    if (nranks_ == 1 || count == 0) return;
    const size_t bytes = count * ctype_size(t);
    auto all = arrive(buf, st);
    RankPtrs in{};
    for (int r = 0; r < nranks_; r++) in.p[r] = static_cast<const uint8_t *>(all[r].buf) + byte_off;
    scratch_.reserve(bytes + 64);
    launch_rank_reduce(t, op, in, nranks_, scratch_.get(), count, st);
    PINOT_HIP(hipGetLastError());
    depart(st);  // the reduced slice may now overwrite this rank's own buffer
    PINOT_HIP(hipMemcpyAsync(static_cast<uint8_t *>(buf) + byte_off, scratch_.get(), bytes, hipMemcpyDeviceToDevice, st));
  }

  std::shared_ptr<Hub> hub_;
  hipEvent_t ready_ = nullptr, done_ = nullptr;
  Pub pub_ready_{}, pub_done_{};
  DeviceBuffer scratch_;
};

}  // namespace

std::unique_ptr<Collective> make_rccl_collective(ncclComm_t comm, int rank, int nranks, std::shared_ptr<Hub> hub) {
  return std::make_unique<RcclCollective>(comm, rank, nranks, std::move(hub));
}

std::unique_ptr<Collective> make_loopback_collective(std::shared_ptr<Hub> hub, int rank, int device) {
  return std::make_unique<LoopbackCollective>(std::move(hub), rank, device);
}

}  // namespace pinot
