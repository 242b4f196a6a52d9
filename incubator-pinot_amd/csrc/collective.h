// Collectives of the multi-GPU server (server.cpp): the exchange steps of the cross-segment combine
// (CombineOperator.java:75-196, CombineGroupByOperator.java:104-228) over one communicator of ranks.
//
//   RcclCollective      RCCL over xGMI: one communicator per GPU (ncclCommInitAll in one process, ncclCommInitRank
//                       across processes). Data steps are RCCL collectives on the engine's stream; control data
//                       (headers, dictionaries, error status) go through an in-process Hub when every rank lives in
//                       this process, else through ncclAllGather.
//   LoopbackCollective  every rank in this process on ONE device (server.loopback=1): the same data steps done by
//                       an in-library device reduce / copy over the ranks' buffers, ordered with HIP events, so the
//                       merge code (slicing, padding, owner finalize, gather, agreement) runs with K > 1 ranks on a
//                       one-GPU box.
// Every rank issues the same sequence of calls (the server's query protocol guarantees it); a rank's buffers may be
// reused as soon as a call returns.
#pragma once
#include <rccl/rccl.h>

#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "common.h"

namespace pinot {

enum class CType { I64, U64, F64, U8 };
enum class COp { SUM, MIN, MAX };
size_t ctype_size(CType t);

constexpr int kMaxLoopbackRanks = 16;

// In-process rendezvous of the ranks of one communicator that live in this process. exchange(): every rank
// publishes one pointer and gets all ranks' pointers back (the pointee must stay valid until the publisher's next
// exchange). A rank that does not arrive within the timeout breaks the hub: every waiter and every later call
// fails instead of hanging.
class Hub {
 public:
  Hub(int n, int timeout_ms) : n_(n), timeout_ms_(timeout_ms) {
    slots_[0].assign(n, nullptr);
    slots_[1].assign(n, nullptr);
  }
  std::vector<const void *> exchange(int rank, const void *mine);
  int size() const { return n_; }
  int device = -1;  // loopback: the one device every rank runs on

 private:
  int n_, timeout_ms_;
  std::mutex mu_;
  std::condition_variable cv_;
  uint64_t gen_ = 0;
  int arrived_ = 0;
  bool broken_ = false;
  std::vector<const void *> slots_[2];  // by generation parity: a rank can be one exchange ahead of the slowest
};

// Process-wide registry of loopback hubs, keyed by the communicator id (multi-process form, loopback ranks).
std::shared_ptr<Hub> loopback_hub(const uint8_t *id, int nranks, int timeout_ms, int device);

class Collective {
 public:
  Collective(int rank, int nranks) : rank_(rank), nranks_(nranks) {}
  virtual ~Collective() = default;
  int rank() const { return rank_; }
  int nranks() const { return nranks_; }
  virtual const char *kind() const = 0;

  // in place: every rank ends with the element-wise reduction of every rank's buf[0, count)
  virtual void all_reduce(void *buf, size_t count, CType t, COp op, hipStream_t st) = 0;
  // in place: buf holds nranks * recvcount elements; rank r ends with the reduction of slice r at
  // buf + r * recvcount (the other slices are left undefined)
  virtual void reduce_scatter(void *buf, size_t recvcount, CType t, COp op, hipStream_t st) = 0;
  // root receives every rank's `bytes` of send at recv + offsets[r]; offsets (nranks + 1 prefix sums, so rank r
  // sends offsets[r + 1] - offsets[r] bytes) and recv are read on the root only
  virtual void gather(const void *send, size_t bytes, void *recv, const std::vector<size_t> &offsets, int root,
                      hipStream_t st) = 0;
  // every rank's host bytes in rank order (control data: agreement headers, dictionaries, small results)
  std::vector<std::vector<uint8_t>> all_gather_host(const std::vector<uint8_t> &mine, hipStream_t st);
  // ranks batch their data steps between group_start / group_end (RCCL groups; no-op for the loopback)
  virtual void group_start() {}
  virtual void group_end() {}

 protected:
  // every rank contributes exactly `bytes` bytes; out = nranks * bytes in rank order
  virtual void all_gather_fixed_host(const void *mine, size_t bytes, uint8_t *out, hipStream_t st) = 0;
  int rank_, nranks_;
};

// hub != nullptr: every rank is in this process (control data through host memory)
std::unique_ptr<Collective> make_rccl_collective(ncclComm_t comm, int rank, int nranks, std::shared_ptr<Hub> hub);
std::unique_ptr<Collective> make_loopback_collective(std::shared_ptr<Hub> hub, int rank, int device);

// collective.hip: out[i] = op over r < n of in[r][i] (loopback reduce), on `st`
struct RankPtrs {
  const void *p[kMaxLoopbackRanks];
};
void launch_rank_reduce(CType t, COp op, const RankPtrs &in, int n, void *out, size_t count, hipStream_t st);

}  // namespace pinot
