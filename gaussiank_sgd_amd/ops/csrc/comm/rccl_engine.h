// Native RCCL communication engine.
//
// Replaces the reference's Horovod background thread + MPI coordinator
// (distributed_optimizer.py:21-26, Horovod 0.19 C++ core) with a direct RCCL
// communicator per process.  Bootstrap: rank 0 creates an ncclUniqueId, the
// Python side ships its 128 bytes through the torch.distributed store, every
// rank calls ncclCommInitRank.  Collectives run on the CALLER's current HIP
// stream, so compress -> all-gather -> scatter is one stream-ordered chain
// (no host sync, no ProcessGroup bookkeeping, capturable in a hipGraph).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <string>
#include <vector>

namespace gk {

class RcclComm {
 public:
  RcclComm() = default;
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  static std::vector<uint8_t> make_unique_id();
  void init(const std::vector<uint8_t>& uid, int rank, int world, int device);
  void destroy();
  bool initialized() const { return comm_ != nullptr; }
  int rank() const { return rank_; }
  int world() const { return world_; }

  // bytes-level all-gather: recv holds world * bytes
  void allgather_bytes(const void* send, void* recv, size_t bytes, hipStream_t s);
  void allreduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t s);
  void broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t s);
  void group_start();
  void group_end();

 private:
  ncclComm_t comm_ = nullptr;
  int rank_ = 0;
  int world_ = 1;
};

std::string rccl_error_string(ncclResult_t r);

}  // namespace gk
