#include "rccl_engine.h"

#include <cstring>
#include <stdexcept>

namespace gk {

std::string rccl_error_string(ncclResult_t r) { return std::string(ncclGetErrorString(r)); }

#define GK_NCCL_CHECK(expr)                                                                     \
  do {                                                                                          \
    ncclResult_t _r = (expr);                                                                   \
    if (_r != ncclSuccess)                                                                      \
      throw std::runtime_error(std::string("RCCL error at " #expr ": ") + rccl_error_string(_r)); \
  } while (0)

RcclComm::~RcclComm() {
  // Never abort from a destructor; communicator teardown is explicit.
  if (comm_ != nullptr) {
    ncclCommDestroy(comm_);
    comm_ = nullptr;
  }
}

std::vector<uint8_t> RcclComm::make_unique_id() {
  ncclUniqueId id;
  GK_NCCL_CHECK(ncclGetUniqueId(&id));
  std::vector<uint8_t> out(sizeof(id.internal));
  std::memcpy(out.data(), id.internal, sizeof(id.internal));
  return out;
}

void RcclComm::init(const std::vector<uint8_t>& uid, int rank, int world, int device) {
  if (comm_ != nullptr) throw std::runtime_error("RcclComm already initialised");
  ncclUniqueId id;
  if (uid.size() != sizeof(id.internal)) throw std::runtime_error("bad ncclUniqueId size");
  std::memcpy(id.internal, uid.data(), sizeof(id.internal));
  if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("hipSetDevice failed");
  GK_NCCL_CHECK(ncclCommInitRank(&comm_, world, id, rank));
  rank_ = rank;
  world_ = world;
}

void RcclComm::destroy() {
  if (comm_ != nullptr) {
    GK_NCCL_CHECK(ncclCommDestroy(comm_));
    comm_ = nullptr;
  }
}

void RcclComm::allgather_bytes(const void* send, void* recv, size_t bytes, hipStream_t s) {
  GK_NCCL_CHECK(ncclAllGather(send, recv, bytes, ncclUint8, comm_, s));
}

void RcclComm::allreduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t s) {
  GK_NCCL_CHECK(ncclAllReduce(buf, buf, count, dt, op, comm_, s));
}

void RcclComm::broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t s) {
  GK_NCCL_CHECK(ncclBroadcast(buf, buf, count, dt, root, comm_, s));
}

void RcclComm::group_start() { GK_NCCL_CHECK(ncclGroupStart()); }
void RcclComm::group_end() { GK_NCCL_CHECK(ncclGroupEnd()); }

}  // namespace gk
