// Native RCCL communication engine.
//
// Replaces the reference's Horovod background thread + MPI coordinator
// (distributed_optimizer.py:21-26, Horovod 0.19 C++ core) with a direct RCCL
// communicator per process (one per device, built once and shared by every
// optimizer of the process, like hvd.init() at dist_trainer.py:125-126).
// Bootstrap: rank 0 creates an ncclUniqueId, the Python side ships its 128
// bytes through the torch.distributed store, every rank starts a NON-BLOCKING
// ncclCommInitRankConfig (config.blocking = 0) and polls it against a
// deadline: a peer that never arrives ends in ncclCommAbort and an exception
// on this rank instead of a process blocked forever inside RCCL.  The Python
// side agrees every bootstrap step over the process group (parallel/comm.py
// _bootstrap_native), so a failure on any rank sends all ranks to the
// torch.distributed path.  Collectives run on the CALLER's current HIP
// stream, so compress -> all-gather -> scatter is one stream-ordered chain
// (no host sync, no ProcessGroup bookkeeping, capturable in a hipGraph).
//
// What the engine adds over a bare communicator:
//   * grouped launches: several buckets' record all-gathers in ONE
//     ncclGroupStart/End (one kernel launch, all xGMI links busy at once);
//   * completion tracking: every collective is bracketed by two HIP events
//     (pooled); a background watchdog thread retires them, keeps per-op
//     latency / byte statistics (the measured alpha-beta of this node's
//     xGMI fabric, fed to the bucket planners) and
//   * failure detection: if a collective has not completed after the
//     timeout, or RCCL reports an asynchronous error, the watchdog aborts
//     the communicator (ncclCommAbort releases the spinning RCCL kernels, so
//     the GPU does not hang) and flags the engine; the next call on any
//     thread throws with the reason instead of deadlocking.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace gk {

enum CommOp : int { kOpAllGather = 0, kOpAllReduce = 1, kOpBroadcast = 2, kOpGroup = 3, kNumOps = 4 };

struct OpStats {
  uint64_t calls = 0;
  uint64_t bytes = 0;       // payload bytes per rank (send side)
  double ms_total = 0.0;    // sum of event-timed GPU durations
  double ms_max = 0.0;
};

class RcclComm {
 public:
  RcclComm() = default;
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  static std::vector<uint8_t> make_unique_id();
  // blocking convenience form: init_async + init_wait(timeout_s)
  void init(const std::vector<uint8_t>& uid, int rank, int world, int device, double timeout_s = 120.0);
  // non-blocking bootstrap: returns once the init is started
  void init_async(const std::vector<uint8_t>& uid, int rank, int world, int device);
  // 0 = ready, 1 = still in progress; aborts + throws on an RCCL error
  int init_poll();
  // polls until ready; on the deadline aborts the communicator and throws
  void init_wait(double timeout_s);
  // unconditional ncclCommAbort (bootstrap failure on this or another rank)
  void abort();
  // bound on how long an enqueue may wait for a non-blocking communicator
  // to leave ncclInProgress (lazy connection setup on the first collectives)
  void set_op_timeout(double s) { op_timeout_s_ = s; }
  void destroy();
  bool initialized() const { return comm_ != nullptr; }
  int rank() const { return rank_; }
  int world() const { return world_; }

  // bytes-level all-gather: recv holds world * bytes
  void allgather_bytes(const void* send, void* recv, size_t bytes, hipStream_t s);
  // several all-gathers in one RCCL group (one launch)
  void allgather_many(const std::vector<const void*>& sends, const std::vector<void*>& recvs,
                      const std::vector<size_t>& bytes, hipStream_t s);
  void allreduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t s);
  void broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t s);

  // completion tracking / failure detection
  void set_tracking(bool on) { tracking_ = on; }
  void start_watchdog(double timeout_s, double poll_ms);
  void stop_watchdog();
  // retire completed collectives on the calling thread (no watchdog running);
  // returns the number still in flight
  int poll();
  bool failed() const { return failed_.load(); }
  std::string error() const;
  void check() const;   // throws std::runtime_error(reason) once failed
  OpStats stats(int op) const;
  void reset_stats();
  int in_flight() const;
  // test hook: fail + abort as the watchdog would, from the calling thread
  void inject_failure(const std::string& why);
  void set_abort_grace_ms(int ms) { abort_grace_ms_ = ms < 0 ? 0 : ms; }

 private:
  struct Pending {
    hipEvent_t start, end;
    int op;
    size_t bytes;
    std::chrono::steady_clock::time_point t_enq;
  };
  hipEvent_t take_event();
  void begin_op(hipStream_t s, hipEvent_t* start);
  void end_op(hipStream_t s, hipEvent_t start, int op, size_t bytes);
  int retire_locked(bool check_timeout);
  // non-blocking communicator: wait (bounded) until an enqueue that returned
  // ncclInProgress has completed; throws on error / deadline
  void settle(ncclResult_t r, const char* what, double timeout_s);
  void fail(const std::string& why);   // caller holds mu_; marks only
  void abort_comm();                    // caller holds neither lock
  void watchdog_loop();

  ncclComm_t comm_ = nullptr;
  int rank_ = 0;
  int world_ = 1;
  int device_ = 0;
  bool tracking_ = true;
  bool init_done_ = false;
  double op_timeout_s_ = 300.0;
  mutable std::mutex mu_;
  std::deque<Pending> pending_;
  std::vector<hipEvent_t> pool_;
  OpStats stats_[kNumOps];
  std::atomic<bool> failed_{false};
  std::atomic<bool> aborted_{false};
  std::mutex enq_mu_;   // held for each collective enqueue (check + RCCL call)
  int abort_grace_ms_ = 2000;
  std::string error_;
  double timeout_s_ = 0.0;
  double poll_ms_ = 5.0;
  std::atomic<bool> stop_{false};
  std::thread watchdog_;
};

std::string rccl_error_string(ncclResult_t r);

}  // namespace gk
