#include "rccl_engine.h"

#include <cstdio>
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

namespace {
size_t dtype_bytes(ncclDataType_t dt) {
  return (dt == ncclFloat64 || dt == ncclInt64 || dt == ncclUint64) ? 8
         : (dt == ncclFloat16 || dt == ncclBfloat16)                 ? 2
         : (dt == ncclInt8 || dt == ncclUint8)                       ? 1
                                                                     : 4;
}

const char* op_name(int op) {
  switch (op) {
    case kOpAllGather: return "all-gather";
    case kOpAllReduce: return "all-reduce";
    case kOpBroadcast: return "broadcast";
    default: return "grouped all-gather";
  }
}
}  // namespace

RcclComm::~RcclComm() {
  // Never abort from a destructor; communicator teardown is explicit.
  stop_watchdog();
  if (comm_ != nullptr) {
    if (!aborted_.load()) ncclCommDestroy(comm_);   // an aborted communicator is already freed
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

void RcclComm::init(const std::vector<uint8_t>& uid, int rank, int world, int device, double timeout_s) {
  init_async(uid, rank, world, device);
  init_wait(timeout_s);
}

void RcclComm::init_async(const std::vector<uint8_t>& uid, int rank, int world, int device) {
  if (comm_ != nullptr) throw std::runtime_error("RcclComm already initialised");
  ncclUniqueId id;
  if (uid.size() != sizeof(id.internal)) throw std::runtime_error("bad ncclUniqueId size");
  std::memcpy(id.internal, uid.data(), sizeof(id.internal));
  if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("hipSetDevice failed");
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;   // returns at once; progress is polled (init_poll / init_wait)
  ncclComm_t c = nullptr;
  const ncclResult_t r = ncclCommInitRankConfig(&c, world, id, rank, &cfg);
  if (r != ncclSuccess && r != ncclInProgress) {
    if (c != nullptr) ncclCommAbort(c);
    throw std::runtime_error(std::string("ncclCommInitRankConfig: ") + rccl_error_string(r));
  }
  comm_ = c;
  rank_ = rank;
  world_ = world;
  device_ = device;
  init_done_ = false;
  aborted_.store(false);
  failed_.store(false);
}

int RcclComm::init_poll() {
  if (comm_ == nullptr) throw std::runtime_error("RcclComm: init_poll before init_async (or after abort)");
  if (init_done_) return 0;
  ncclResult_t st = ncclSuccess;
  const ncclResult_t q = ncclCommGetAsyncError(comm_, &st);
  if (q != ncclSuccess) st = q;
  if (st == ncclInProgress) return 1;
  if (st != ncclSuccess) {
    const std::string why = std::string("RCCL communicator init failed: ") + rccl_error_string(st);
    abort();
    throw std::runtime_error(why);
  }
  init_done_ = true;
  return 0;
}

void RcclComm::init_wait(double timeout_s) {
  const auto t0 = std::chrono::steady_clock::now();
  while (init_poll() != 0) {
    const double waited = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (timeout_s > 0.0 && waited > timeout_s) {
      char buf[160];
      std::snprintf(buf, sizeof(buf), "rank %d: RCCL communicator init not complete after %.1f s (world %d)",
                    rank_, waited, world_);
      abort();
      throw std::runtime_error(buf);
    }
    std::this_thread::sleep_for(std::chrono::microseconds(500));
  }
}

// Bootstrap failure (here or on another rank): release the communicator at
// once.  ncclCommAbort also frees a communicator whose init is still in
// progress and releases RCCL kernels spinning on a peer that never arrived.
void RcclComm::abort() {
  stop_watchdog();
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (!failed_.load()) fail("aborted by the bootstrap protocol");
  }
  std::lock_guard<std::mutex> ek(enq_mu_);
  bool expected = false;
  if (comm_ != nullptr && aborted_.compare_exchange_strong(expected, true)) ncclCommAbort(comm_);
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& p : pending_) {
    pool_.push_back(p.start);
    pool_.push_back(p.end);
  }
  pending_.clear();
  comm_ = nullptr;
}

void RcclComm::settle(ncclResult_t r, const char* what, double timeout_s) {
  if (r == ncclSuccess) return;
  if (r != ncclInProgress)
    throw std::runtime_error(std::string("RCCL error at ") + what + ": " + rccl_error_string(r));
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    ncclResult_t st = ncclSuccess;
    const ncclResult_t q = ncclCommGetAsyncError(comm_, &st);
    if (q != ncclSuccess) st = q;
    if (st == ncclSuccess) return;
    if (st != ncclInProgress) {
      const std::string why = std::string("RCCL error at ") + what + ": " + rccl_error_string(st);
      std::lock_guard<std::mutex> lk(mu_);
      fail(why);   // the watchdog (or destroy) aborts the communicator
      throw std::runtime_error(why);
    }
    const double waited = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (timeout_s > 0.0 && waited > timeout_s) {
      char buf[200];
      std::snprintf(buf, sizeof(buf), "rank %d: %s still in progress after %.1f s (world %d)", rank_, what, waited,
                    world_);
      std::lock_guard<std::mutex> lk(mu_);
      fail(buf);
      throw std::runtime_error(buf);
    }
    std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
}

void RcclComm::destroy() {
  stop_watchdog();
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (!failed_.load()) {
      // in-flight collectives finish before their events are released
      for (auto& p : pending_) hipEventSynchronize(p.end);
    }
    retire_locked(false);
    for (auto& p : pending_) {
      hipEventDestroy(p.start);
      hipEventDestroy(p.end);
    }
    pending_.clear();
    for (hipEvent_t e : pool_) hipEventDestroy(e);
    pool_.clear();
  }
  std::lock_guard<std::mutex> ek(enq_mu_);
  if (comm_ == nullptr) return;
  ncclComm_t c = comm_;
  comm_ = nullptr;
  if (aborted_.load()) return;   // an aborted communicator is already freed
  if (failed_.load() || !init_done_) {
    aborted_.store(true);
    ncclCommAbort(c);
    return;
  }
  // non-blocking teardown: finalize (flush), bounded wait, then free; a
  // finalize that does not finish (dead peer) ends in an abort
  ncclResult_t r = ncclCommFinalize(c);
  const auto t0 = std::chrono::steady_clock::now();
  while (r == ncclSuccess || r == ncclInProgress) {
    ncclResult_t st = ncclSuccess;
    if (ncclCommGetAsyncError(c, &st) != ncclSuccess) {
      r = ncclInternalError;
      break;
    }
    if (st != ncclInProgress) {
      r = st;
      break;
    }
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > op_timeout_s_) {
      r = ncclInProgress;
      break;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  if (r != ncclSuccess) {
    aborted_.store(true);
    ncclCommAbort(c);
    return;
  }
  GK_NCCL_CHECK(ncclCommDestroy(c));
}

// ---------------------------------------------------------------------------
// completion tracking
// ---------------------------------------------------------------------------
hipEvent_t RcclComm::take_event() {
  if (!pool_.empty()) {
    hipEvent_t e = pool_.back();
    pool_.pop_back();
    return e;
  }
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) throw std::runtime_error("hipEventCreate failed");
  return e;
}

void RcclComm::begin_op(hipStream_t s, hipEvent_t* start) {
  check();
  if (comm_ == nullptr) throw std::runtime_error("RcclComm not initialised");
  *start = nullptr;
  if (!tracking_) return;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) return;  // graph capture
  std::lock_guard<std::mutex> lk(mu_);
  *start = take_event();
  hipEventRecord(*start, s);
}

void RcclComm::end_op(hipStream_t s, hipEvent_t start, int op, size_t bytes) {
  if (start == nullptr) return;
  std::lock_guard<std::mutex> lk(mu_);
  Pending p;
  p.start = start;
  p.end = take_event();
  p.op = op;
  p.bytes = bytes;
  p.t_enq = std::chrono::steady_clock::now();
  hipEventRecord(p.end, s);
  pending_.push_back(p);
}

int RcclComm::retire_locked(bool check_timeout) {
  while (!pending_.empty()) {
    Pending& p = pending_.front();
    const hipError_t q = hipEventQuery(p.end);
    if (q == hipErrorNotReady) {
      if (check_timeout && timeout_s_ > 0.0) {
        const double waited =
            std::chrono::duration<double>(std::chrono::steady_clock::now() - p.t_enq).count();
        if (waited > timeout_s_) {
          char buf[256];
          std::snprintf(buf, sizeof(buf), "rank %d: %s of %zu bytes not complete after %.1f s (world %d)", rank_,
                        op_name(p.op), p.bytes, waited, world_);
          fail(buf);
          return (int)pending_.size();
        }
      }
      break;
    }
    if (q == hipSuccess) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, p.start, p.end) == hipSuccess) {
        OpStats& st = stats_[p.op];
        st.calls += 1;
        st.bytes += p.bytes;
        st.ms_total += ms;
        if (ms > st.ms_max) st.ms_max = ms;
      }
    }
    pool_.push_back(p.start);
    pool_.push_back(p.end);
    pending_.pop_front();
  }
  return (int)pending_.size();
}

// Failure protocol (watchdog thread vs the owning thread's enqueues):
//  * fail() only marks the failure (under mu_); it never touches comm_.
//  * every collective is enqueued under enq_mu_ after check(), so once
//    failed_ is set no NEW enqueue reads comm_;
//  * abort_comm() -- outside mu_ -- waits (bounded) for an enqueue already
//    past its check() to leave enq_mu_, then aborts.  If that enqueue is
//    itself stuck inside RCCL (a dead peer during lazy connection setup) the
//    grace period ends and the abort runs concurrently with it, which is what
//    ncclCommAbort exists for (it releases blocked calls and spinning kernels).
//  * comm_ stays a valid handle value; only the owner's destroy() clears it,
//    and an aborted communicator is never destroyed again.
void RcclComm::fail(const std::string& why) {
  bool expected = false;
  if (!failed_.compare_exchange_strong(expected, true)) return;
  error_ = why;
  std::fprintf(stderr, "[gk::RcclComm] %s -- aborting the communicator\n", why.c_str());
}

void RcclComm::abort_comm() {
  if (!failed_.load() || aborted_.load()) return;
  std::unique_lock<std::mutex> ek(enq_mu_, std::defer_lock);
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(abort_grace_ms_);
  while (!ek.try_lock()) {
    if (std::chrono::steady_clock::now() >= deadline) break;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  bool expected = false;
  if (comm_ != nullptr && aborted_.compare_exchange_strong(expected, true))
    ncclCommAbort(comm_);   // releases RCCL kernels spinning on a dead peer
}

void RcclComm::inject_failure(const std::string& why) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    fail(why);
  }
  abort_comm();
}

int RcclComm::poll() {
  int left;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (comm_ != nullptr && !failed_.load()) {
      ncclResult_t st = ncclSuccess;
      if (ncclCommGetAsyncError(comm_, &st) == ncclSuccess && st != ncclSuccess && st != ncclInProgress)
        fail(std::string("asynchronous RCCL error: ") + rccl_error_string(st));
    }
    left = retire_locked(true);
  }
  abort_comm();   // no-op unless this poll (or an earlier one) failed the communicator
  return left;
}

void RcclComm::watchdog_loop() {
  hipSetDevice(device_);
  while (!stop_.load()) {
    std::this_thread::sleep_for(std::chrono::microseconds((int64_t)(poll_ms_ * 1000.0)));
    poll();
    if (failed_.load()) break;
  }
}

void RcclComm::start_watchdog(double timeout_s, double poll_ms) {
  stop_watchdog();
  timeout_s_ = timeout_s;
  poll_ms_ = poll_ms > 0.1 ? poll_ms : 0.1;
  stop_.store(false);
  watchdog_ = std::thread([this] { watchdog_loop(); });
}

void RcclComm::stop_watchdog() {
  if (watchdog_.joinable()) {
    stop_.store(true);
    watchdog_.join();
  }
}

std::string RcclComm::error() const {
  std::lock_guard<std::mutex> lk(mu_);
  return error_;
}

void RcclComm::check() const {
  if (failed_.load()) throw std::runtime_error("RCCL engine failed: " + error());
}

OpStats RcclComm::stats(int op) const {
  std::lock_guard<std::mutex> lk(mu_);
  if (op < 0 || op >= kNumOps) return OpStats();
  return stats_[op];
}

void RcclComm::reset_stats() {
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& s : stats_) s = OpStats();
}

int RcclComm::in_flight() const {
  std::lock_guard<std::mutex> lk(mu_);
  return (int)pending_.size();
}

// ---------------------------------------------------------------------------
// collectives
// ---------------------------------------------------------------------------
void RcclComm::allgather_bytes(const void* send, void* recv, size_t bytes, hipStream_t s) {
  std::lock_guard<std::mutex> ek(enq_mu_);   // see the failure protocol above fail()
  hipEvent_t st;
  begin_op(s, &st);
  settle(ncclAllGather(send, recv, bytes, ncclUint8, comm_, s), "ncclAllGather", op_timeout_s_);
  end_op(s, st, kOpAllGather, bytes);
}

void RcclComm::allgather_many(const std::vector<const void*>& sends, const std::vector<void*>& recvs,
                              const std::vector<size_t>& bytes, hipStream_t s) {
  if (sends.size() != recvs.size() || sends.size() != bytes.size())
    throw std::invalid_argument("allgather_many: list lengths differ");
  if (sends.empty()) return;
  std::lock_guard<std::mutex> ek(enq_mu_);
  hipEvent_t st;
  begin_op(s, &st);
  size_t total = 0;
  GK_NCCL_CHECK(ncclGroupStart());
  for (size_t i = 0; i < sends.size(); ++i) {
    const ncclResult_t r = ncclAllGather(sends[i], recvs[i], bytes[i], ncclUint8, comm_, s);
    if (r != ncclSuccess) {
      ncclGroupEnd();
      throw std::runtime_error(std::string("RCCL error in grouped all-gather: ") + rccl_error_string(r));
    }
    total += bytes[i];
  }
  settle(ncclGroupEnd(), "grouped ncclAllGather", op_timeout_s_);
  end_op(s, st, kOpGroup, total);
}

void RcclComm::allreduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t s) {
  std::lock_guard<std::mutex> ek(enq_mu_);
  hipEvent_t st;
  begin_op(s, &st);
  settle(ncclAllReduce(buf, buf, count, dt, op, comm_, s), "ncclAllReduce", op_timeout_s_);
  end_op(s, st, kOpAllReduce, count * dtype_bytes(dt));
}

void RcclComm::broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t s) {
  std::lock_guard<std::mutex> ek(enq_mu_);
  hipEvent_t st;
  begin_op(s, &st);
  settle(ncclBroadcast(buf, buf, count, dt, root, comm_, s), "ncclBroadcast", op_timeout_s_);
  end_op(s, st, kOpBroadcast, count * dtype_bytes(dt));   // bytes, like the other ops
}

}  // namespace gk
