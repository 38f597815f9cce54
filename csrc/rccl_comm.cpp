#include "rccl_comm.h"

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>

namespace dpt {

#define DPT_HIP_CHECK(expr)                                                                  \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess)                                                                    \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                   \
  } while (0)

#define DPT_RCCL_CHECK(expr)                                                                 \
  do {                                                                                       \
    ncclResult_t _r = (expr);                                                                \
    if (_r != ncclSuccess)                                                                   \
      throw std::runtime_error(std::string("RCCL error ") + ncclGetErrorString(_r) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                   \
  } while (0)

static ncclDataType_t to_nccl(WireType t) {
  switch (t) {
    case WireType::kF32: return ncclFloat32;
    case WireType::kBF16: return ncclBfloat16;
    case WireType::kF16: return ncclFloat16;
    case WireType::kI64: return ncclInt64;
  }
  return ncclFloat32;
}

std::string RcclComm::new_unique_id() {
  ncclUniqueId id;
  DPT_RCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

RcclComm::RcclComm(const std::string& unique_id, int rank, int world_size, int device, int min_ctas,
                   int max_ctas, double init_timeout_s)
    : rank_(rank), world_size_(world_size), device_(device), min_ctas_(min_ctas), max_ctas_(max_ctas) {
  if (unique_id.size() != sizeof(ncclUniqueId))
    throw std::invalid_argument("RcclComm: unique id must be " + std::to_string(sizeof(ncclUniqueId)) + " bytes");
  ncclUniqueId id;
  std::memcpy(&id, unique_id.data(), sizeof(id));
  DPT_HIP_CHECK(hipSetDevice(device));
  // Highest priority: bucket all-reduces should not queue behind backward kernels.
  int lo = 0, hi = 0;
  DPT_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  DPT_HIP_CHECK(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi));
  // RCCL's init is collective and blocking: a peer that failed inside its own init leaves this
  // rank blocked in bootstrap forever.  Run it on a helper thread and give up after
  // init_timeout_s (the caller then agrees on a fallback with its peers, parallel/comm.py).  A
  // thread that is still blocked is detached and marked abandoned: if its init ever returns, it
  // aborts the communicator it got (never used, and nobody else holds it to free it).
  auto st = std::make_shared<InitState>();
  std::thread worker([st, id, rank, world_size, device, min_ctas, max_ctas] {
    ncclComm_t c = nullptr;
    ncclResult_t r = ncclSuccess;
    if (hipSetDevice(device) != hipSuccess) {
      r = ncclUnhandledCudaError;
    } else if (min_ctas > 0 || max_ctas > 0) {
      // Only fields every config version since 2.14 carries are set; size/magic/version come
      // from the header's initializer and the library copies what it knows.
      ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
      if (min_ctas > 0) cfg.minCTAs = min_ctas;
      if (max_ctas > 0) cfg.maxCTAs = max_ctas;
      cfg.blocking = 1;
      r = ncclCommInitRankConfig(&c, world_size, id, rank, &cfg);
    } else {
      r = ncclCommInitRank(&c, world_size, id, rank);
    }
    std::lock_guard<std::mutex> lk(st->mu);
    if (st->abandoned) {
      // the caller gave up and already fell back: nobody will ever use or free this one
      if (c != nullptr) ncclCommAbort(c);
      c = nullptr;
    }
    st->comm = c;
    st->result = r;
    st->done = true;
    st->cv.notify_all();
  });
  std::unique_lock<std::mutex> lk(st->mu);
  const bool finished = init_timeout_s <= 0
      ? (st->cv.wait(lk, [&] { return st->done; }), true)
      : st->cv.wait_for(lk, std::chrono::duration<double>(init_timeout_s), [&] { return st->done; });
  if (!finished) {
    st->abandoned = true;   // under st->mu: the worker sees it when (if) its init returns
    lk.unlock();
    worker.detach();
    hipStreamDestroy(stream_);
    stream_ = nullptr;
    throw std::runtime_error("RcclComm: ncclCommInitRank did not complete within " +
                             std::to_string(init_timeout_s) + " s (a peer failed or never joined)");
  }
  lk.unlock();
  worker.join();
  if (st->result != ncclSuccess) {
    hipStreamDestroy(stream_);
    stream_ = nullptr;
    throw std::runtime_error(std::string("RCCL error ") + ncclGetErrorString(st->result) +
                             " in communicator init (rank " + std::to_string(rank) + ")");
  }
  comm_ = st->comm;
}

RcclComm::~RcclComm() { destroy(); }

void RcclComm::enable_watchdog(double timeout_s, double poll_s, double exit_grace_s) {
  if (watchdog_) return;
  watchdog_ = std::make_unique<StreamWatchdog>(
      "rccl rank " + std::to_string(rank_), timeout_s, poll_s, exit_grace_s, [this] { this->abort(); },
      [this] { return this->async_error(); });
}

void RcclComm::inject_async_error(const std::string& msg) {
  std::lock_guard<std::mutex> lk(inject_mu_);
  injected_error_ = msg;
}

void RcclComm::track(hipStream_t stream) {
  if (watchdog_ && !aborted_.load()) watchdog_->track(stream);
}

std::string RcclComm::async_error() const {
  {
    std::lock_guard<std::mutex> lk(inject_mu_);
    if (!injected_error_.empty()) return injected_error_;
  }
  if (comm_ == nullptr || aborted_.load()) return "";
  ncclResult_t r = ncclSuccess;
  if (ncclCommGetAsyncError(comm_, &r) != ncclSuccess) return "";
  if (r == ncclSuccess || r == ncclInProgress) return "";
  return ncclGetErrorString(r);
}

void RcclComm::check() const {
  if (watchdog_ && watchdog_->tripped())
    throw std::runtime_error("RcclComm (rank " + std::to_string(rank_) + "): " + watchdog_->reason());
  if (aborted_.load()) throw std::runtime_error("RcclComm: communicator was aborted");
}

void RcclComm::destroy() {
  if (watchdog_) watchdog_->stop();
  if (comm_ != nullptr && !aborted_.load()) {
    hipStreamSynchronize(stream_);
    ncclCommDestroy(comm_);
  }
  comm_ = nullptr;
  watchdog_.reset();
  if (stream_ != nullptr) hipStreamDestroy(stream_);
  stream_ = nullptr;
}

void RcclComm::all_reduce(void* ptr, size_t count, WireType t, hipStream_t stream) {
  if (aborted_.load() || comm_ == nullptr) throw std::runtime_error("RcclComm: communicator was aborted or destroyed");
  if (count == 0) return;
  hipStream_t s = stream;  // nullptr = the null stream, ordered like any other
  note_op(0, count, t, 0);
  DPT_RCCL_CHECK(ncclAllReduce(ptr, ptr, count, to_nccl(t), ncclSum, comm_, s));
  if (watchdog_) watchdog_->track(s);
}

void RcclComm::broadcast(void* ptr, size_t count, WireType t, int root, hipStream_t stream) {
  if (aborted_.load() || comm_ == nullptr) throw std::runtime_error("RcclComm: communicator was aborted or destroyed");
  if (count == 0) return;
  hipStream_t s = stream;  // nullptr = the null stream, ordered like any other
  note_op(1, count, t, root);
  DPT_RCCL_CHECK(ncclBroadcast(ptr, ptr, count, to_nccl(t), root, comm_, s));
  if (watchdog_) watchdog_->track(s);
}

void RcclComm::abort() {
  bool expected = false;
  if (comm_ != nullptr && aborted_.compare_exchange_strong(expected, true)) ncclCommAbort(comm_);
}

const char* rccl_version_string() {
  static std::string s;
  int v = 0;
  if (ncclGetVersion(&v) == ncclSuccess) s = std::to_string(v);
  return s.c_str();
}

}  // namespace dpt
