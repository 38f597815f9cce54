// Framework-owned RCCL communicator (MI355X, xGMI).
//
// The reference reaches NCCL only through torch's ProcessGroupNCCL (reference
// train_ddp.py:65), which exposes no raw communicator.  The gradient
// hot path here owns its own RCCL communicator instead:
//   * bootstrap: rank 0 calls ncclGetUniqueId, the 128-byte id travels over torch's
//     TCPStore-backed process group (control plane only), every rank ncclCommInitRank;
//   * a dedicated high-priority HIP stream carries every bucket all-reduce so RCCL's
//     kernels run beside the backward kernels on the compute stream, ordered by hipEvents;
//   * buffers are persistent flat arenas (no caching-allocator recordStream bookkeeping);
//   * a StreamWatchdog (watchdog.h) enforces the timeout and polls ncclCommGetAsyncError.
// Links against torch's bundled librccl.so so one RCCL copy lives in the process (SURVEY.md
// §7.5 hard part 1).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>

#include "comm.h"
#include "watchdog.h"

namespace dpt {

class RcclComm : public Collective {
 public:
  // `min_ctas` / `max_ctas` > 0: per-communicator RCCL channel (CTA) bounds through
  // ncclCommInitRankConfig (ncclConfig_t.minCTAs / maxCTAs) - only this communicator is
  // affected, unlike the process-wide NCCL_MIN/MAX_NCHANNELS environment, which RCCL reads
  // once per process (torch's own communicator may already have read it).  0 = RCCL default.
  // `init_timeout_s` > 0 bounds the (collective, blocking) ncclCommInitRank: past it the
  // constructor throws instead of waiting forever for a peer that failed.
  RcclComm(const std::string& unique_id, int rank, int world_size, int device, int min_ctas = 0,
           int max_ctas = 0, double init_timeout_s = 0.0);
  ~RcclComm() override;
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  static std::string new_unique_id();

  void all_reduce(void* ptr, size_t count, WireType t, hipStream_t stream) override;
  void broadcast(void* ptr, size_t count, WireType t, int root, hipStream_t stream) override;

  hipStream_t stream() const override { return stream_; }
  int rank() const override { return rank_; }
  int world_size() const override { return world_size_; }
  int device() const override { return device_; }
  void abort() override;
  void destroy() override;
  void check() const override;
  std::string kind() const override { return "rccl"; }
  void track(hipStream_t stream) override;
  int min_ctas() const { return min_ctas_; }
  // The ncclComm_t as an integer: matches the "comm 0x..." of RCCL's NCCL_DEBUG=INFO init lines,
  // which is how bench.py reads the channel count this communicator actually opened.
  uintptr_t handle() const { return reinterpret_cast<uintptr_t>(comm_); }
  int max_ctas() const { return max_ctas_; }

  // Start the watchdog: a collective older than `timeout_s` (or an RCCL async error) aborts
  // the communicator; `exit_grace_s` < 0 disables the last-resort process exit.
  void enable_watchdog(double timeout_s, double poll_s, double exit_grace_s);
  bool watchdog_tripped() const { return watchdog_ && watchdog_->tripped(); }
  size_t watchdog_outstanding() const { return watchdog_ ? watchdog_->outstanding() : 0; }
  uint64_t watchdog_tracked() const { return watchdog_ ? watchdog_->tracked() : 0; }
  std::string async_error() const;
  // Test hook: make async_error() report `msg` (exercises the watchdog's async-error branch
  // without a broken peer).  Empty string clears it.
  void inject_async_error(const std::string& msg);

 private:
  struct InitState {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
    bool abandoned = false;   // the constructor timed out: a late-finishing worker aborts its comm
    ncclComm_t comm = nullptr;
    ncclResult_t result = ncclSuccess;
  };
  int min_ctas_ = 0, max_ctas_ = 0;
  std::string injected_error_;
  mutable std::mutex inject_mu_;
  ncclComm_t comm_ = nullptr;
  hipStream_t stream_ = nullptr;
  int rank_, world_size_, device_;
  std::atomic<bool> aborted_{false};
  std::unique_ptr<StreamWatchdog> watchdog_;
};

const char* rccl_version_string();

}  // namespace dpt
