// ProcessGroupComm: the Collective contract (comm.h) served by a torch c10d process group on
// device memory - on ROCm the "nccl" group IS RCCL, driven by torch's ProcessGroupNCCL.
//
// Why a second RCCL-backed path next to RcclComm: RcclComm owns its communicator (unique-id
// exchange, ncclCommInitRankConfig with per-communicator CTA bounds, its own watchdog).  This
// one reuses the communicator torch already built for the default group (init_process_group
// with device_id, utils/dist.py), with torch's own watchdog and error handling.  It is
//   * the fallback when the framework communicator cannot be created (parallel/comm.py
//     make_comm: an RcclComm init failure on a new node degrades to this, loudly, instead of
//     ending the run), and
//   * an A/B arm for the framework communicator (`--comm c10d`).
//
// Ordering: the call makes `stream` (the reducer's comm stream, or the caller's) torch's current
// stream on this thread, so ProcessGroupNCCL orders the collective after the work already
// enqueued there; Work::wait() then makes that stream wait for the collective's end event
// (no host block unless TORCH_NCCL_BLOCKING_WAIT is set).  The autograd thread never blocks.
// Reference: the bucket all-reduce torch DDP issues through ProcessGroupNCCL
// (reference train_ddp.py:65,303-311).
#pragma once

#include <ATen/ATen.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>

#include <atomic>
#include <mutex>
#include <string>

#include "comm.h"

namespace dpt {

class ProcessGroupComm : public Collective {
 public:
  ProcessGroupComm(c10::intrusive_ptr<c10d::ProcessGroup> pg, int device);
  ~ProcessGroupComm() override;

  void all_reduce(void* ptr, size_t count, WireType t, hipStream_t stream) override;
  void broadcast(void* ptr, size_t count, WireType t, int root, hipStream_t stream) override;
  hipStream_t stream() const override { return stream_; }
  int rank() const override { return rank_; }
  int world_size() const override { return world_size_; }
  int device() const override { return device_; }
  void abort() override;
  void destroy() override;
  void check() const override;
  std::string kind() const override { return "c10d"; }
  std::string backend() const { return backend_; }

 private:
  void run(int op, void* ptr, size_t count, WireType t, int root, hipStream_t stream);

  c10::intrusive_ptr<c10d::ProcessGroup> pg_;
  hipStream_t stream_ = nullptr;
  int rank_ = 0, world_size_ = 1, device_ = 0;
  std::string backend_;
  std::atomic<bool> aborted_{false};
  mutable std::mutex err_mu_;
  std::string error_;
};

}  // namespace dpt
