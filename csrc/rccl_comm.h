// Framework-owned RCCL communicator (MI355X, xGMI).
//
// The reference reaches NCCL only through torch's ProcessGroupNCCL (reference
// train_ddp.py:65), which exposes no raw communicator.  The gradient
// hot path here owns its own RCCL communicator instead:
//   * bootstrap: rank 0 calls ncclGetUniqueId, the 128-byte id travels over torch's
//     TCPStore-backed process group (control plane only), every rank ncclCommInitRank;
//   * a dedicated high-priority HIP stream carries every bucket all-reduce so RCCL's
//     kernels run beside the backward kernels on the compute stream, ordered by hipEvents;
//   * buffers are persistent flat arenas (no caching-allocator recordStream bookkeeping).
// Links against torch's bundled librccl.so so one RCCL copy lives in the process (SURVEY.md
// §7.5 hard part 1).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <string>

namespace dpt {

enum class WireType { kF32 = 0, kBF16 = 1, kF16 = 2, kI64 = 3 };

class RcclComm {
 public:
  RcclComm(const std::string& unique_id, int rank, int world_size, int device);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  static std::string new_unique_id();

  // In-place SUM all-reduce of `count` elements at `ptr`, enqueued on `stream`.
  void all_reduce(void* ptr, size_t count, WireType t, hipStream_t stream);
  void broadcast(void* ptr, size_t count, WireType t, int root, hipStream_t stream);

  hipStream_t stream() const { return stream_; }
  int rank() const { return rank_; }
  int world_size() const { return world_size_; }
  int device() const { return device_; }
  // Abort outstanding operations (failure path); the object is unusable after.
  void abort();
  // Orderly teardown (idempotent): destroy the communicator and its stream now, not at
  // interpreter exit when the HIP runtime may already be gone.
  void destroy();

 private:
  ncclComm_t comm_ = nullptr;
  hipStream_t stream_ = nullptr;
  int rank_, world_size_, device_;
  bool aborted_ = false;
};

const char* rccl_version_string();

}  // namespace dpt
