// HostBridgeComm: the Collective contract (comm.h) served by a host-side collective.
//
// all_reduce / broadcast on device memory: wait for the work enqueued on the given stream,
// copy the payload to a pinned host staging buffer, hand it to a Python callable as a CPU
// tensor of the wire dtype (typically torch.distributed over gloo), copy the result back on
// the same stream and wait for it.  Synchronous by construction - it exists to run the whole
// multi-rank GPU data path (reducer bucket events, comm stream, bf16 wire pack/unpack,
// comm-stream grad_check, steal-mode gathers, buffer broadcasts) with several ranks sharing
// one GPU, where RCCL cannot run (one device per rank), and as an opt-in transport
// (--comm host) for debugging.  It is not a performance path.
#pragma once

#include <ATen/ATen.h>
#include <pybind11/pybind11.h>

#include "comm.h"

namespace dpt {

class HostBridgeComm : public Collective {
 public:
  HostBridgeComm(pybind11::object all_reduce_fn, pybind11::object broadcast_fn, int rank, int world_size,
                 int device);
  ~HostBridgeComm() override;

  void all_reduce(void* ptr, size_t count, WireType t, hipStream_t stream) override;
  void broadcast(void* ptr, size_t count, WireType t, int root, hipStream_t stream) override;
  hipStream_t stream() const override { return stream_; }
  int rank() const override { return rank_; }
  int world_size() const override { return world_size_; }
  int device() const override { return device_; }
  void abort() override { aborted_ = true; }
  void destroy() override;
  void check() const override;
  std::string kind() const override { return "host"; }

 private:
  // D2H of `bytes` from `ptr` behind `stream`, returns the host view as a CPU tensor.
  at::Tensor stage_in(void* ptr, size_t count, WireType t, hipStream_t stream);
  void stage_out(void* ptr, size_t count, WireType t, hipStream_t stream);
  void* host_ = nullptr;
  size_t host_bytes_ = 0;
  hipStream_t stream_ = nullptr;
  pybind11::object all_reduce_fn_, broadcast_fn_;
  int rank_, world_size_, device_;
  bool aborted_ = false;
};

}  // namespace dpt
