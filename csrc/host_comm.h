// HostBridgeComm: the Collective contract (comm.h) served by a host-side collective.
//
// all_reduce / broadcast on device memory: copy the payload (behind the work already enqueued
// on the given stream) to a pinned host staging buffer, hand it to a Python callable as a CPU
// tensor of the wire dtype (typically torch.distributed over gloo), copy the result back on
// the same stream.  It exists to run the whole multi-rank GPU data path (reducer bucket events,
// comm stream, bf16 wire pack/unpack, comm-stream grad_check, steal-mode gathers, buffer
// broadcasts) with several ranks sharing one GPU, where RCCL cannot run (one device per rank),
// and as an opt-in transport (--comm host) for debugging.  It is not a performance path.
//
// Two modes:
//   * synchronous (default): the calling thread waits for the D2H copy, runs the callable and
//     waits for the H2D copy - the autograd thread is blocked for the whole collective;
//   * asynchronous (`async_mode`): like RCCL, the call only ENQUEUES on the stream: the D2H
//     copy, a host function (hipLaunchHostFunc) that runs the collective - the stream does
//     not proceed until it returns - and the H2D copy.  The calling thread returns at once, so
//     backward keeps running while the host collective is in flight and overlap / exposed
//     communication are observable on one GPU (bench.py --rehearse-shared-gpu).  The host
//     function calls a c10d ProcessGroup (gloo, CPU tensors) from C++ WITHOUT the GIL: the
//     main thread may block on the stream (tensor.item(), a D2H copy) while holding the GIL,
//     so a host function that needed it would deadlock.  The group must be one of its own
//     (parallel/comm.py) so its collectives never interleave with the main thread's; the host
//     functions of one device run in issue order, which is the same on every rank (the reducer
//     launches buckets in index order, broadcasts are issued in program order).
#pragma once

#include <ATen/ATen.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>
#include <pybind11/pybind11.h>

#include <atomic>
#include <map>
#include <memory>
#include <set>
#include <tuple>
#include <vector>
#include <mutex>
#include <string>

#include "comm.h"

namespace dpt {

class HostBridgeComm : public Collective {
 public:
  HostBridgeComm(pybind11::object all_reduce_fn, pybind11::object broadcast_fn, int rank, int world_size,
                 int device, bool async_mode = false,
                 c10::intrusive_ptr<c10d::ProcessGroup> process_group = {});
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
  std::string kind() const override { return async_ ? "host-async" : "host"; }
  bool async_mode() const { return async_; }
  // Host collectives the async host functions have completed.
  uint64_t completed() const { return completed_.load(); }
  // Free the jobs and pinned staging buffers of collectives recorded into a hipGraph.  Call it
  // once every graph that captured them is gone (engine/graph.py GraphedStep.reset); a later
  // capture records new ones.  Returns the number of jobs released.
  size_t release_graph_resources();

 private:
  struct Job {
    HostBridgeComm* self;
    int op;  // 0 all-reduce, 1 broadcast
    int root;
    void* host;
    size_t count;
    WireType t;
    // Enqueued while a hipGraph was being captured: the host node runs once per REPLAY, so the
    // job outlives every call (owned by graph_jobs_, freed by release_graph_resources()), never
    // by host_fn.  destroy() without that release retires the job with self = nullptr: a replay
    // after destroy then aborts the process with a message instead of touching freed memory.
    bool persistent;
  };
  using StagingKey = std::tuple<void*, size_t, hipStream_t>;
  // Bound on cached pinned staging buffers; past it the idle ones are released (drain first).
  static constexpr size_t kMaxStaging = 256;
  void trim_staging();
  static void host_fn(void* job);
  // D2H of `bytes` from `ptr` behind `stream`, returns the host view as a CPU tensor.
  at::Tensor stage_in(void* ptr, size_t count, WireType t, hipStream_t stream);
  void stage_out(void* ptr, size_t count, WireType t, hipStream_t stream);
  void run(int op, void* ptr, size_t count, WireType t, int root, hipStream_t stream);
  void call(int op, const at::Tensor& h, int root);

  void* host_ = nullptr;
  size_t host_bytes_ = 0;
  hipStream_t stream_ = nullptr;
  pybind11::object all_reduce_fn_, broadcast_fn_;
  int rank_, world_size_, device_;
  std::atomic<bool> aborted_{false};
  bool async_ = false;
  // async: (device ptr, bytes, stream) -> pinned buffer.  Keyed by stream too: the caching
  // allocator may hand one address to two streams, and two in-flight operations must never
  // share a staging buffer.  Buffers a captured graph references are never released.
  std::map<StagingKey, void*> staging_;
  std::set<void*> graph_staging_;
  std::vector<std::unique_ptr<Job>> graph_jobs_;
  c10::intrusive_ptr<c10d::ProcessGroup> pg_;  // async mode: the collective the host function runs
  std::atomic<uint64_t> completed_{0};
  mutable std::mutex err_mu_;
  std::string error_;
};

}  // namespace dpt
