// C++ gradient reducer: bucketed, backward-overlapped gradient all-reduce over RCCL.
//
// Re-provides what the reference inherits from torch's c10d Reducer (SURVEY.md §2.2 I1b,
// reducer.hpp:73,135,279,285,327,499) with an MI355X-first data layout:
//   * gradients are *views* into one flat fp32 arena ordered by bucket, so autograd's
//     AccumulateGrad writes straight into the bucket: no grad->bucket copy (K11), no
//     bucket->grad copy (K13), no per-bucket 1/world_size pass (the factor moves into the
//     fused optimizer);
//   * a post-hook on every parameter's AccumulateGrad node counts readiness; when the last
//     gradient of a bucket lands, the bucket is launched at once: hipEvent on the producing
//     stream -> the comm stream waits -> ncclAllReduce (fp32, or bf16 after a pack kernel)
//     -> non-finite check kernel into the device found_inf flag, all on the comm stream, so
//     the all-reduce and the AMP check overlap the rest of backward;
//   * at the end of backward (autograd final callback) any bucket not yet launched is
//     launched and the caller's stream waits on the comm stream's completion event: no
//     host synchronisation anywhere on the step;
//   * the observed gradient-ready order of the first backward is recorded so the Python
//     front-end can rebuild buckets in that order (torch DDP's iteration-2 rebuild).
// Steal mode (GPU): .grad is cleared before backward so AccumulateGrad hands each fresh
// gradient over without a kernel; a completed bucket is gathered into the arena with ONE
// multi-tensor launch (gather_kernels.hip) instead of one accumulate launch per parameter.
// With no communicator (world size 1) the reducer still runs locally: gather + AMP check.
// Without a GPU (gloo/CPU runs) the same bookkeeping drives a Python all-reduce callback.
#pragma once

#include <ATen/ATen.h>
#include <torch/csrc/autograd/function.h>
#include <pybind11/pybind11.h>

#include <hip/hip_runtime.h>

#include <memory>
#include <mutex>
#include <vector>

#include "comm.h"

namespace dpt {

class Reducer {
 public:
  Reducer(std::vector<at::Tensor> params, std::vector<at::Tensor> grad_views, at::Tensor flat_grad,
          std::vector<int64_t> bucket_offsets, std::vector<int64_t> bucket_numels,
          std::vector<int64_t> param_bucket, std::shared_ptr<Collective> comm,
          pybind11::object py_allreduce, int wire, at::Tensor wire_buf, at::Tensor found_inf,
          at::Tensor scale, double host_factor, bool check_inf, bool profile, bool steal_grads);
  ~Reducer();

  void prepare_for_backward();
  void mark_ready(int64_t index);
  void finalize();
  void set_require_sync(bool v) { require_sync_ = v; }
  bool require_sync() const { return require_sync_; }
  void set_check_inf(bool v) { check_inf_ = v; }
  // Next synced backward adds into the arena (it holds no_sync micro-batch gradients).
  void set_accumulate(bool v) { accumulate_ = v; }
  // Debug mode: a parameter marked ready twice in one backward, or a bucket
  // launched twice, raises instead of being tolerated.
  void set_debug(bool v) { debug_ = v; }
  bool debug() const { return debug_; }
  std::vector<int64_t> ready_order() const { return ready_order_; }
  int64_t num_buckets() const { return (int64_t)bucket_offsets_.size(); }
  int64_t backward_count() const { return backward_count_; }
  // Profiling (profile=true): every backward records its events into slot
  // (backward_count % profile_slots), so a window of up to `profile_slots` steps can run without
  // host synchronisation and be read afterwards.  slot < 0: the last finished backward.
  // Per bucket {comm start->done ms}, plus {first grad ready->bwd end, bwd_end->comm_done ms
  // (exposed), first bucket start->comm done (comm span)}.
  void set_profile_slots(int64_t n);
  int64_t profile_slots() const { return slots_; }
  int64_t last_slot() const { return backward_count_ > 0 ? (backward_count_ - 1) % slots_ : -1; }
  std::vector<double> bucket_times_ms(int64_t slot = -1);
  std::vector<double> step_times_ms(int64_t slot = -1);
  // Per bucket: first gradient ready -> the bucket's collective starts on the comm stream (its
  // ready time when the comm stream is idle, e.g. a 1-rank communicator).  -1 = not complete.
  std::vector<double> bucket_start_ms(int64_t slot = -1);
  void remove_hooks();

 private:
  void launch_bucket(int64_t b);
  void gather_bucket(int64_t b, hipStream_t s);

  std::vector<at::Tensor> params_, grad_views_;
  at::Tensor flat_grad_, wire_buf_, found_inf_, scale_;
  std::vector<int64_t> bucket_offsets_, bucket_numels_, param_bucket_;
  std::vector<int64_t> bucket_size_;      // params per bucket
  std::vector<int64_t> pending_;          // params still missing per bucket
  std::vector<char> launched_, marked_;
  std::vector<int64_t> ready_order_;
  std::vector<std::shared_ptr<torch::autograd::Node>> accumulators_;
  std::vector<uintptr_t> hook_keys_;
  std::shared_ptr<Collective> comm_;
  pybind11::object py_allreduce_;
  int wire_;
  float host_factor_;
  bool check_inf_, profile_, gpu_, steal_ = false, accumulate_ = false, debug_ = false;
  std::vector<at::Tensor> stolen_;        // gradients autograd handed over (steal mode)
  std::vector<std::vector<int64_t>> members_;
  bool require_sync_ = true;
  bool callback_queued_ = false;
  bool record_order_ = true;
  int64_t next_launch_ = 0;  // buckets launch strictly in index order (RCCL needs one global order)
  int64_t backward_count_ = 0;
  hipStream_t caller_stream_ = nullptr;
  void create_profile_events();
  void destroy_profile_events();
  std::vector<hipEvent_t> ev_ready_;
  // profiling events: [slot * B + b] per bucket, [slot] per backward
  std::vector<hipEvent_t> ev_start_, ev_end_, ev_bwd_end_, ev_done_, ev_first_;
  hipEvent_t ev_join_ = nullptr;   // comm-stream completion the caller's stream waits on
  int64_t slots_ = 1, slot_ = 0;
  std::mutex mu_;
};

}  // namespace dpt
