#include "reducer.h"

#include <c10/hip/HIPStream.h>
#include <torch/csrc/autograd/engine.h>
#include <torch/csrc/autograd/utils/lambda_post_hook.h>
#include <torch/csrc/autograd/variable.h>

#include <cstdlib>
#include <stdexcept>

#include "kernels/kernels.h"

namespace py = pybind11;

namespace dpt {

#define DPT_HIP_OK(expr)                                                                     \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess)                                                                    \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                   \
  } while (0)

Reducer::Reducer(std::vector<at::Tensor> params, std::vector<at::Tensor> grad_views,
                 at::Tensor flat_grad, std::vector<int64_t> bucket_offsets,
                 std::vector<int64_t> bucket_numels, std::vector<int64_t> param_bucket,
                 std::shared_ptr<Collective> comm, py::object py_allreduce, int wire,
                 at::Tensor wire_buf, at::Tensor found_inf, at::Tensor scale, double host_factor,
                 bool check_inf, bool profile, bool steal_grads)
    : params_(std::move(params)),
      grad_views_(std::move(grad_views)),
      flat_grad_(std::move(flat_grad)),
      wire_buf_(std::move(wire_buf)),
      found_inf_(std::move(found_inf)),
      scale_(std::move(scale)),
      bucket_offsets_(std::move(bucket_offsets)),
      bucket_numels_(std::move(bucket_numels)),
      param_bucket_(std::move(param_bucket)),
      comm_(std::move(comm)),
      py_allreduce_(std::move(py_allreduce)),
      wire_(wire),
      host_factor_((float)host_factor),
      check_inf_(check_inf),
      profile_(profile) {
  const size_t P = params_.size(), B = bucket_offsets_.size();
  if (grad_views_.size() != P || param_bucket_.size() != P || bucket_numels_.size() != B)
    throw std::invalid_argument("Reducer: inconsistent parameter/bucket metadata");
  gpu_ = flat_grad_.is_cuda();
  steal_ = steal_grads && gpu_;
  // gpu_ && !comm_: local reducer (world size 1): gather + AMP check, no collectives.
  if (!gpu_ && py_allreduce_.is_none())
    throw std::invalid_argument("Reducer: CPU arena needs a Python all-reduce callback");
  if (gpu_ && wire_ == 1 && (!wire_buf_.defined() || wire_buf_.numel() < flat_grad_.numel()))
    throw std::invalid_argument("Reducer: bf16 wire needs a wire buffer as large as the arena");
  for (size_t b = 0; b < B; ++b) {
    if (bucket_offsets_[b] < 0 || bucket_offsets_[b] + bucket_numels_[b] > flat_grad_.numel())
      throw std::invalid_argument("Reducer: bucket out of arena bounds");
    if (gpu_ && (bucket_offsets_[b] % 8 != 0 || bucket_numels_[b] % 8 != 0))
      throw std::invalid_argument("Reducer: GPU buckets must be 8-element aligned");
  }
  bucket_size_.assign(B, 0);
  for (size_t i = 0; i < P; ++i) {
    if (param_bucket_[i] < 0 || param_bucket_[i] >= (int64_t)B)
      throw std::invalid_argument("Reducer: parameter mapped to a missing bucket");
    bucket_size_[param_bucket_[i]]++;
  }
  pending_ = bucket_size_;
  launched_.assign(B, 0);
  marked_.assign(P, 0);
  stolen_.resize(P);
  members_.assign(B, {});
  for (size_t i = 0; i < P; ++i) members_[param_bucket_[i]].push_back((int64_t)i);
  if (steal_ && flat_grad_.scalar_type() != at::kFloat)
    throw std::invalid_argument("Reducer: steal mode needs a float32 arena");

  if (gpu_) {
    ev_ready_.resize(B);
    for (auto& e : ev_ready_) DPT_HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    DPT_HIP_OK(hipEventCreateWithFlags(&ev_join_, hipEventDisableTiming));
    if (profile_) create_profile_events();
  }

  // One post-hook per parameter on its AccumulateGrad node: fires after the gradient has
  // been accumulated into the arena view.
  for (size_t i = 0; i < P; ++i) {
    auto acc = torch::autograd::impl::grad_accumulator(params_[i]);
    if (!acc) throw std::invalid_argument("Reducer: parameter without a gradient accumulator");
    const int64_t idx = (int64_t)i;
    auto key = acc->add_post_hook(std::make_unique<torch::autograd::utils::LambdaPostHook>(
        [this, idx](const torch::autograd::variable_list& outputs,
                    const torch::autograd::variable_list& /*inputs*/) {
          this->mark_ready(idx);
          return outputs;
        }));
    accumulators_.push_back(std::move(acc));
    hook_keys_.push_back(key);
  }
}

void Reducer::remove_hooks() {
  for (size_t i = 0; i < accumulators_.size(); ++i) accumulators_[i]->del_post_hook(hook_keys_[i]);
  accumulators_.clear();
  hook_keys_.clear();
}

void Reducer::create_profile_events() {
  const size_t B = bucket_offsets_.size(), S = (size_t)slots_;
  auto make = [](std::vector<hipEvent_t>& v, size_t n) {
    v.resize(n);
    for (auto& e : v) DPT_HIP_OK(hipEventCreateWithFlags(&e, hipEventDefault));
  };
  make(ev_start_, S * B);
  make(ev_end_, S * B);
  make(ev_bwd_end_, S);
  make(ev_done_, S);
  make(ev_first_, S);
}

void Reducer::destroy_profile_events() {
  for (auto* v : {&ev_start_, &ev_end_, &ev_bwd_end_, &ev_done_, &ev_first_}) {
    for (auto e : *v) hipEventDestroy(e);
    v->clear();
  }
}

void Reducer::set_profile_slots(int64_t n) {
  if (n < 1) throw std::invalid_argument("Reducer: profile_slots must be >= 1");
  std::lock_guard<std::mutex> lk(mu_);
  if (!gpu_ || !profile_) {
    slots_ = n;
    return;
  }
  DPT_HIP_OK(hipDeviceSynchronize());  // no event of the old set may still be pending
  destroy_profile_events();
  slots_ = n;
  create_profile_events();
}

Reducer::~Reducer() {
  remove_hooks();
  if (gpu_) {
    for (auto e : ev_ready_) hipEventDestroy(e);
    if (ev_join_) hipEventDestroy(ev_join_);
    destroy_profile_events();
  }
  if (!py_allreduce_.is_none()) {
    py::gil_scoped_acquire g;
    py_allreduce_ = py::none();
  }
}

void Reducer::prepare_for_backward() {
  std::lock_guard<std::mutex> lk(mu_);
  pending_ = bucket_size_;
  std::fill(launched_.begin(), launched_.end(), 0);
  std::fill(marked_.begin(), marked_.end(), 0);
  next_launch_ = 0;
  callback_queued_ = false;
  slot_ = backward_count_ % slots_;
  if (record_order_) ready_order_.clear();
  if (gpu_) caller_stream_ = c10::hip::getCurrentHIPStream(flat_grad_.device().index()).stream();
  if (steal_) {
    // Undefined .grad: AccumulateGrad steals the fresh gradient (no per-parameter kernel).
    for (size_t i = 0; i < params_.size(); ++i) params_[i].mutable_grad().reset();
    return;
  }
  // Re-attach arena views if someone replaced or cleared .grad (e.g. zero_grad(set_to_none)).
  for (size_t i = 0; i < params_.size(); ++i) {
    const at::Tensor& g = params_[i].grad();
    if (!g.defined() || g.data_ptr() != grad_views_[i].data_ptr()) {
      if (g.defined()) grad_views_[i].copy_(g);
      else grad_views_[i].zero_();
      params_[i].mutable_grad() = grad_views_[i];
    }
  }
}

void Reducer::mark_ready(int64_t index) {
  if (!require_sync_) return;
  std::lock_guard<std::mutex> lk(mu_);
  if (marked_[index]) {  // second accumulation in one backward: already counted
    if (debug_)
      throw std::runtime_error("Reducer(debug): parameter " + std::to_string(index) +
                               " marked ready twice in one backward (reentrant backward or a "
                               "second backward without a forward?)");
    return;
  }
  marked_[index] = 1;
  if (record_order_) ready_order_.push_back(index);
  if (!callback_queued_) {
    callback_queued_ = true;
    if (gpu_ && profile_) DPT_HIP_OK(hipEventRecord(ev_first_[slot_], caller_stream_));
    torch::autograd::Engine::get_default_engine().queue_callback([this] { this->finalize(); });
  }
  if (steal_) stolen_[index] = params_[index].grad();
  const int64_t b = param_bucket_[index];
  if (debug_ && launched_[b] == 2)
    throw std::runtime_error("Reducer(debug): gradient of parameter " + std::to_string(index) +
                             " arrived after its bucket " + std::to_string(b) +
                             " was already all-reduced (it would be missing from the sum)");
  if (--pending_[b] == 0) {
    if (gpu_) {
      // The gradient was produced on this thread's current stream.
      hipStream_t producer = c10::hip::getCurrentHIPStream(flat_grad_.device().index()).stream();
      if (steal_) gather_bucket(b, producer);
      DPT_HIP_OK(hipEventRecord(ev_ready_[b], producer));
    }
    launched_[b] = 1;  // "ready"; the launch itself happens in index order below
    while (next_launch_ < (int64_t)launched_.size() && launched_[next_launch_] == 1) {
      launch_bucket(next_launch_);
      launched_[next_launch_] = 2;
      ++next_launch_;
    }
  }
}

// Same element order in memory: both dense, equal strides on every dimension longer than 1
// (AccumulateGrad's layout contract ignores size-1 dimensions, so a 1x1 conv weight's gradient
// may arrive with strides (C,1,1,1) for a channels_last (C,1,C,C) parameter - the same bytes).
static bool same_dense_layout(const at::Tensor& g, const at::Tensor& v) {
  if (!g.is_non_overlapping_and_dense() || !v.is_non_overlapping_and_dense()) return false;
  for (int64_t d = 0; d < g.dim(); ++d)
    if (g.size(d) > 1 && g.stride(d) != v.stride(d)) return false;
  return true;
}

// Move the stolen gradients of bucket b into the arena (one launch per <= kGatherMax
// tensors).  Gradients whose layout differs from their arena view (rare: a non-dense or
// differently-strided gradient) go through a strided copy instead; parameters that got no
// gradient this backward have their region zeroed unless accumulating.
void Reducer::gather_bucket(int64_t b, hipStream_t s) {
  GatherBatch batch;
  batch.count = 0;
  for (int64_t i : members_[b]) {
    at::Tensor& g = stolen_[i];
    const at::Tensor& v = grad_views_[i];
    if (!g.defined()) {
      if (!accumulate_) DPT_HIP_OK(hipMemsetAsync(v.data_ptr<float>(), 0, v.numel() * sizeof(float), s));
      continue;
    }
    const auto dt = g.scalar_type();
    const int kind = dt == at::kFloat ? 0 : dt == at::kBFloat16 ? 1 : dt == at::kHalf ? 2 : -1;
    const bool same = kind >= 0 && g.is_cuda() && g.sizes() == v.sizes() && same_dense_layout(g, v);
    if (!same) {
      at::Tensor vv = v;  // strided / odd-dtype fallback on the current stream
      if (accumulate_) vv.add_(g.to(at::kFloat));
      else vv.copy_(g);
      continue;
    }
    batch.src[batch.count] = g.data_ptr();
    batch.dst[batch.count] = v.data_ptr<float>();
    batch.numel[batch.count] = v.numel();
    batch.kind[batch.count] = (int8_t)kind;
    if (++batch.count == kGatherMax) {
      launch_gather(batch, accumulate_, s);
      batch.count = 0;
    }
  }
  launch_gather(batch, accumulate_, s);
}

void Reducer::launch_bucket(int64_t b) {
  const int64_t off = bucket_offsets_[b], n = bucket_numels_[b];
  if (!gpu_) {
    py::gil_scoped_acquire g;
    py_allreduce_(b, off, n);
    return;
  }
  if (!comm_) {  // local reducer: the AMP check runs right behind the gather, same stream
    const float* scale = (scale_.defined() && scale_.numel() > 0) ? scale_.data_ptr<float>() : nullptr;
    hipStream_t producer = c10::hip::getCurrentHIPStream(flat_grad_.device().index()).stream();
    if (check_inf_) launch_grad_check(flat_grad_.data_ptr<float>() + off, n, scale, host_factor_,
                                      found_inf_.data_ptr<float>(), producer);
    return;
  }
  hipStream_t cs = comm_->stream();
  DPT_HIP_OK(hipStreamWaitEvent(cs, ev_ready_[b], 0));
  const size_t pe = (size_t)slot_ * bucket_offsets_.size() + (size_t)b;
  if (profile_) DPT_HIP_OK(hipEventRecord(ev_start_[pe], cs));
  float* g = flat_grad_.data_ptr<float>() + off;
  const float* scale = (scale_.defined() && scale_.numel() > 0) ? scale_.data_ptr<float>() : nullptr;
  float* finf = check_inf_ ? found_inf_.data_ptr<float>() : nullptr;
  // DPT_FORCE_COLLECTIVES=1 runs the RCCL path even at world size 1 (single-GPU tests of the
  // collective + wire-format code path; a 1-rank all-reduce is an identity).
  static const bool force = [] {
    const char* e = std::getenv("DPT_FORCE_COLLECTIVES");
    return e != nullptr && e[0] == '1';
  }();
  if (comm_->world_size() > 1 || force) {
    if (wire_ == 1) {
      uint16_t* w = reinterpret_cast<uint16_t*>(wire_buf_.data_ptr()) + off;
      launch_pack_bf16(g, w, n, cs);
      comm_->all_reduce(w, (size_t)n, WireType::kBF16, cs);
      launch_unpack_bf16(w, g, n, scale, host_factor_, finf, cs);
    } else {
      comm_->all_reduce(g, (size_t)n, WireType::kF32, cs);
      if (finf) launch_grad_check(g, n, scale, host_factor_, finf, cs);
    }
  } else if (finf) {
    launch_grad_check(g, n, scale, host_factor_, finf, cs);
  }
  if (profile_) DPT_HIP_OK(hipEventRecord(ev_end_[pe], cs));
}

void Reducer::finalize() {
  std::lock_guard<std::mutex> lk(mu_);
  // Buckets whose parameters received no gradient this backward (unused parameters) are
  // still reduced, in order, so every rank issues the same collective sequence.
  if (gpu_) {
    hipStream_t producer = c10::hip::getCurrentHIPStream(flat_grad_.device().index()).stream();
    for (size_t b = 0; b < launched_.size(); ++b) {
      if (launched_[b] == 0) {
        if (steal_) gather_bucket((int64_t)b, producer);
        DPT_HIP_OK(hipEventRecord(ev_ready_[b], producer));
      }
    }
    if (profile_) DPT_HIP_OK(hipEventRecord(ev_bwd_end_[slot_], caller_stream_));
  }
  for (size_t b = 0; b < launched_.size(); ++b) {
    if (launched_[b] != 2) {
      launch_bucket((int64_t)b);
      launched_[b] = 2;
    }
  }
  next_launch_ = (int64_t)launched_.size();
  if (gpu_ && comm_) {
    if (profile_) DPT_HIP_OK(hipEventRecord(ev_done_[slot_], comm_->stream()));
    DPT_HIP_OK(hipEventRecord(ev_join_, comm_->stream()));
    DPT_HIP_OK(hipStreamWaitEvent(caller_stream_, ev_join_, 0));
  } else if (gpu_ && profile_) {
    DPT_HIP_OK(hipEventRecord(ev_done_[slot_], caller_stream_));
  }
  if (steal_) {
    // Hand the arena views back as .grad and drop the stolen tensors (their memory returns to
    // the caching allocator stream-ordered behind the gather kernels).
    for (size_t i = 0; i < params_.size(); ++i) {
      // fp32 parameters get their arena view back as .grad; 16-bit weight-shadow leaves
      // keep an undefined .grad (their gradient lives, converted, in the fp32 arena).
      if (params_[i].scalar_type() == at::kFloat) params_[i].mutable_grad() = grad_views_[i];
      stolen_[i].reset();
    }
  }
  accumulate_ = false;
  if (record_order_ && !ready_order_.empty()) record_order_ = false;
  ++backward_count_;
}

std::vector<double> Reducer::bucket_times_ms(int64_t slot) {
  std::vector<double> out;
  if (!gpu_ || !profile_ || !comm_ || backward_count_ == 0) return out;
  if (slot < 0) slot = last_slot();
  const size_t B = bucket_offsets_.size();
  for (size_t b = 0; b < B; ++b) {
    float ms = 0.f;
    const size_t pe = (size_t)(slot % slots_) * B + b;
    if (hipEventElapsedTime(&ms, ev_start_[pe], ev_end_[pe]) != hipSuccess) ms = -1.f;
    out.push_back(ms);
  }
  (void)hipGetLastError();  // a not-yet-complete event leaves hipErrorNotReady pending: clear it
  return out;
}

std::vector<double> Reducer::bucket_start_ms(int64_t slot) {
  std::vector<double> out;
  if (!gpu_ || !profile_ || !comm_ || backward_count_ == 0) return out;
  if (slot < 0) slot = last_slot();
  const size_t s = (size_t)(slot % slots_), B = bucket_offsets_.size();
  for (size_t b = 0; b < B; ++b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, ev_first_[s], ev_start_[s * B + b]) != hipSuccess) ms = -1.f;
    out.push_back(ms);
  }
  (void)hipGetLastError();
  return out;
}

std::vector<double> Reducer::step_times_ms(int64_t slot) {
  // {first-grad-ready -> backward end, backward end -> comm done (exposed), first bucket
  //  start -> comm done (comm span)}
  std::vector<double> out;
  if (!gpu_ || !profile_ || ev_start_.empty() || !comm_ || backward_count_ == 0) return out;
  if (slot < 0) slot = last_slot();
  const size_t s = (size_t)(slot % slots_), B = bucket_offsets_.size();
  float a = 0.f, b = 0.f, c = 0.f;
  // -1 marks a pair that is not complete yet (the caller read the slot too early)
  if (hipEventElapsedTime(&a, ev_first_[s], ev_bwd_end_[s]) != hipSuccess) a = -1.f;
  if (hipEventElapsedTime(&b, ev_bwd_end_[s], ev_done_[s]) != hipSuccess) b = -1.f;
  if (hipEventElapsedTime(&c, ev_start_[s * B], ev_done_[s]) != hipSuccess) c = -1.f;
  (void)hipGetLastError();
  out = {a, b, c};
  return out;
}

}  // namespace dpt
