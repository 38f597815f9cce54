#include "host_comm.h"

#include <cstdio>
#include <cstdlib>

#include <torch/extension.h>  // at::Tensor <-> torch.Tensor caster for the callbacks

#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace dpt {

#define DPT_HIP_THROW(expr)                                                                  \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess)                                                                    \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                   \
  } while (0)

static at::ScalarType to_scalar(WireType t) {
  switch (t) {
    case WireType::kF32: return at::kFloat;
    case WireType::kBF16: return at::kBFloat16;
    case WireType::kF16: return at::kHalf;
    case WireType::kI64: return at::kLong;
  }
  return at::kFloat;
}

HostBridgeComm::HostBridgeComm(py::object all_reduce_fn, py::object broadcast_fn, int rank, int world_size,
                               int device, bool async_mode, c10::intrusive_ptr<c10d::ProcessGroup> process_group)
    : all_reduce_fn_(std::move(all_reduce_fn)),
      broadcast_fn_(std::move(broadcast_fn)),
      rank_(rank),
      world_size_(world_size),
      device_(device),
      async_(async_mode),
      pg_(std::move(process_group)) {
  if (async_ && world_size > 1 && !pg_)
    throw std::invalid_argument("HostBridgeComm: async mode needs a (gloo) process group for world_size > 1");
  DPT_HIP_THROW(hipSetDevice(device));
  int lo = 0, hi = 0;
  DPT_HIP_THROW(hipDeviceGetStreamPriorityRange(&lo, &hi));
  DPT_HIP_THROW(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi));
}

HostBridgeComm::~HostBridgeComm() {
  destroy();
  py::gil_scoped_acquire g;
  all_reduce_fn_ = py::none();
  broadcast_fn_ = py::none();
}

void HostBridgeComm::destroy() {
  if (stream_ != nullptr) {
    {
      // async mode: host functions may be pending on any stream the caller used, and they read
      // the staging buffers freed below - drain the device (without the GIL: a gloo peer may
      // still need this process's Python side to reach its own matching collective)
      std::unique_ptr<py::gil_scoped_release> rel;
      if (PyGILState_Check()) rel = std::make_unique<py::gil_scoped_release>();
      if (async_) hipDeviceSynchronize();
      else hipStreamSynchronize(stream_);
    }
    hipStreamDestroy(stream_);
    stream_ = nullptr;
  }
  if (host_ != nullptr) {
    hipHostFree(host_);
    host_ = nullptr;
    host_bytes_ = 0;
  }
  if (!graph_jobs_.empty()) {
    // A graph that captured these collectives may still exist (the caller did not reset it
    // first).  Its host nodes point at the jobs and its copy nodes at the staging buffers, so
    // neither is freed: the jobs are retired (self = nullptr, a replay aborts loudly in
    // host_fn) and both are kept for the life of the process.
    static std::mutex mu;
    static std::vector<std::unique_ptr<Job>>* retired = new std::vector<std::unique_ptr<Job>>();
    std::lock_guard<std::mutex> lk(mu);
    for (auto& j : graph_jobs_) {
      j->self = nullptr;
      retired->push_back(std::move(j));
    }
    graph_jobs_.clear();
  }
  for (auto& kv : staging_)
    if (!graph_staging_.count(kv.second)) hipHostFree(kv.second);
  staging_.clear();
  graph_staging_.clear();
}

size_t HostBridgeComm::release_graph_resources() {
  const size_t n = graph_jobs_.size();
  if (n == 0) return 0;
  {
    std::unique_ptr<py::gil_scoped_release> rel;
    if (PyGILState_Check()) rel = std::make_unique<py::gil_scoped_release>();
    DPT_HIP_THROW(hipDeviceSynchronize());  // no replay still in flight
  }
  graph_jobs_.clear();
  graph_staging_.clear();  // the buffers stay cached in staging_ for eager reuse; trim may free them
  return n;
}

// Release the cached pinned buffers no captured graph references.  Only called outside capture;
// drains the device first (a host function may still be reading a buffer), without the GIL so a
// gloo peer that needs this process's Python side can still reach its matching collective.
void HostBridgeComm::trim_staging() {
  {
    std::unique_ptr<py::gil_scoped_release> rel;
    if (PyGILState_Check()) rel = std::make_unique<py::gil_scoped_release>();
    DPT_HIP_THROW(hipDeviceSynchronize());
  }
  for (auto it = staging_.begin(); it != staging_.end();) {
    if (graph_staging_.count(it->second)) {
      ++it;
      continue;
    }
    hipHostFree(it->second);
    it = staging_.erase(it);
  }
}

void HostBridgeComm::check() const {
  std::lock_guard<std::mutex> lk(err_mu_);
  if (!error_.empty()) throw std::runtime_error("HostBridgeComm: host collective failed: " + error_);
  if (aborted_) throw std::runtime_error("HostBridgeComm: communicator was aborted");
}

at::Tensor HostBridgeComm::stage_in(void* ptr, size_t count, WireType t, hipStream_t stream) {
  const size_t bytes = count * wire_bytes(t);
  if (bytes > host_bytes_) {
    if (host_ != nullptr) DPT_HIP_THROW(hipHostFree(host_));
    host_ = nullptr;
    DPT_HIP_THROW(hipHostMalloc(&host_, bytes, hipHostMallocDefault));
    host_bytes_ = bytes;
  }
  DPT_HIP_THROW(hipMemcpyAsync(host_, ptr, bytes, hipMemcpyDeviceToHost, stream));
  DPT_HIP_THROW(hipStreamSynchronize(stream));
  return at::from_blob(host_, {(int64_t)count}, at::TensorOptions().dtype(to_scalar(t)));
}

void HostBridgeComm::stage_out(void* ptr, size_t count, WireType t, hipStream_t stream) {
  DPT_HIP_THROW(hipMemcpyAsync(ptr, host_, count * wire_bytes(t), hipMemcpyHostToDevice, stream));
  DPT_HIP_THROW(hipStreamSynchronize(stream));  // the staging buffer is reused by the next call
}

void HostBridgeComm::call(int op, const at::Tensor& h, int root) {
  py::gil_scoped_acquire g;
  if (op == 0) all_reduce_fn_(h);
  else broadcast_fn_(h, root);
}

// Runs on HIP's host-function thread, between the D2H and the H2D copy of the stream.  No GIL,
// no HIP call: a blocking c10d collective on the pinned staging buffer.
void HostBridgeComm::host_fn(void* arg) {
  Job* j = static_cast<Job*>(arg);
  std::unique_ptr<Job> owned(j->persistent ? nullptr : j);  // graph jobs are reused per replay
  HostBridgeComm* self = j->self;
  if (self == nullptr) {
    std::fprintf(stderr, "HostBridgeComm: a hipGraph replayed a host collective whose communicator was "
                         "destroyed (reset the graph before closing the trainer); aborting\n");
    std::abort();
  }
  try {
    if (self->aborted_.load()) throw std::runtime_error("aborted before the collective ran");
    std::vector<at::Tensor> v{
        at::from_blob(j->host, {(int64_t)j->count}, at::TensorOptions().dtype(to_scalar(j->t)))};
    if (j->op == 0) {
      self->pg_->allreduce(v)->wait();
    } else {
      c10d::BroadcastOptions o;
      o.rootRank = j->root;
      self->pg_->broadcast(v, o)->wait();
    }
  } catch (const std::exception& e) {
    std::lock_guard<std::mutex> lk(self->err_mu_);
    if (self->error_.empty()) self->error_ = e.what();
    self->aborted_ = true;
  }
  self->completed_.fetch_add(1);
}

void HostBridgeComm::run(int op, void* ptr, size_t count, WireType t, int root, hipStream_t stream) {
  if (aborted_ || stream_ == nullptr) throw std::runtime_error("HostBridgeComm: aborted or destroyed");
  if (count == 0) return;
  note_op(op, count, t, root);
  // nullptr is the null stream (torch's default current stream), a real stream to order behind,
  // not "use the comm stream": substituting stream_ would race the caller's work.
  hipStream_t s = stream;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  DPT_HIP_THROW(hipStreamIsCapturing(s, &cap));
  const bool capturing = cap != hipStreamCaptureStatusNone;
  if (!async_) {
    // the synchronous bridge blocks on the stream, which a capture forbids: fail the capture
    // loudly (the graph engine falls back to eager) instead of recording a broken graph
    if (capturing) throw std::runtime_error("HostBridgeComm(host): a synchronous host collective cannot be captured");
    at::Tensor h = stage_in(ptr, count, t, s);
    call(op, h, root);
    stage_out(ptr, count, t, s);
    return;
  }
  if (world_size_ == 1) return;  // identity; stream order is all a caller can observe
  const size_t bytes = count * wire_bytes(t);
  const StagingKey key{ptr, bytes, s};
  if (!capturing && staging_.size() >= kMaxStaging && !staging_.count(key)) trim_staging();
  void*& buf = staging_[key];  // one pinned buffer per (tensor, size, stream): reuse is stream-ordered
  if (buf == nullptr) {
    // pinned allocation is not a stream operation a graph can record: warm up before capturing
    if (capturing) {
      staging_.erase(key);
      throw std::runtime_error("HostBridgeComm(host-async): no staging buffer for this collective yet; "
                               "run it eagerly once before capturing");
    }
    DPT_HIP_THROW(hipHostMalloc(&buf, bytes, hipHostMallocDefault));
  }
  DPT_HIP_THROW(hipMemcpyAsync(buf, ptr, bytes, hipMemcpyDeviceToHost, s));
  Job* job = new Job{this, op, root, buf, count, t, capturing};
  if (capturing) {
    graph_jobs_.emplace_back(job);  // owned here; every replay's host node reads it
    graph_staging_.insert(buf);
  }
  hipError_t e = hipLaunchHostFunc(s, &HostBridgeComm::host_fn, job);
  if (e != hipSuccess) {
    if (capturing) graph_jobs_.pop_back();
    else delete job;
    DPT_HIP_THROW(e);
  }
  DPT_HIP_THROW(hipMemcpyAsync(ptr, buf, bytes, hipMemcpyHostToDevice, s));
}

void HostBridgeComm::all_reduce(void* ptr, size_t count, WireType t, hipStream_t stream) {
  run(0, ptr, count, t, 0, stream);
}

void HostBridgeComm::broadcast(void* ptr, size_t count, WireType t, int root, hipStream_t stream) {
  run(1, ptr, count, t, root, stream);
}

}  // namespace dpt
