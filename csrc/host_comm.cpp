#include "host_comm.h"

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
                               int device)
    : all_reduce_fn_(std::move(all_reduce_fn)),
      broadcast_fn_(std::move(broadcast_fn)),
      rank_(rank),
      world_size_(world_size),
      device_(device) {
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
    hipStreamSynchronize(stream_);
    hipStreamDestroy(stream_);
    stream_ = nullptr;
  }
  if (host_ != nullptr) {
    hipHostFree(host_);
    host_ = nullptr;
    host_bytes_ = 0;
  }
}

void HostBridgeComm::check() const {
  if (aborted_) throw std::runtime_error("HostBridgeComm: communicator was aborted");
}

at::Tensor HostBridgeComm::stage_in(void* ptr, size_t count, WireType t, hipStream_t stream) {
  if (aborted_ || stream_ == nullptr) throw std::runtime_error("HostBridgeComm: aborted or destroyed");
  const size_t bytes = count * wire_bytes(t);
  if (bytes > host_bytes_) {
    if (host_ != nullptr) DPT_HIP_THROW(hipHostFree(host_));
    host_ = nullptr;
    DPT_HIP_THROW(hipHostMalloc(&host_, bytes, hipHostMallocDefault));
    host_bytes_ = bytes;
  }
  hipStream_t s = stream ? stream : stream_;
  DPT_HIP_THROW(hipMemcpyAsync(host_, ptr, bytes, hipMemcpyDeviceToHost, s));
  DPT_HIP_THROW(hipStreamSynchronize(s));
  return at::from_blob(host_, {(int64_t)count}, at::TensorOptions().dtype(to_scalar(t)));
}

void HostBridgeComm::stage_out(void* ptr, size_t count, WireType t, hipStream_t stream) {
  hipStream_t s = stream ? stream : stream_;
  DPT_HIP_THROW(hipMemcpyAsync(ptr, host_, count * wire_bytes(t), hipMemcpyHostToDevice, s));
  DPT_HIP_THROW(hipStreamSynchronize(s));  // the staging buffer is reused by the next call
}

void HostBridgeComm::all_reduce(void* ptr, size_t count, WireType t, hipStream_t stream) {
  if (count == 0) return;
  note_op(0, count, t, 0);
  at::Tensor h = stage_in(ptr, count, t, stream);
  {
    py::gil_scoped_acquire g;
    all_reduce_fn_(h);
  }
  stage_out(ptr, count, t, stream);
}

void HostBridgeComm::broadcast(void* ptr, size_t count, WireType t, int root, hipStream_t stream) {
  if (count == 0) return;
  note_op(1, count, t, root);
  at::Tensor h = stage_in(ptr, count, t, stream);
  {
    py::gil_scoped_acquire g;
    broadcast_fn_(h, root);
  }
  stage_out(ptr, count, t, stream);
}

}  // namespace dpt
