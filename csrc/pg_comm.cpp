#include "pg_comm.h"

#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>

#include <stdexcept>
#include <string>
#include <vector>

namespace dpt {

#define DPT_PG_HIP(expr)                                                                     \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess)                                                                    \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                   \
  } while (0)

static at::ScalarType pg_scalar(WireType t) {
  switch (t) {
    case WireType::kF32: return at::kFloat;
    case WireType::kBF16: return at::kBFloat16;
    case WireType::kF16: return at::kHalf;
    case WireType::kI64: return at::kLong;
  }
  return at::kFloat;
}

ProcessGroupComm::ProcessGroupComm(c10::intrusive_ptr<c10d::ProcessGroup> pg, int device)
    : pg_(std::move(pg)), device_(device) {
  if (!pg_) throw std::invalid_argument("ProcessGroupComm: no process group");
  rank_ = pg_->getRank();
  world_size_ = pg_->getSize();
  backend_ = pg_->getBackendName();
  DPT_PG_HIP(hipSetDevice(device));
  int lo = 0, hi = 0;
  DPT_PG_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
  DPT_PG_HIP(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi));
}

ProcessGroupComm::~ProcessGroupComm() { destroy(); }

void ProcessGroupComm::destroy() {
  if (stream_ != nullptr) {
    hipStreamSynchronize(stream_);
    hipStreamDestroy(stream_);
    stream_ = nullptr;
  }
  pg_.reset();
}

void ProcessGroupComm::abort() {
  aborted_ = true;
  // torch's own watchdog owns the communicator's abort (TORCH_NCCL_ASYNC_ERROR_HANDLING);
  // this object only refuses further work
}

void ProcessGroupComm::check() const {
  std::lock_guard<std::mutex> lk(err_mu_);
  if (!error_.empty()) throw std::runtime_error("ProcessGroupComm: collective failed: " + error_);
  if (aborted_) throw std::runtime_error("ProcessGroupComm: communicator was aborted");
}

void ProcessGroupComm::run(int op, void* ptr, size_t count, WireType t, int root, hipStream_t stream) {
  if (aborted_ || !pg_) throw std::runtime_error("ProcessGroupComm: aborted or destroyed");
  if (count == 0) return;
  note_op(op, count, t, root);
  // the caller's stream becomes torch's current stream on this thread (the autograd thread for
  // bucket all-reduces): ProcessGroupNCCL orders its collective behind it and wait() joins it back
  c10::hip::HIPStreamGuard guard(c10::hip::getStreamFromExternal(stream, (c10::DeviceIndex)device_));
  std::vector<at::Tensor> v{at::from_blob(
      ptr, {(int64_t)count},
      at::TensorOptions().dtype(pg_scalar(t)).device(at::Device(at::kCUDA, (c10::DeviceIndex)device_)))};
  try {
    c10::intrusive_ptr<c10d::Work> w;
    if (op == 0) {
      w = pg_->allreduce(v);
    } else {
      c10d::BroadcastOptions o;
      o.rootRank = root;
      w = pg_->broadcast(v, o);
    }
    w->wait();
  } catch (const std::exception& e) {
    std::lock_guard<std::mutex> lk(err_mu_);
    if (error_.empty()) error_ = e.what();
    aborted_ = true;
    throw;
  }
}

void ProcessGroupComm::all_reduce(void* ptr, size_t count, WireType t, hipStream_t stream) {
  run(0, ptr, count, t, 0, stream);
}

void ProcessGroupComm::broadcast(void* ptr, size_t count, WireType t, int root, hipStream_t stream) {
  run(1, ptr, count, t, root, stream);
}

}  // namespace dpt
