// The collective seam of the gradient hot path.
//
// The C++ reducer (reducer.h) and the DDP front-end's buffer broadcasts talk to a
// `Collective`: an in-place SUM all-reduce and a broadcast of device memory, enqueued behind
// a given HIP stream.  Two implementations:
//   * RcclComm (rccl_comm.h)       - the production path: RCCL over xGMI on a dedicated
//                                    high-priority comm stream, with a watchdog;
//   * HostBridgeComm (host_comm.h) - the same device-pointer contract served by a host
//                                    collective (D2H -> Python callback, e.g. gloo -> H2D),
//                                    so several processes can share ONE GPU and still run
//                                    every line of the multi-rank GPU data path (event
//                                    ordering, comm stream, bf16 wire pack/unpack, the
//                                    comm-stream non-finite check, steal-mode gathers,
//                                    buffer broadcasts) except the ncclAllReduce call itself.
// The reference reaches all of this through torch DDP over ProcessGroupNCCL
// (reference train_ddp.py:65,303-311).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <string>

namespace dpt {

enum class WireType { kF32 = 0, kBF16 = 1, kF16 = 2, kI64 = 3 };

inline size_t wire_bytes(WireType t) {
  switch (t) {
    case WireType::kF32: return 4;
    case WireType::kBF16: return 2;
    case WireType::kF16: return 2;
    case WireType::kI64: return 8;
  }
  return 4;
}

class Collective {
 public:
  virtual ~Collective() = default;
  // In-place SUM all-reduce of `count` elements at device pointer `ptr`, ordered after the
  // work already enqueued on `stream` (and, for asynchronous backends, enqueued on it).
  // `stream` is used as given: nullptr is the null stream (torch's default current stream on
  // ROCm), never a request for the comm stream - substituting stream() would race the caller.
  virtual void all_reduce(void* ptr, size_t count, WireType t, hipStream_t stream) = 0;
  virtual void broadcast(void* ptr, size_t count, WireType t, int root, hipStream_t stream) = 0;
  // The stream bucket collectives are issued on (the reducer orders it behind the producer
  // stream with events and joins it back at the end of backward).
  virtual hipStream_t stream() const = 0;
  virtual int rank() const = 0;
  virtual int world_size() const = 0;
  virtual int device() const = 0;
  // Failure path: abort outstanding operations; unusable afterwards.
  virtual void abort() = 0;
  // Orderly, idempotent teardown.
  virtual void destroy() = 0;
  // Host touch point: throws if the watchdog (or the backend) recorded an error.
  virtual void check() const {}
  virtual std::string kind() const = 0;
  // Hand the watchdog (if any) a completion marker for the work enqueued on `stream` so far:
  // collectives replayed from a captured hipGraph are not seen by all_reduce()/broadcast(),
  // so the graph engine calls this after every replay.  No-op for backends without one.
  virtual void track(hipStream_t /*stream*/) {}
  // Collectives issued so far and a running hash of their (kind, count, dtype, root)
  // sequence: compared across ranks by the debug sequence check (parallel/ddp.py).  Written
  // by the autograd thread (reducer, under its mutex), read by the main thread: atomics.
  uint64_t ops() const { return ops_.load(std::memory_order_acquire); }
  uint64_t sequence_hash() const { return seq_hash_.load(std::memory_order_acquire); }

 protected:
  void note_op(int kind, size_t count, WireType t, int root) {
    uint64_t v = ((uint64_t)kind << 56) ^ ((uint64_t)(int)t << 48) ^ ((uint64_t)(root & 0xff) << 40) ^ (uint64_t)count;
    // single writer at a time (callers are serialised); FNV-1a style running hash
    seq_hash_.store((seq_hash_.load(std::memory_order_relaxed) ^ v) * 0x100000001b3ull, std::memory_order_release);
    ops_.fetch_add(1, std::memory_order_release);
  }
  std::atomic<uint64_t> ops_{0}, seq_hash_{0xcbf29ce484222325ull};
};

}  // namespace dpt
