// Watchdog for the framework-owned communicator.
//
// In the reference every collective runs on torch's ProcessGroupNCCL, whose watchdog thread
// enforces the process-group timeout (reference train_ddp.py:65 takes the defaults).  The
// gradient all-reduces here run on a communicator torch never sees, so it gets its own:
//   * every collective enqueued on the comm stream is followed by a hipEvent (outside
//     hipGraph capture) and queued with its enqueue time;
//   * a background thread pops completed events in FIFO order (one stream => in-order
//     completion) and polls the backend's asynchronous error (ncclCommGetAsyncError);
//   * when the oldest outstanding collective is older than the timeout, or the backend
//     reports an error, it trips ONCE: records the reason, aborts the communicator
//     (ncclCommAbort makes the spinning RCCL kernels exit so the device drains), and from then
//     on every host touch point (Collective::check(): print boundaries, epoch end, close)
//     throws; if the process is still alive `exit_grace_s` later (main thread wedged in a
//     synchronize) the thread ends it with exit code 75.
// The decision logic lives in WatchdogCore with an explicit clock and completion predicate,
// so it is unit-tested with a fake clock on CPU (tests/test_watchdog.py).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace dpt {

class WatchdogCore {
 public:
  explicit WatchdogCore(double timeout_s) : timeout_s_(timeout_s) {}
  void enqueue(uint64_t seq, double now) { q_.push_back({seq, now}); }
  // Pops completed items (front first); returns the trip reason the first time it trips,
  // "" otherwise.  `done(seq)`: completion of item seq; `async_error`: "" or a backend error.
  std::string poll(double now, const std::function<bool(uint64_t)>& done, const std::string& async_error,
                   std::vector<uint64_t>* completed = nullptr);
  bool tripped() const { return tripped_; }
  const std::string& reason() const { return reason_; }
  size_t outstanding() const { return q_.size(); }
  double timeout_s() const { return timeout_s_; }
  // Age of the oldest outstanding item (0 when idle).
  double oldest_age(double now) const { return q_.empty() ? 0.0 : now - q_.front().t; }

 private:
  struct Item {
    uint64_t seq;
    double t;
  };
  std::deque<Item> q_;
  double timeout_s_;
  bool tripped_ = false;
  std::string reason_;
};

class StreamWatchdog {
 public:
  // on_trip: called once from the watchdog thread (abort the communicator).
  // async_error: polled every period ("" = healthy).
  StreamWatchdog(std::string name, double timeout_s, double poll_s, double exit_grace_s,
                 std::function<void()> on_trip, std::function<std::string()> async_error);
  ~StreamWatchdog();
  // Record a completion event behind the work just enqueued on `s` (no-op while `s` is being
  // captured into a hipGraph: a captured event only completes at replay).
  void track(hipStream_t s);
  void stop();
  bool tripped() const { return tripped_.load(); }
  std::string reason() const;
  size_t outstanding() const;
  // Completion markers handed to the watchdog so far (retired = tracked - outstanding).
  uint64_t tracked() const;

 private:
  void loop();
  std::string name_;
  WatchdogCore core_;
  double poll_s_, exit_grace_s_;
  std::function<void()> on_trip_;
  std::function<std::string()> async_error_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::unordered_map<uint64_t, hipEvent_t> events_;
  std::vector<hipEvent_t> pool_;
  uint64_t next_seq_ = 0;
  std::atomic<bool> tripped_{false}, stop_{false};
  std::thread thread_;
};

}  // namespace dpt
