#include "watchdog.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <sstream>

namespace dpt {

static double now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

std::string WatchdogCore::poll(double now, const std::function<bool(uint64_t)>& done,
                               const std::string& async_error, std::vector<uint64_t>* completed) {
  while (!q_.empty() && done(q_.front().seq)) {
    if (completed) completed->push_back(q_.front().seq);
    q_.pop_front();
  }
  if (tripped_) return "";
  if (!async_error.empty()) {
    tripped_ = true;
    reason_ = "communicator reported an asynchronous error: " + async_error;
    return reason_;
  }
  if (!q_.empty() && now - q_.front().t > timeout_s_) {
    tripped_ = true;
    std::ostringstream os;
    os << "collective #" << q_.front().seq << " did not complete within " << timeout_s_ << " s ("
       << q_.size() << " outstanding)";
    reason_ = os.str();
    return reason_;
  }
  return "";
}

StreamWatchdog::StreamWatchdog(std::string name, double timeout_s, double poll_s, double exit_grace_s,
                               std::function<void()> on_trip, std::function<std::string()> async_error)
    : name_(std::move(name)),
      core_(timeout_s),
      poll_s_(poll_s),
      exit_grace_s_(exit_grace_s),
      on_trip_(std::move(on_trip)),
      async_error_(std::move(async_error)) {
  thread_ = std::thread([this] { loop(); });
}

StreamWatchdog::~StreamWatchdog() {
  stop();
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& kv : events_) hipEventDestroy(kv.second);
  for (auto e : pool_) hipEventDestroy(e);
  events_.clear();
  pool_.clear();
}

void StreamWatchdog::stop() {
  if (stop_.exchange(true)) return;
  cv_.notify_all();
  if (thread_.joinable()) thread_.join();
}

void StreamWatchdog::track(hipStream_t s) {
  if (stop_.load()) return;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return;
  std::lock_guard<std::mutex> lk(mu_);
  hipEvent_t e = nullptr;
  if (!pool_.empty()) {
    e = pool_.back();
    pool_.pop_back();
  } else if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
    return;
  }
  if (hipEventRecord(e, s) != hipSuccess) {
    pool_.push_back(e);
    return;
  }
  const uint64_t seq = next_seq_++;
  events_[seq] = e;
  core_.enqueue(seq, now_s());
}

std::string StreamWatchdog::reason() const {
  std::lock_guard<std::mutex> lk(mu_);
  return core_.reason();
}

size_t StreamWatchdog::outstanding() const {
  std::lock_guard<std::mutex> lk(mu_);
  return core_.outstanding();
}

uint64_t StreamWatchdog::tracked() const {
  std::lock_guard<std::mutex> lk(mu_);
  return next_seq_;
}

void StreamWatchdog::loop() {
  double tripped_at = -1.0;
  std::unique_lock<std::mutex> lk(mu_);
  while (!stop_.load()) {
    cv_.wait_for(lk, std::chrono::duration<double>(poll_s_));
    if (stop_.load()) break;
    const std::string aerr = async_error_ ? async_error_() : std::string();
    std::vector<uint64_t> completed;
    const std::string trip = core_.poll(
        now_s(),
        [this](uint64_t seq) {
          auto it = events_.find(seq);
          return it == events_.end() || hipEventQuery(it->second) == hipSuccess;
        },
        aerr, &completed);
    for (uint64_t seq : completed) {
      auto it = events_.find(seq);
      if (it != events_.end()) {
        pool_.push_back(it->second);
        events_.erase(it);
      }
    }
    if (!trip.empty()) {
      tripped_.store(true);
      tripped_at = now_s();
      std::fprintf(stderr, "[dpt watchdog %s] %s; aborting the communicator\n", name_.c_str(), trip.c_str());
      std::fflush(stderr);
      lk.unlock();
      if (on_trip_) on_trip_();
      lk.lock();
    }
    if (tripped_at >= 0.0 && exit_grace_s_ >= 0.0 && now_s() - tripped_at > exit_grace_s_) {
      std::fprintf(stderr, "[dpt watchdog %s] process still alive %.0f s after the abort; exiting\n",
                   name_.c_str(), exit_grace_s_);
      std::fflush(stderr);
      std::_Exit(75);
    }
  }
}

}  // namespace dpt
