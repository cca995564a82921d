// Native request queue of the serving scheduler (runtime/scheduler.py).
//
// The reference serves every /generate on its own FastAPI threadpool thread
// with no shared queue at all (`server.py:154-210`): concurrent
// requests never batch.  Here producers (HTTP handler threads) push request
// ids; ONE scheduler thread pops them as rounds:
//
//   next_groups(window): block until a request arrives (or close()), keep
//   collecting for up to `window` seconds or until `max_batch` requests, then
//   split the batch into generation-length groups (sorted by max_new_tokens;
//   a group spans at most `length_ratio` x its shortest request, because a
//   pipeline round runs max(max_new_tokens) steps for all its sequences).
//
// The payloads (prompts, sampling params, completion events) stay in Python,
// keyed by id; only ids and lengths cross this boundary.  One mutex + one
// condition variable; every wait is a timed wait on the same predicate, so
// close() always wakes the consumer.  Header-only so the pybind module and the
// standalone sanitizer stress test (csrc/runtime/tests) compile the same code.
#pragma once

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <stdexcept>
#include <vector>

namespace lsd_rt {

class BatchQueue {
 public:
  BatchQueue(int max_batch, double length_ratio) : max_batch_(max_batch), ratio_(length_ratio) {
    if (max_batch < 1) throw std::invalid_argument("max_batch must be >= 1");
    if (length_ratio < 1.0) throw std::invalid_argument("length_ratio must be >= 1");
  }

  // false once closed (the caller fails the request itself)
  bool push(int64_t id, int max_new_tokens) {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (closed_) return false;
      q_.push_back(Item{id, max_new_tokens < 1 ? 1 : max_new_tokens});
      ++pushed_;
    }
    cv_.notify_one();
    return true;
  }

  // push() of a whole batch under one lock / one wake-up: false (nothing
  // queued) when closed.
  bool push_many(const std::vector<int64_t>& ids, const std::vector<int>& max_new) {
    if (ids.size() != max_new.size()) throw std::invalid_argument("push_many: length mismatch");
    {
      std::lock_guard<std::mutex> g(mu_);
      if (closed_) return false;
      for (size_t i = 0; i < ids.size(); ++i)
        q_.push_back(Item{ids[i], max_new[i] < 1 ? 1 : max_new[i]});
      pushed_ += (int64_t)ids.size();
    }
    cv_.notify_all();
    return true;
  }

  // One scheduling decision.  Empty result == closed (nothing more will come
  // out; remaining ids are returned by drain()).
  std::vector<std::vector<int64_t>> next_groups(double window_s) {
    std::vector<Item> batch;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return closed_ || !q_.empty(); });
      if (closed_) return {};
      const auto deadline = std::chrono::steady_clock::now() +
                            std::chrono::duration_cast<std::chrono::steady_clock::duration>(
                                std::chrono::duration<double>(window_s > 0 ? window_s : 0.0));
      for (;;) {
        while (!q_.empty() && (int)batch.size() < max_batch_) {
          batch.push_back(q_.front());
          q_.pop_front();
        }
        if ((int)batch.size() >= max_batch_ || closed_) break;
        // The deadline is steady_clock; each wait is a system_clock
        // timed wait of the remaining time (pthread_cond_timedwait).  A
        // steady_clock wait_until is pthread_cond_clockwait, which GCC 11's
        // ThreadSanitizer does not intercept (it then reports the consumer as
        // still holding the mutex); clock jumps only shorten/lengthen one
        // wait, the loop re-checks the steady deadline.
        const auto left = deadline - std::chrono::steady_clock::now();
        if (left <= std::chrono::steady_clock::duration::zero()) break;
        cv_.wait_until(lk, std::chrono::system_clock::now() +
                               std::chrono::duration_cast<std::chrono::system_clock::duration>(left));
      }
      popped_ += (int64_t)batch.size();
      if ((int)batch.size() > max_seen_) max_seen_ = (int)batch.size();
    }
    std::stable_sort(batch.begin(), batch.end(),
                     [](const Item& a, const Item& b) { return a.n < b.n; });
    std::vector<std::vector<int64_t>> groups;
    int first_n = 0;
    for (const Item& it : batch) {
      if (groups.empty() || (double)it.n > ratio_ * first_n) {
        groups.emplace_back();
        first_n = it.n;
      }
      groups.back().push_back(it.id);
    }
    return groups;
  }

  // Continuous batching (runtime/scheduler.py): the scheduler admits queued
  // requests at every decode step without waiting -- up to k ids, FIFO.
  std::vector<int64_t> try_pop(int k) {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<int64_t> out;
    while (!q_.empty() && (int)out.size() < k) {
      out.push_back(q_.front().id);
      q_.pop_front();
    }
    popped_ += (int64_t)out.size();
    return out;
  }

  // Idle scheduler: block until a request is queued, close(), or timeout.
  bool wait_nonempty(double timeout_s) {
    std::unique_lock<std::mutex> lk(mu_);
    return cv_.wait_until(lk, std::chrono::system_clock::now() +
                                  std::chrono::duration_cast<std::chrono::system_clock::duration>(
                                      std::chrono::duration<double>(timeout_s > 0 ? timeout_s : 0.0)),
                          [&] { return closed_ || !q_.empty(); });
  }

  void close() {
    {
      std::lock_guard<std::mutex> g(mu_);
      closed_ = true;
    }
    cv_.notify_all();
  }

  // ids still queued (call after close(): they will never be scheduled)
  std::vector<int64_t> drain() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<int64_t> out;
    for (const Item& it : q_) out.push_back(it.id);
    q_.clear();
    return out;
  }

  int depth() const {
    std::lock_guard<std::mutex> g(mu_);
    return (int)q_.size();
  }
  bool closed() const {
    std::lock_guard<std::mutex> g(mu_);
    return closed_;
  }
  int max_seen() const {
    std::lock_guard<std::mutex> g(mu_);
    return max_seen_;
  }
  int64_t pushed() const {
    std::lock_guard<std::mutex> g(mu_);
    return pushed_;
  }
  int64_t popped() const {
    std::lock_guard<std::mutex> g(mu_);
    return popped_;
  }

 private:
  struct Item {
    int64_t id;
    int n;  // max_new_tokens
  };
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Item> q_;
  bool closed_ = false;
  int max_batch_;
  double ratio_;
  int max_seen_ = 0;
  int64_t pushed_ = 0, popped_ = 0;
};

}  // namespace lsd_rt
