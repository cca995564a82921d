// Sanitizer stress test of the serving scheduler's request queue
// (csrc/runtime/batch_queue.h), run by tests/test_native_runtime.py under
// ThreadSanitizer and under AddressSanitizer + UBSan.
//
// P producer threads push ids concurrently while one consumer forms rounds
// with a short collection window; a closer thread closes the queue while
// producers are still pushing.  Checks: every accepted id comes out exactly
// once (scheduled or drained), no round exceeds max_batch, every group
// respects the length-ratio rule, rejected pushes only happen after close.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "../batch_queue.h"

using lsd_rt::BatchQueue;

static int fail(const char* what, long long v) {
  std::fprintf(stderr, "FAIL: %s (%lld)\n", what, v);
  return 1;
}

int main(int argc, char** argv) {
  const int P = argc > 1 ? std::atoi(argv[1]) : 8;
  const int N = argc > 2 ? std::atoi(argv[2]) : 4000;  // pushes per producer
  const int MAXB = 37;
  const double RATIO = 4.0;
  BatchQueue q(MAXB, RATIO);
  std::vector<int> lens((size_t)P * N);
  std::vector<std::atomic<int>> seen((size_t)P * N);
  std::vector<std::atomic<int>> accepted((size_t)P * N);
  for (auto& s : seen) s = 0;
  for (auto& a : accepted) a = 0;
  std::atomic<int> bad_round{0}, bad_group{0}, rejected_open{0};

  std::thread consumer([&] {
    for (;;) {
      auto groups = q.next_groups(0.0002);
      if (groups.empty()) break;
      size_t total = 0;
      for (auto& g : groups) {
        total += g.size();
        int lo = 1 << 30, hi = 0;
        for (long long id : g) {
          seen[(size_t)id].fetch_add(1);
          lo = std::min(lo, lens[(size_t)id]);
          hi = std::max(hi, lens[(size_t)id]);
        }
        if ((double)hi > RATIO * lo) bad_group++;
      }
      if (total > (size_t)MAXB) bad_round++;
    }
  });
  std::vector<std::thread> producers;
  for (int p = 0; p < P; ++p) {
    // lengths are written before the id is pushed (the mutex orders them for the consumer)
    producers.emplace_back([&, p] {
      std::mt19937 rng(1234 + p);
      for (int i = 0; i < N; ++i) {
        const long long id = (long long)p * N + i;
        const int n = 1 + (int)(rng() % 512);
        lens[(size_t)id] = n;
        if (q.push(id, n)) {
          accepted[(size_t)id] = 1;
        } else if (!q.closed()) {
          rejected_open++;
        }
        if ((i & 255) == 0) std::this_thread::yield();
      }
    });
  }
  std::thread closer([&] {
    while (q.pushed() < (long long)P * N / 2) std::this_thread::yield();
    q.close();
  });
  for (auto& t : producers) t.join();
  closer.join();
  consumer.join();
  for (long long id : q.drain()) seen[(size_t)id].fetch_add(1);

  long long n_acc = 0;
  for (size_t i = 0; i < seen.size(); ++i) {
    const int a = accepted[i].load(), s = seen[i].load();
    n_acc += a;
    if (s != a) return fail("id delivered != accepted", (long long)i);
  }
  if (bad_round) return fail("round above max_batch", bad_round);
  if (bad_group) return fail("group breaks the length ratio", bad_group);
  if (rejected_open) return fail("push rejected while open", rejected_open);
  if (q.pushed() != n_acc) return fail("pushed counter", q.pushed());
  std::printf("ok accepted=%lld scheduled=%lld max_round=%d\n", n_acc, (long long)q.popped(),
              q.max_seen());
  return 0;
}
