// ThreadSanitizer / ASan+UBSan stress test of the one-node control plane's
// shared-memory broadcast ring (csrc/runtime/shm_ring.h; parallel/comm.py
// ShmPlanChannel), run by tests/test_loop_handshake.py.
//
// One producer thread publishes N variable-length messages into a small ring
// (many laps) while R reader threads -- each with its own attached mapping,
// as follower ranks have -- read them; one reader is slow, so the producer
// keeps hitting the "slowest reader" wait.  Checks: every reader sees every
// message, in order, intact; the producer never overwrites an unread slot
// (payload checks); attach acquires the header the creator published; a
// reader blocked on an idle ring times out, and close() ends every reader's
// wait once the ring is drained.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

#include "../shm_ring.h"

using lsd_rt::ShmRing;

static std::atomic<int> g_fail{0};

static void check(bool ok, const char* what, long long v) {
  if (!ok && g_fail.fetch_add(1) < 10) std::fprintf(stderr, "FAIL: %s (%lld)\n", what, v);
}

static std::string msg(int i) {
  std::string s(1 + (i * 37) % 200, '\0');
  for (size_t j = 0; j < s.size(); ++j) s[j] = (char)(i * 13 + j * 3);
  return s;
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? std::atoi(argv[1]) : 4;
  const int N = argc > 2 ? std::atoi(argv[2]) : 20000;
  const std::string name = "/lsd-stress-" + std::to_string(getpid());
  std::unique_ptr<ShmRing> w(ShmRing::create(name, 8, 256, R));
  std::atomic<int> attached{0};
  std::vector<std::thread> th;
  for (int r = 0; r < R; ++r) {
    th.emplace_back([&, r] {
      std::unique_ptr<ShmRing> rd(ShmRing::attach(name, r));  // own mapping, like a follower rank
      attached.fetch_add(1);
      std::string out;
      for (int i = 0; i < N; ++i) {
        if (!rd->read(&out, 30.0)) {
          check(false, "read timed out at message", i);
          return;
        }
        check(out == msg(i), "message corrupt or out of order", i);
        if (r == 0 && (i % 97) == 0) std::this_thread::sleep_for(std::chrono::microseconds(200));  // slow reader
      }
      // drained: an idle ring times out ...
      check(!rd->read(&out, 0.02), "read past the last message", N);
      // ... until the producer closes it: then every wait ends
      while (!rd->closed()) std::this_thread::yield();
      check(!rd->read(&out, 30.0), "read after close", N);
      check(rd->producer_alive(), "producer alive", r);
    });
  }
  while (attached.load() < R) std::this_thread::yield();
  w->unlink();  // every reader attached: the mappings outlive the name
  for (int i = 0; i < N; ++i) {
    const std::string m = msg(i);
    if (!w->publish(m.data(), m.size(), 30.0)) {
      check(false, "publish timed out at", i);
      break;
    }
  }
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  w->close_ring();
  for (auto& t : th) t.join();
  for (int r = 0; r < R; ++r) check(w->cursor(r) == (uint64_t)N, "reader cursor", r);
  if (g_fail.load()) return 1;
  std::printf("ok %d readers x %d messages\n", R, N);
  return 0;
}
