// ThreadSanitizer / ASan+UBSan stress test of the device-loopback channels'
// host enqueue handshake (csrc/runtime/loop_handshake.h; csrc/loop_fabric.cpp
// runs it for every pipeline edge of the single-GPU rehearsal).  Run by
// tests/test_loop_handshake.py.
//
// Model: "enqueue == execute" (a device that runs each op the moment it is
// enqueued), so the ring bytes are touched by the host threads themselves:
// a sender writes its message into the ring at its placement right after the
// handshake admits it, the receiver reads and checks it right after its own
// admission.  Every ring access is a plain memory access, so TSan reports
// any pair the handshake's release/acquire pairs fail to order (a send that
// overwrites bytes a receive has not consumed, a receive that reads before
// the send wrote).  Per channel: one sender and one receiver thread, random
// sizes (ring wraparound and lap skips), I/O lists of several receives
// admitted cumulatively (k > 0), and header-slot pressure (more messages in
// flight than kLoopHeaders).  Then: an abort wakes a blocked waiter, a
// receive with no sender times out.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <stdexcept>
#include <thread>
#include <vector>

#include "../loop_handshake.h"

using namespace lsd_rt;

static std::atomic<int> g_fail{0};

static void check(bool ok, const char* what, long long v) {
  if (!ok && g_fail.fetch_add(1) < 10) std::fprintf(stderr, "FAIL: %s (%lld)\n", what, v);
}

struct Channel {
  LoopMirror m;
  std::vector<uint8_t> ring;
  uint64_t cap;
  explicit Channel(uint64_t c) : ring(c), cap(c) { loop_mirror_init(&m); }
};

static uint8_t pattern(uint64_t msg, uint64_t i) { return (uint8_t)(msg * 131 + i * 7 + 1); }

int main(int argc, char** argv) {
  const int C = argc > 1 ? std::atoi(argv[1]) : 4;     // channels
  const int N = argc > 2 ? std::atoi(argv[2]) : 3000;  // messages per channel
  std::atomic<bool> never{false};
  std::vector<std::unique_ptr<Channel>> chans;
  for (int c = 0; c < C; ++c) chans.push_back(std::make_unique<Channel>(8192 + 4096 * (uint64_t)c));
  // message sizes per channel, shared by both ends (like a static plan); at
  // most cap / 8, so a receive list (<= 4) fits the ring with its alignment
  // and lap-skip waste -- the engine sizes its rings to 8 x the largest
  // message (runtime/engine.py _loop_ring_bytes) for the same reason: a list
  // is admitted only when ALL its sends are enqueued
  std::vector<std::vector<uint64_t>> sizes(C);
  std::mt19937_64 rng(12345);
  for (int c = 0; c < C; ++c)
    for (int i = 0; i < N; ++i) sizes[c].push_back(1 + rng() % (chans[c]->cap / 8));

  std::vector<std::thread> th;
  for (int c = 0; c < C; ++c) {
    Channel* ch = chans[c].get();
    th.emplace_back([&, ch, c] {  // sender: one send at a time
      uint64_t head = 0;
      for (int i = 0; i < N; ++i) {
        const uint64_t b = sizes[c][i];
        loop_wait_until([&] { return loop_can_send(&ch->m, 0, head, b, ch->cap); }, [&] { return never.load(); },
                        30.0, "aborted", "send timed out");
        const uint64_t off = loop_place(head, b, ch->cap);
        for (uint64_t j = 0; j < b; ++j) ch->ring[(off + j) % ch->cap] = pattern(i, j);
        loop_advance(&ch->m, 0, b, ch->cap);
        head = off + b;
        if ((i & 127) == 0) std::this_thread::yield();
      }
    });
    th.emplace_back([&, ch, c] {  // receiver: I/O lists of up to 4 receives, admitted cumulatively
      std::mt19937 r2(c + 7);
      uint64_t head = 0;
      for (int i = 0; i < N;) {
        const int L = std::min<int>(N - i, 1 + (int)(r2() % 4));
        uint64_t h = head;
        std::vector<uint64_t> offs;
        for (int k = 0; k < L; ++k) {  // wait for receive #(recv_n + k) of the list
          loop_wait_until([&] { return loop_can_recv(&ch->m, (uint64_t)k); }, [&] { return never.load(); }, 30.0,
                          "aborted", "recv timed out");
          const uint64_t off = loop_place(h, sizes[c][i + k], ch->cap);
          offs.push_back(off);
          h = off + sizes[c][i + k];
        }
        for (int k = 0; k < L; ++k) {  // "launch" the list in order: read, check, release
          const uint64_t b = sizes[c][i + k];
          bool ok = true;
          for (uint64_t j = 0; j < b; ++j) ok &= ch->ring[(offs[k] + j) % ch->cap] == pattern(i + k, j);
          check(ok, "payload mismatch on channel", c);
          loop_advance(&ch->m, 1, b, ch->cap);
        }
        head = h;
        i += L;
      }
    });
  }
  for (auto& t : th) t.join();
  for (int c = 0; c < C; ++c) {
    check(chans[c]->m.send_n.load() == (uint64_t)N && chans[c]->m.recv_n.load() == (uint64_t)N, "counts", c);
    check(chans[c]->m.send_end.load() == chans[c]->m.recv_end.load(), "ring ends", c);
  }

  // abort: a receiver blocked with no sender is woken by the abort flag
  {
    Channel ch(4096);
    std::atomic<bool> abort_flag{false};
    std::atomic<int> got{0};
    std::thread w([&] {
      try {
        loop_wait_until([&] { return loop_can_recv(&ch.m, 0); }, [&] { return abort_flag.load(); }, 30.0,
                        "aborted", "timeout");
      } catch (const std::runtime_error& e) {
        got = std::strcmp(e.what(), "aborted") == 0 ? 1 : 2;
      }
    });
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    abort_flag = true;
    w.join();
    check(got.load() == 1, "abort did not wake the waiter", got.load());
  }
  // timeout: a send into a full header window gives up
  {
    Channel ch(1 << 20);
    for (uint64_t i = 0; i < kLoopHeaders; ++i) loop_advance(&ch.m, 0, 16, ch.cap);
    int got = 0;
    try {
      loop_wait_until([&] { return loop_can_send(&ch.m, 0, ch.m.send_end.load(), 16, ch.cap); },
                      [&] { return false; }, 0.05, "aborted", "timeout");
    } catch (const std::runtime_error& e) {
      got = std::strcmp(e.what(), "timeout") == 0 ? 1 : 2;
    }
    check(got == 1, "full header window did not time out", got);
  }
  if (g_fail.load()) return 1;
  std::printf("ok %d channels x %d messages\n", C, N);
  return 0;
}
