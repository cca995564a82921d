// Sanitizer stress test of the continuous-batching core
// (csrc/runtime/sched_core.h), run by tests/test_sched_core.py under
// AddressSanitizer + UBSan.
//
// Random workloads are driven through SchedCore with readouts arriving 0-3
// steps late. The workloads mix several replicas and groups, slot pools
// smaller than the demand, chunked prefill under a token budget, and EOS
// stops. Checks:
//   * every sequence receives min(want, tokens up to its first EOS) tokens,
//     exactly once each;
//   * no event is reported for an unknown or finished sequence;
//   * each sequence is released exactly once;
//   * slots are conserved (every pool is full again at the end);
//   * no readout is left pending, and no decode bucket exceeds the group
//     capacity.
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <map>
#include <random>
#include <tuple>
#include <vector>

#include "../sched_core.h"

using namespace lsd_rt;

static int fail(const char* what, long long v) {
  std::fprintf(stderr, "FAIL: %s (%lld)\n", what, v);
  return 1;
}

struct Track {
  int want = 0;
  bool stop_at_eos = false;
  int got = 0;
  bool finished = false, released = false, eos_seen = false;
};

static int run(unsigned seed) {
  std::mt19937 rnd(seed);
  auto pick = [&](std::vector<int> v) { return v[rnd() % v.size()]; };
  const int R = pick({1, 2, 3}), M = pick({1, 2, 4}), cap = pick({1, 3, 8, 16});
  const int slots = pick({1, 5, cap * M * R});
  const int budget = pick({0, 7, 64}), chunk = pick({0, 4, 9});
  const int eos = 7;
  std::vector<SlotAllocator> pools;
  for (int r = 0; r < R; ++r) pools.emplace_back(slots);
  std::vector<SlotAllocator*> pp;
  for (auto& p : pools) pp.push_back(&p);
  SchedCore core(R, M, cap, budget, chunk, 4096, pp);
  std::map<int64_t, Track> seqs;
  std::deque<std::tuple<int64_t, int, int, int>> pending;  // step, rep, g, n
  int64_t sid = 0;
  auto drain = [&](int64_t upto) -> int {
    while (!pending.empty() && std::get<0>(pending.front()) <= upto) {
      const auto [st, rep, g, n] = pending.front();
      pending.pop_front();
      std::vector<int> toks(n);
      for (int& t : toks) t = rnd() % 6 == 0 ? eos : 11;
      for (const auto& e : core.assign(rep, st, g, toks, eos)) {
        const int64_t s = std::get<0>(e);
        const int tok = std::get<1>(e), fl = std::get<2>(e);
        auto it = seqs.find(s);
        if (it == seqs.end()) return fail("event for an unknown sequence", s);
        Track& t = it->second;
        if (fl & EV_RELEASE) {
          if (t.released) return fail("released twice", s);
          t.released = true;
          if (fl & EV_FINISH) t.finished = true;
          continue;
        }
        if (t.finished) return fail("token after finish", s);
        if ((fl & EV_FIRST) != (t.got == 0 ? EV_FIRST : 0)) return fail("first-token flag", s);
        ++t.got;
        if (t.stop_at_eos && tok == eos) t.eos_seen = true;
        const bool done = t.got >= t.want || t.eos_seen;
        if (done != bool(fl & EV_FINISH)) return fail("finish flag", s);
        if (done) t.finished = true;
      }
    }
    return 0;
  };
  for (int64_t step = 0; step < 2000000; ++step) {
    if (step < 300 && rnd() % 3 == 0)
      for (int k = rnd() % 5; k >= 0; --k) {
        Track t;
        t.want = 1 + rnd() % 30;
        t.stop_at_eos = rnd() % 2 == 0;
        seqs[sid] = t;
        core.add(sid++, 1 + rnd() % 60, t.want, t.stop_at_eos);
      }
    if (!core.has_work()) {
      if (step >= 300) break;
      continue;
    }
    std::vector<int64_t> adm;
    const auto plans = core.plan(step, &adm);
    for (size_t rep = 0; rep < plans.size(); ++rep)
      for (const auto& go : plans[rep]) {
        if (std::get<3>(go) > cap) return fail("bucket above capacity", std::get<3>(go));
        if (std::get<2>(go) > std::get<3>(go)) return fail("rows above bucket", std::get<2>(go));
        if (std::get<1>(go)) pending.emplace_back(step, (int)rep, std::get<0>(go), std::get<1>(go));
      }
    if (int rc = drain(step - (int64_t)(rnd() % 4))) return rc;
  }
  if (int rc = drain(1LL << 60)) return rc;
  if (core.has_work()) return fail("work left", core.n_seqs());
  if (core.n_expect() != 0) return fail("readouts left", core.n_expect());
  for (auto& p : pools)
    if (p.available() != slots) return fail("slots leaked", slots - p.available());
  for (const auto& kv : seqs) {
    const Track& t = kv.second;
    if (!t.released || !t.finished) return fail("sequence never completed", kv.first);
    if (!t.eos_seen && t.got != t.want) return fail("token count", kv.first);
  }
  return 0;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 50;
  for (int s = 0; s < n; ++s)
    if (int rc = run((unsigned)s)) {
      std::fprintf(stderr, "seed %d\n", s);
      return rc;
    }
  std::printf("ok %d workloads\n", n);
  return 0;
}
