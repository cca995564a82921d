// Native host runtime for the pipeline engine (pure C++17, pybind11).
//
// The reference has no native runtime at all: its "scheduler" is the
// coordinator's Python for-loop (`server.py:169-206`) and its memory manager
// is "reload the full model in every pod" (`server.py:40-42`).  This module
// holds the host-side pieces of the MI355X engine that sit on the request path:
//
//   * SlotAllocator   -- KV-cache slot free list (each slot = one sequence's
//                        [layers][2][heads][max_seq][hd] region on every stage).
//   * split_even      -- microbatch boundaries for a round.
//   * partition_minmax-- exact min-max contiguous layer partition (DP), the
//                        cost model lives in Python (parallel/partition.py).
//   * simulate_pipeline -- discrete-event model of the static per-stage
//                        schedule (parallel/pipeline.py): proves every send has
//                        a matching receive in FIFO order per edge (deadlock
//                        freedom) and returns the makespan / bubble fraction
//                        for given stage and link costs.
//   * percentile      -- latency statistics for /metrics and bench.
//   * BatchQueue      -- the serving scheduler's request queue (batch_queue.h):
//                        thread-safe push from HTTP threads, window/length-group
//                        round formation for the one scheduler thread (GIL
//                        released while it waits).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "batch_queue.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <map>
#include <stdexcept>
#include <tuple>
#include <vector>

namespace py = pybind11;

class SlotAllocator {
 public:
  explicit SlotAllocator(int n) : cap_(n), used_(n, false) {
    for (int i = n - 1; i >= 0; --i) free_.push_back(i);
  }
  std::vector<int> alloc(int k) {
    if (k > (int)free_.size())
      throw std::runtime_error("out of KV slots: want " + std::to_string(k) + ", have " +
                               std::to_string(free_.size()));
    std::vector<int> out;
    out.reserve(k);
    for (int i = 0; i < k; ++i) {
      int s = free_.back();
      free_.pop_back();
      used_[s] = true;
      out.push_back(s);
    }
    return out;
  }
  void free(const std::vector<int>& slots) {
    for (int s : slots) {
      if (s < 0 || s >= cap_ || !used_[s]) throw std::runtime_error("double free / bad slot " + std::to_string(s));
      used_[s] = false;
      free_.push_back(s);
    }
  }
  int available() const { return (int)free_.size(); }
  int capacity() const { return cap_; }

 private:
  int cap_;
  std::vector<bool> used_;
  std::vector<int> free_;
};

std::vector<int> split_even(int n, int m) {
  if (m < 1) throw std::invalid_argument("m >= 1");
  std::vector<int> b(m + 1);
  for (int i = 0; i <= m; ++i) b[i] = (int)std::llround((double)i * n / m);
  return b;
}

// costs[i] = cost of layer i; head = extra cost of the last stage.
std::vector<std::pair<int, int>> partition_minmax(const std::vector<double>& costs, int P,
                                                  double head) {
  const int L = (int)costs.size();
  if (P < 1 || P > L) throw std::invalid_argument("need 1 <= P <= layers");
  std::vector<double> pre(L + 1, 0.0);
  for (int i = 0; i < L; ++i) pre[i + 1] = pre[i] + costs[i];
  const double INF = std::numeric_limits<double>::infinity();
  std::vector<std::vector<double>> best(P + 1, std::vector<double>(L + 1, INF));
  std::vector<std::vector<int>> arg(P + 1, std::vector<int>(L + 1, 0));
  best[0][0] = 0;
  for (int p = 1; p <= P; ++p)
    for (int i = p; i <= L - (P - p); ++i)
      for (int j = p - 1; j < i; ++j) {
        double c = pre[i] - pre[j] + (p == P ? head : 0.0);
        double v = std::max(best[p - 1][j], c);
        if (v < best[p][i]) { best[p][i] = v; arg[p][i] = j; }
      }
  std::vector<std::pair<int, int>> plan;
  int i = L;
  for (int p = P; p >= 1; --p) {
    int j = arg[p][i];
    plan.push_back({j, i});
    i = j;
  }
  std::reverse(plan.begin(), plan.end());
  return plan;
}

// Simulate the static schedule of parallel/pipeline.py.  stage_cost[r] = time
// of one microbatch forward on stage r; link = one-hop latency.  Receives are
// matched FIFO per directed edge; a stage blocks only on its own next input.
py::dict simulate_pipeline(int P, int M, int G, const std::vector<double>& stage_cost,
                           double link) {
  if ((int)stage_cost.size() != P) throw std::invalid_argument("stage_cost must have P entries");
  // arrival time of the input of item (s, m) at stage r
  std::map<std::tuple<int, int, int>, double> arrive;
  std::vector<double> free_at(P, 0.0);
  std::vector<double> busy(P, 0.0);
  // Process items in schedule order per stage; because every dependency
  // points to an earlier (stage, item) in the global topological order
  // (s, m, r), iterating in that order resolves all inputs.
  double makespan = 0;
  for (int s = 0; s < G; ++s)
    for (int m = 0; m < M; ++m)
      for (int r = 0; r < P; ++r) {
        double ready;
        if (r == 0)
          ready = (s == 0) ? 0.0 : arrive.at({0, s, m});
        else
          ready = arrive.at({r, s, m});
        double start = std::max(ready, free_at[r]);
        double end = start + stage_cost[r];
        free_at[r] = end;
        busy[r] += stage_cost[r];
        makespan = std::max(makespan, end);
        if (r + 1 < P)
          arrive[{r + 1, s, m}] = end + link;
        else if (s + 1 < G)
          arrive[{0, s + 1, m}] = end + (P > 1 ? link : 0.0);
      }
  double bubble = 0;
  for (int r = 0; r < P; ++r) bubble += 1.0 - busy[r] / makespan;
  py::dict d;
  d["makespan"] = makespan;
  d["bubble_fraction"] = bubble / P;
  d["tokens_per_time"] = (double)M * G / makespan;
  return d;
}

double percentile(std::vector<double> xs, double q) {
  if (xs.empty()) return 0.0;
  std::sort(xs.begin(), xs.end());
  double k = (xs.size() - 1) * q;
  size_t lo = (size_t)k, hi = std::min(lo + 1, xs.size() - 1);
  return xs[lo] + (xs[hi] - xs[lo]) * (k - lo);
}

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "native host runtime for llm_sharding_demo_amd";
  py::class_<SlotAllocator>(m, "SlotAllocator")
      .def(py::init<int>())
      .def("alloc", &SlotAllocator::alloc, py::arg("k") = 1)
      .def("free", &SlotAllocator::free)
      .def_property_readonly("available", &SlotAllocator::available)
      .def_property_readonly("capacity", &SlotAllocator::capacity);
  m.def("split_even", &split_even);
  m.def("partition_minmax", &partition_minmax);
  m.def("simulate_pipeline", &simulate_pipeline, py::arg("P"), py::arg("M"), py::arg("G"),
        py::arg("stage_cost"), py::arg("link") = 0.0);
  m.def("percentile", &percentile);
  using lsd_rt::BatchQueue;
  py::class_<BatchQueue>(m, "BatchQueue")
      .def(py::init<int, double>(), py::arg("max_batch"), py::arg("length_ratio") = 4.0)
      .def("push", &BatchQueue::push, py::arg("id"), py::arg("max_new_tokens"),
           py::call_guard<py::gil_scoped_release>())
      .def("next_groups", &BatchQueue::next_groups, py::arg("window_s"),
           py::call_guard<py::gil_scoped_release>())
      .def("try_pop", &BatchQueue::try_pop, py::arg("k"))
      .def("wait_nonempty", &BatchQueue::wait_nonempty, py::arg("timeout_s"),
           py::call_guard<py::gil_scoped_release>())
      .def("close", &BatchQueue::close, py::call_guard<py::gil_scoped_release>())
      .def("drain", &BatchQueue::drain)
      .def_property_readonly("depth", &BatchQueue::depth)
      .def_property_readonly("closed", &BatchQueue::closed)
      .def_property_readonly("max_seen", &BatchQueue::max_seen)
      .def_property_readonly("pushed", &BatchQueue::pushed)
      .def_property_readonly("popped", &BatchQueue::popped);
}
