// Native host runtime for the pipeline engine (pure C++17, pybind11).
//
// The reference has no native runtime at all: its "scheduler" is the
// coordinator's Python for-loop (`server.py:169-206`) and its memory manager
// is "reload the full model in every pod" (`server.py:40-42`).  This module
// holds the host-side pieces of the MI355X engine that sit on the request path:
//
//   * SlotAllocator   -- KV-cache slot free list (each slot = one sequence's
//                        [layers][2][heads][max_seq][hd] region on every stage).
//   * partition_minmax-- exact min-max contiguous layer partition (DP), the
//                        cost model lives in Python (parallel/partition.py).
//   * BatchQueue      -- the serving scheduler's admission queue (batch_queue.h):
//                        thread-safe push from HTTP threads; the continuous-
//                        batching scheduler drains it at every decode step
//                        (try_pop); window/length-group round formation
//                        (next_groups) for batch jobs.
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

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "native host runtime for llm_sharding_demo_amd";
  py::class_<SlotAllocator>(m, "SlotAllocator")
      .def(py::init<int>())
      .def("alloc", &SlotAllocator::alloc, py::arg("k") = 1)
      .def("free", &SlotAllocator::free)
      .def_property_readonly("available", &SlotAllocator::available)
      .def_property_readonly("capacity", &SlotAllocator::capacity);
  m.def("partition_minmax", &partition_minmax);
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
