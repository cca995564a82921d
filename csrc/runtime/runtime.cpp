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
//   * SchedCore       -- the continuous-batching state machine (sched_core.h):
//                        admission into slots, per-step group plans (leaves,
//                        joins, prefill chunks, decode rows / buckets), token
//                        readout events and slot release.
//   * ShmRing         -- one-node control plane (shm_ring.h): rank 0 writes a
//                        step plan once into shared memory, every follower
//                        rank of the pipeline replica reads it.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "batch_queue.h"
#include "sched_core.h"
#include "shm_ring.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <map>
#include <stdexcept>
#include <tuple>
#include <vector>

namespace py = pybind11;

using lsd_rt::SlotAllocator;

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
      .def("push_many", &BatchQueue::push_many, py::arg("ids"), py::arg("max_new_tokens"))
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
  using lsd_rt::SchedCore;
  py::class_<SchedCore>(m, "SchedCore")
      .def(py::init<int, int, int, int64_t, int, int, std::vector<SlotAllocator*>>(),
           py::arg("replicas"), py::arg("groups"), py::arg("cap"), py::arg("prefill_budget"),
           py::arg("chunk"), py::arg("max_seq"), py::arg("pools"),
           py::keep_alive<1, 8>())  // the pools outlive the core
      .def("add", &SchedCore::add, py::arg("sid"), py::arg("prompt_len"), py::arg("want"),
           py::arg("stop_at_eos"))
      .def("add_many", &SchedCore::add_many, py::arg("sids"), py::arg("prompt_lens"),
           py::arg("wants"), py::arg("stops"))
      .def("has_work", &SchedCore::has_work)
      .def("plan", [](SchedCore& c, int64_t step) {
             std::vector<int64_t> admitted;
             auto p = c.plan(step, &admitted);
             return py::make_tuple(p, admitted);
           }, py::arg("step"))
      .def("assign", &SchedCore::assign, py::arg("rep"), py::arg("step"), py::arg("g"),
           py::arg("tokens"), py::arg("eos"))
      .def("assign_collect",
           [](SchedCore& c, int rep, int64_t step, int g,
              py::array_t<int32_t, py::array::c_style | py::array::forcecast> tokens, int eos) {
             auto r = tokens.unchecked<1>();
             return c.assign_collect(rep, step, g, r.shape(0) ? r.data(0) : nullptr, (int)r.shape(0), eos);
           },
           py::arg("rep"), py::arg("step"), py::arg("g"), py::arg("tokens"), py::arg("eos"))
      .def("reset", &SchedCore::reset)
      .def("set_join_policy", &SchedCore::set_join_policy, py::arg("join_min"), py::arg("max_wait"))
      .def_property_readonly("deferred", &SchedCore::deferred)
      .def_property_readonly("joins", &SchedCore::joins)
      .def_property_readonly("leaves", &SchedCore::leaves)
      .def_property_readonly("max_rows", &SchedCore::max_rows)
      .def_property_readonly("steps", &SchedCore::steps)
      .def_property_readonly("n_waiting", &SchedCore::n_waiting)
      .def_property_readonly("n_seqs", &SchedCore::n_seqs)
      .def_property_readonly("n_expect", &SchedCore::n_expect);
  using lsd_rt::ShmRing;
  py::class_<ShmRing>(m, "ShmRing")
      .def_static("create", &ShmRing::create, py::arg("name"), py::arg("slots"), py::arg("slot_bytes"),
                  py::arg("readers"), py::return_value_policy::take_ownership)
      .def_static("attach", &ShmRing::attach, py::arg("name"), py::arg("index"),
                  py::return_value_policy::take_ownership)
      .def("publish", [](ShmRing& r, py::bytes b, double timeout_s) {
             std::string s = b;
             py::gil_scoped_release nogil;
             return r.publish(s.data(), s.size(), timeout_s);
           }, py::arg("data"), py::arg("timeout_s"))
      .def("read", [](ShmRing& r, double timeout_s) -> py::object {
             std::string out;
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = r.read(&out, timeout_s);
             }
             if (!ok) return py::none();
             return py::bytes(out);
           }, py::arg("timeout_s"))
      .def("unlink", &ShmRing::unlink)
      .def("close", &ShmRing::close_ring)
      .def_property_readonly("closed", &ShmRing::closed)
      .def("producer_alive", &ShmRing::producer_alive)
      .def_property_readonly("head", &ShmRing::head)
      .def("cursor", &ShmRing::cursor)
      .def_property_readonly("slots", &ShmRing::slots)
      .def_property_readonly("slot_bytes", &ShmRing::slot_bytes);
}
