// Native stage executor: the steady-state decode step of one pipeline stage
// issued by ONE call.
//
// The Python stage worker (parallel/pipeline.py) plans and prepares every
// item of a step: composition changes, prefill chunks, graph capture and the
// first use of a bucket stay there.  A step whose items are all steady-state
// decode items -- a cached hipGraph per item, no row changes, no eager
// transfers (one stage, or the native RCCL transport whose graphs carry their
// own edge send / receive) -- is handed to `exec_items` as a list of plain
// handles, and the whole step is enqueued here without returning to the
// interpreter between items.  Per item, in stream order on its lane:
//   [token-return receive (stage 0 of a multi-stage pipeline, ncclRecv, or a
//    loopback-channel receive in the single-GPU rehearsal)]
//   [busy-timing event]
//   [token readout: D2H copy of the previous item's sampled ids into a pinned
//    host buffer + completion event the scheduler polls]
//   [composition change: host-to-device copy of the packed row state from a
//    pinned buffer + the apply_rows scatter / token gather (elementwise.hip)]
//   hipGraphLaunch of the item's decode graph (its captured loopback ops
//    pass the enqueue handshake first and advance the host mirrors after)
//   [busy-timing event]
// The reference's equivalent is its per-token coordinator loop of two HTTP
// hops (`server.py:169-206`); here the loop body is one C++ call per step.
#include <torch/extension.h>

#include <hip/hip_runtime.h>

#include <array>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

void lsd_rccl_recv_raw(int64_t h, void* ptr, size_t bytes, int peer, hipStream_t st);  // comm.cpp
void lsd_loop_recv_raw(int64_t chan, void* ptr, size_t bytes, hipStream_t st);          // loop_fabric.cpp
void lsd_loop_io_wait(int64_t io);
void lsd_loop_io_done(int64_t io);
extern "C" hipError_t lsd_apply_rows(const int64_t* args, int b, hipStream_t st);  // elementwise.hip

namespace {

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// Item fields (all int64; 0 = absent)
enum : int {
  X_GRAPH = 0,   // hipGraphExec_t
  X_STREAM,      // hipStream_t (the group's lane)
  X_RCOMM,       // token-return receive: communicator
  X_RPTR,        //   device buffer
  X_RBYTES,      //   bytes
  X_RPEER,       //   peer rank in the communicator
  X_T0,          // busy-timing event before the item
  X_SRC,         // token readout: device source
  X_DST,         //   pinned host destination
  X_BYTES,       //   bytes
  X_EV,          //   completion event
  X_T1,          // busy-timing event after the item
  X_RLOOP,       // token-return receive on a loopback channel (instead of X_RCOMM)
  X_IO,          // loopback I/O list captured in the graph (enqueue handshake + mirrors)
  X_ROWS_ARGS,   // composition change: host int64 record of lsd_apply_rows (its [2] = device buffer)
  X_ROWS_SRC,    //   pinned host source of the packed row state
  X_ROWS_BYTES,  //   bytes
  X_ROWS_B,      //   bucket rows
  X_FIELDS
};

}  // namespace

void lsd_register_exec(py::module& m) {
  m.def("exec_items", [](const std::vector<std::array<int64_t, X_FIELDS>>& items) {
    py::gil_scoped_release nogil;  // launches may block on a full queue
    for (const auto& it : items) {
      auto st = reinterpret_cast<hipStream_t>(it[X_STREAM]);
      if (it[X_RCOMM])
        lsd_rccl_recv_raw(it[X_RCOMM], reinterpret_cast<void*>(it[X_RPTR]), (size_t)it[X_RBYTES],
                          (int)it[X_RPEER], st);
      if (it[X_RLOOP]) lsd_loop_recv_raw(it[X_RLOOP], reinterpret_cast<void*>(it[X_RPTR]), (size_t)it[X_RBYTES], st);
      if (it[X_T0]) hip_check(hipEventRecord(reinterpret_cast<hipEvent_t>(it[X_T0]), st), "hipEventRecord");
      if (it[X_BYTES]) {
        hip_check(hipMemcpyAsync(reinterpret_cast<void*>(it[X_DST]), reinterpret_cast<const void*>(it[X_SRC]),
                                 (size_t)it[X_BYTES], hipMemcpyDeviceToHost, st),
                  "hipMemcpyAsync");
        hip_check(hipEventRecord(reinterpret_cast<hipEvent_t>(it[X_EV]), st), "hipEventRecord");
      }
      if (it[X_ROWS_ARGS]) {
        const auto* args = reinterpret_cast<const int64_t*>(it[X_ROWS_ARGS]);
        hip_check(hipMemcpyAsync(reinterpret_cast<void*>(args[2]), reinterpret_cast<const void*>(it[X_ROWS_SRC]),
                                 (size_t)it[X_ROWS_BYTES], hipMemcpyHostToDevice, st),
                  "hipMemcpyAsync");
        hip_check(lsd_apply_rows(args, (int)it[X_ROWS_B], st), "apply_rows");
      }
      if (!it[X_GRAPH]) throw std::invalid_argument("exec_items: item without a graph");
      if (it[X_IO]) lsd_loop_io_wait(it[X_IO]);  // instant: the caller pre-waited the step's ops
      hip_check(hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(it[X_GRAPH]), st), "hipGraphLaunch");
      if (it[X_IO]) lsd_loop_io_done(it[X_IO]);
      if (it[X_T1]) hip_check(hipEventRecord(reinterpret_cast<hipEvent_t>(it[X_T1]), st), "hipEventRecord");
    }
  }, py::arg("items"));
  m.def("exec_fields", [] { return (int)X_FIELDS; });
}
