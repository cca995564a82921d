// Native RCCL point-to-point communicator.
//
// The reference moves hidden states between shards as JSON over HTTP
// (`server.py:169-181`).  Here a pipeline edge (stage i -> i+1, and the
// token-id return edge P-1 -> 0) gets one 2-rank RCCL communicator per
// microbatch lane.  Its ncclSend / ncclRecv are enqueued on the CURRENT
// stream -- the lane's stream, eagerly or inside the lane's hipGraph capture
// (parallel/comm.py RcclTransport) -- so they are device-async and ordered
// by the lane's own stream order, with no comm stream or event hop.
//
// RCCL is resolved at run time from the librccl.so.1 that torch already
// loaded (dlopen RTLD_NOLOAD): one RCCL instance per process, the same one
// torch.distributed uses.  This avoids linking the ROCm 7.2 library against
// torch's bundled ROCm 7.0 runtime (SURVEY.md §5.8 hazard).  Only the types
// come from <rccl/rccl.h>.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <mutex>
#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace {

struct Rccl {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  ncclResult_t (*get_version)(int*) = nullptr;
  ncclResult_t (*get_async_error)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW);  // not loaded yet: load torch's by soname
    if (!h) throw std::runtime_error(std::string("RCCL not found: ") + dlerror());
    auto sym = [&](const char* n) {
      void* p = dlsym(h, n);
      if (!p) throw std::runtime_error(std::string("RCCL symbol missing: ") + n);
      return p;
    };
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(sym("ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(sym("ncclCommInitRank"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(sym("ncclCommDestroy"));
    r.send = reinterpret_cast<decltype(r.send)>(sym("ncclSend"));
    r.recv = reinterpret_cast<decltype(r.recv)>(sym("ncclRecv"));
    r.group_start = reinterpret_cast<decltype(r.group_start)>(sym("ncclGroupStart"));
    r.group_end = reinterpret_cast<decltype(r.group_end)>(sym("ncclGroupEnd"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(sym("ncclGetErrorString"));
    r.get_version = reinterpret_cast<decltype(r.get_version)>(sym("ncclGetVersion"));
    r.get_async_error = reinterpret_cast<decltype(r.get_async_error)>(sym("ncclCommGetAsyncError"));
    r.comm_abort = reinterpret_cast<decltype(r.comm_abort)>(sym("ncclCommAbort"));
  });
  return r;
}

void check(ncclResult_t e, const char* what) {
  if (e != ncclSuccess)
    throw std::runtime_error(std::string(what) + ": " + rccl().error_string(e));
}

ncclComm_t as_comm(int64_t h) {
  if (h == 0) throw std::invalid_argument("null RCCL communicator");
  return reinterpret_cast<ncclComm_t>(h);
}

void need_dense(const torch::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), what, ": contiguous device tensor required");
}

hipStream_t cur() { return c10::hip::getCurrentHIPStream().stream(); }

}  // namespace

// Raw receive for the native stage executor (csrc/stage_exec.cpp).
void lsd_rccl_recv_raw(int64_t h, void* ptr, size_t bytes, int peer, hipStream_t st) {
  check(rccl().recv(ptr, bytes, ncclUint8, peer, as_comm(h), st), "ncclRecv");
}

void lsd_register_comm(py::module& m) {
  m.def("rccl_version", [] {
    int v = 0;
    check(rccl().get_version(&v), "ncclGetVersion");
    return v;
  });
  m.def("rccl_unique_id", [] {
    ncclUniqueId id;
    check(rccl().get_unique_id(&id), "ncclGetUniqueId");
    return py::bytes(id.internal, NCCL_UNIQUE_ID_BYTES);
  });
  // Blocking until every rank of the communicator has joined (current device).
  m.def("rccl_comm_init", [](int nranks, int rank, py::bytes id_bytes) {
    const std::string s = id_bytes;
    if (s.size() != NCCL_UNIQUE_ID_BYTES) throw std::invalid_argument("bad RCCL unique id");
    ncclUniqueId id;
    std::memcpy(id.internal, s.data(), NCCL_UNIQUE_ID_BYTES);
    ncclComm_t c = nullptr;
    {
      py::gil_scoped_release nogil;
      check(rccl().comm_init_rank(&c, nranks, id, rank), "ncclCommInitRank");
    }
    return reinterpret_cast<int64_t>(c);
  });
  m.def("rccl_comm_destroy", [](int64_t h) { check(rccl().comm_destroy(as_comm(h)), "ncclCommDestroy"); });
  // Failure handling: the communicator's asynchronous error
  // state (ncclSuccess = 0, ncclInProgress = 7 while a non-blocking init or
  // abort runs; anything else is a failed peer / network / internal error),
  // polled by the engine watchdog ...
  m.def("rccl_async_error", [](int64_t h) {
    ncclResult_t e = ncclSuccess;
    check(rccl().get_async_error(as_comm(h), &e), "ncclCommGetAsyncError");
    return (int)e;
  });
  m.def("rccl_error_string", [](int code) { return std::string(rccl().error_string((ncclResult_t)code)); });
  // ... and the way out of a hang: ncclCommAbort sets the communicator's
  // abort flag, which every RCCL kernel of it polls in its wait loops, so an
  // unmatched ncclRecv / ncclSend (a dead or stalled peer) returns and the
  // streams behind it drain.  Frees the communicator (do not destroy after).
  // Called from the watchdog thread while another thread may be blocked in a
  // stream / event synchronize on work of this communicator.
  m.def("rccl_comm_abort", [](int64_t h) {
    py::gil_scoped_release nogil;
    check(rccl().comm_abort(as_comm(h)), "ncclCommAbort");
  });
  // Byte-wise send / receive of a dense tensor on the CURRENT stream.
  m.def("rccl_send", [](int64_t h, torch::Tensor t, int peer) {
    need_dense(t, "rccl_send");
    check(rccl().send(t.data_ptr(), (size_t)t.numel() * t.element_size(), ncclUint8, peer, as_comm(h),
                      cur()), "ncclSend");
  });
  m.def("rccl_recv", [](int64_t h, torch::Tensor t, int peer) {
    need_dense(t, "rccl_recv");
    check(rccl().recv(t.data_ptr(), (size_t)t.numel() * t.element_size(), ncclUint8, peer, as_comm(h),
                      cur()), "ncclRecv");
  });
  m.def("rccl_group_start", [] { check(rccl().group_start(), "ncclGroupStart"); });
  m.def("rccl_group_end", [] { check(rccl().group_end(), "ncclGroupEnd"); });
}
