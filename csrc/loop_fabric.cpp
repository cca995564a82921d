// Host side of the device loopback channels (csrc/kernels/loopback.hip):
// the single-GPU rehearsal of the RCCL pipeline edges (SURVEY.md §2.6 items
// 2 and 5; parallel/comm.py DeviceLoopTransport).
//
// RCCL's p2p kernels on an 8-GPU node spin on their peer's FIFO; two
// spinning kernels there never share a hardware queue, because each GPU runs
// its own.  P stage threads on ONE GPU share that GPU's hardware queues
// (GPU_MAX_HW_QUEUES, default 4), and a wait kernel queued in front of the
// kernel it waits for would spin until its deadline.  So every op first
// passes a host-side enqueue handshake, per channel:
//   receive #n is enqueued only after send #n was enqueued,
//   send #n only after the receives that free its ring bytes / header slot
//   were enqueued.
// Every device wait then targets work that is already ahead of it in every
// queue, whatever the stream -> hardware-queue mapping (induction on enqueue
// time), and the spins are brief.  The handshake is host-only bookkeeping
// (enqueue counters + a mirror of the ring placement); the device protocol is
// self-contained and is what a captured hipGraph replays.
//
// Waits run with the GIL released; the Python caller also drops its hold on
// the capture gate around them (parallel/pipeline.py GPU_GATE), so a stage
// waiting on its peer never blocks a sibling's graph capture.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cstddef>
#include <chrono>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "kernels/loopback.h"
#include "runtime/loop_handshake.h"

namespace py = pybind11;

extern "C" hipError_t lsd_loop_send(LoopChan* ch, void* ring, const void* src, uint64_t bytes,
                                    LoopStatus* st, hipStream_t s);
extern "C" hipError_t lsd_loop_recv(LoopChan* ch, const void* ring, void* dst, uint64_t bytes,
                                    LoopStatus* st, hipStream_t s);
extern "C" uint64_t lsd_loop_place(uint64_t head, uint64_t bytes, uint64_t cap);

namespace {

struct Fabric;

// Enqueue mirrors of one channel (each side written by its one owning stage
// thread / process): in process memory, or in a POSIX shared-memory block
// when the two ends are different processes on one GPU (loop_chan_attach).
// The handshake itself lives in runtime/loop_handshake.h (HIP-free, TSan-tested).
using Mirror = lsd_rt::LoopMirror;
static_assert(LOOP_HEADERS == lsd_rt::kLoopHeaders, "handshake header count");

struct Chan {
  Fabric* fab = nullptr;
  LoopChan* dev = nullptr;  // device state (torch-owned storage, or an IPC mapping)
  uint8_t* ring = nullptr;  // this process's address of the ring
  uint64_t cap = 0;
  uint32_t id = 0;
  Mirror* m = nullptr;      // own_m, or a slot of a shared-memory block
  std::unique_ptr<Mirror> own_m;
};

struct Fabric {
  LoopStatus* host = nullptr;  // pinned, mapped
  LoopStatus* dev = nullptr;
  std::atomic<bool> aborted{false};
  double timeout_s = 60.0;
  std::vector<std::unique_ptr<Chan>> chans;
  std::mutex mu;
};

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

Fabric* as_fab(int64_t h) {
  if (!h) throw std::invalid_argument("null loopback fabric");
  return reinterpret_cast<Fabric*>(h);
}
Chan* as_chan(int64_t h) {
  if (!h) throw std::invalid_argument("null loopback channel");
  return reinterpret_cast<Chan*>(h);
}

hipStream_t cur() { return c10::hip::getCurrentHIPStream().stream(); }

// One op of an I/O list: direction 0 = send, 1 = receive.
struct Op {
  Chan* ch;
  int dir;
  uint64_t bytes;
};
using Ops = std::vector<Op>;

std::string chan_name(const Chan* c) { return "loopback channel " + std::to_string(c->id); }

// Block until every op of `ops`, issued in order, satisfies the enqueue
// handshake (module comment).  Several ops on one channel are accounted
// cumulatively.  Throws on abort or after the fabric timeout.
void wait_ops(Fabric* f, const Ops& ops) {
  for (size_t i = 0; i < ops.size(); ++i) {
    const Op& op = ops[i];
    Chan* c = op.ch;
    if (op.bytes > c->cap)
      throw std::runtime_error(chan_name(c) + ": message of " + std::to_string(op.bytes) +
                               " bytes exceeds the ring (" + std::to_string(c->cap) +
                               " bytes; raise LSD_LOOP_RING_MB)");
    // earlier ops of this list on the same channel and direction
    uint64_t k = 0, head = op.dir ? c->m->recv_end.load(std::memory_order_relaxed)
                                  : c->m->send_end.load(std::memory_order_relaxed);
    for (size_t j = 0; j < i; ++j)
      if (ops[j].ch == c && ops[j].dir == op.dir) {
        ++k;
        head = lsd_rt::loop_place(head, ops[j].bytes, c->cap) + ops[j].bytes;
      }
    lsd_rt::loop_wait_until(
        [&] { return op.dir ? lsd_rt::loop_can_recv(c->m, k) : lsd_rt::loop_can_send(c->m, k, head, op.bytes, c->cap); },
        [&] { return f->aborted.load(std::memory_order_relaxed); }, f->timeout_s,
        chan_name(c) + ": data plane aborted",
        chan_name(c) + ": timed out waiting for the peer stage (" +
            std::string(op.dir ? "receive: no matching send" : "send: ring full") + ")");
  }
}

// Enqueue one op on `st` (no wait) and advance its side's mirror.
void launch_op(Fabric* f, const Op& op, void* ptr, hipStream_t st, bool mirror) {
  Chan* c = op.ch;
  if (op.dir == 0)
    hip_check(lsd_loop_send(c->dev, c->ring, ptr, op.bytes, f->dev, st), "loopback send");
  else
    hip_check(lsd_loop_recv(c->dev, c->ring, ptr, op.bytes, f->dev, st), "loopback recv");
  if (mirror) lsd_rt::loop_advance(c->m, op.dir, op.bytes, c->cap);
}

// Ops captured inside a hipGraph: replayed with the graph, mirrored here.
struct IoList {
  Fabric* fab;
  Ops ops;
};

void check_dense(const torch::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), what, ": contiguous device tensor required");
}

}  // namespace

// --- used by the native stage executor (csrc/stage_exec.cpp) --------------
void lsd_loop_recv_raw(int64_t chan, void* ptr, size_t bytes, hipStream_t st) {
  Chan* c = as_chan(chan);
  Ops ops{{c, 1, (uint64_t)bytes}};
  wait_ops(c->fab, ops);
  launch_op(c->fab, ops[0], ptr, st, true);
}
void lsd_loop_io_wait(int64_t io) {
  auto* l = reinterpret_cast<IoList*>(io);
  wait_ops(l->fab, l->ops);
}
void lsd_loop_io_done(int64_t io) {
  // advance the mirrors of a launched graph's captured ops (in op order)
  auto* l = reinterpret_cast<IoList*>(io);
  for (const Op& op : l->ops) lsd_rt::loop_advance(op.ch->m, op.dir, op.bytes, op.ch->cap);
}

void lsd_register_loopback(py::module& m) {
  m.def("loop_state_bytes", [] { return (int64_t)sizeof(LoopChan); });
  m.def("loop_headers", [] { return (int)LOOP_HEADERS; });
  m.def("loop_fabric_create", [](double timeout_s) {
    // the host mirror of the ring placement must be the device kernels' rule
    for (uint64_t h : {0ull, 1ull, 255ull, 256ull, 4000ull, 65280ull})
      for (uint64_t b : {1ull, 256ull, 3000ull})
        if (lsd_rt::loop_place(h, b, 65536) != lsd_loop_place(h, b, 65536))
          throw std::logic_error("loop_place differs from the device placement");
    auto* f = new Fabric();
    f->timeout_s = timeout_s;
    void* p = nullptr;
    hip_check(hipHostMalloc(&p, sizeof(LoopStatus), hipHostMallocMapped | hipHostMallocCoherent),
              "hipHostMalloc");
    std::memset(p, 0, sizeof(LoopStatus));
    f->host = static_cast<LoopStatus*>(p);
    void* d = nullptr;
    hip_check(hipHostGetDevicePointer(&d, p, 0), "hipHostGetDevicePointer");
    f->dev = static_cast<LoopStatus*>(d);
    return reinterpret_cast<int64_t>(f);
  });
  // Channel state lives in `state` (uint8 device tensor of loop_state_bytes()),
  // its ring in `ring`; both stay owned by the Python fabric.
  m.def("loop_chan_create", [](int64_t fab, torch::Tensor state, torch::Tensor ring, double spin_limit_s) {
    Fabric* f = as_fab(fab);
    check_dense(state, "loop_chan_create(state)");
    check_dense(ring, "loop_chan_create(ring)");
    TORCH_CHECK(state.numel() >= (int64_t)sizeof(LoopChan), "loop_chan_create: state too small");
    TORCH_CHECK(((uintptr_t)ring.data_ptr() & 255) == 0, "loop_chan_create: ring must be 256-B aligned");
    std::lock_guard<std::mutex> g(f->mu);
    auto c = std::make_unique<Chan>();
    c->fab = f;
    c->own_m = std::make_unique<Mirror>();
    c->m = c->own_m.get();
    lsd_rt::loop_mirror_init(c->m);
    c->dev = reinterpret_cast<LoopChan*>(state.data_ptr());
    c->ring = static_cast<uint8_t*>(ring.data_ptr());
    c->cap = (uint64_t)ring.numel();
    c->id = (uint32_t)f->chans.size();
    LoopChan init;
    std::memset(&init, 0, sizeof(init));
    init.cap = c->cap;
    init.spin_limit = (uint64_t)(spin_limit_s * 1e8);  // s_memrealtime runs at 100 MHz
    init.ring = static_cast<uint8_t*>(ring.data_ptr());
    init.id = c->id;
    init.stall_from = ~0ull;
    hip_check(hipMemcpy(c->dev, &init, sizeof(init), hipMemcpyHostToDevice), "hipMemcpy(chan init)");
    Chan* raw = c.get();
    f->chans.push_back(std::move(c));
    return reinterpret_cast<int64_t>(raw);
  });
  m.def("loop_fabric_destroy", [](int64_t fab) {
    Fabric* f = as_fab(fab);
    if (f->host) hipHostFree(f->host);
    delete f;
  });
  // handshake wait for a list of (chan, dir, bytes) ops (GIL released)
  m.def("loop_wait", [](const std::vector<std::tuple<int64_t, int, int64_t>>& ops) {
    if (ops.empty()) return;
    Ops v;
    for (auto& [c, d, b] : ops) v.push_back({as_chan(c), d, (uint64_t)b});
    py::gil_scoped_release nogil;
    wait_ops(v[0].ch->fab, v);
  });
  // eager op on the current stream: handshake (instant after loop_wait) +
  // launch + mirror; capture=true: launch only (the op is inside a hipGraph
  // being captured; its mirror advances at every replay, loop_graph_launch)
  auto op_fn = [](int dir) {
    return [dir](int64_t chan, torch::Tensor t, bool capture) {
      check_dense(t, dir ? "loop_recv" : "loop_send");
      Chan* c = as_chan(chan);
      Op op{c, dir, (uint64_t)t.numel() * t.element_size()};
      if (op.bytes > c->cap)
        throw std::runtime_error(chan_name(c) + ": message exceeds the ring (raise LSD_LOOP_RING_MB)");
      if (c->fab->aborted.load()) throw std::runtime_error(chan_name(c) + ": data plane aborted");
      hipStream_t st = cur();
      if (!capture) {
        py::gil_scoped_release nogil;
        wait_ops(c->fab, Ops{op});
      }
      launch_op(c->fab, op, t.data_ptr(), st, !capture);
    };
  };
  m.def("loop_send", op_fn(0), py::arg("chan"), py::arg("t"), py::arg("capture") = false);
  m.def("loop_recv", op_fn(1), py::arg("chan"), py::arg("t"), py::arg("capture") = false);
  m.def("loop_io_create", [](const std::vector<std::tuple<int64_t, int, int64_t>>& ops) {
    auto* l = new IoList();
    l->fab = nullptr;
    for (auto& [c, d, b] : ops) {
      l->ops.push_back({as_chan(c), d, (uint64_t)b});
      l->fab = as_chan(c)->fab;
    }
    return reinterpret_cast<int64_t>(l);
  });
  m.def("loop_io_free", [](int64_t io) { delete reinterpret_cast<IoList*>(io); });
  // replay a captured graph whose I/O ops are `io`: handshake, launch, mirrors
  m.def("loop_graph_launch", [](int64_t graph_exec, int64_t io) {
    auto* l = reinterpret_cast<IoList*>(io);
    if (l->fab && l->fab->aborted.load()) throw std::runtime_error("loopback data plane aborted");
    hipStream_t st = cur();
    py::gil_scoped_release nogil;
    if (l->fab) wait_ops(l->fab, l->ops);
    hip_check(hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(graph_exec), st), "hipGraphLaunch");
    lsd_loop_io_done(io);
  });
  m.def("loop_abort", [](int64_t fab) {
    Fabric* f = as_fab(fab);
    f->aborted.store(true);
    __atomic_store_n(&f->host->abort, 1u, __ATOMIC_SEQ_CST);
  });
  m.def("loop_aborted", [](int64_t fab) { return as_fab(fab)->aborted.load(); });
  // (err code, channel id) recorded by the kernels; 0 = healthy
  m.def("loop_status", [](int64_t fab) {
    Fabric* f = as_fab(fab);
    const uint32_t e = __atomic_load_n(&f->host->err, __ATOMIC_ACQUIRE);
    const uint32_t c = __atomic_load_n(&f->host->err_chan, __ATOMIC_ACQUIRE);
    return std::make_tuple((int)e, (int)c);
  });
  m.def("loop_counts", [](int64_t chan) {
    Chan* c = as_chan(chan);
    return std::make_tuple((int64_t)c->m->send_n.load(), (int64_t)c->m->recv_n.load(),
                           (int64_t)c->m->send_end.load(), (int64_t)c->m->recv_end.load());
  });
  // fault injection (tests, device idle): the send kernels stop publishing at
  // message `from` of this channel -- eager or graph-replayed alike
  m.def("loop_stall", [](int64_t chan, int64_t from) {
    Chan* c = as_chan(chan);
    const uint64_t v = (uint64_t)from;
    hip_check(hipMemcpy(reinterpret_cast<char*>(c->dev) + offsetof(LoopChan, stall_from), &v, sizeof(v),
                        hipMemcpyHostToDevice), "hipMemcpy(stall)");
  });

  // --- one GPU, several processes (dist-mode rehearsal, parallel/comm.py
  // IpcLoopTransport): the receiving rank allocates its channels' state and
  // ring with hipMalloc and exports them (hipIpcGetMemHandle, dmabuf); the
  // sending rank maps them (hipIpcOpenMemHandle); both ends' enqueue mirrors
  // live in one POSIX shared-memory block of 64-B slots.
  m.def("loop_dev_alloc", [](int64_t bytes) {
    void* p = nullptr;
    hip_check(hipMalloc(&p, (size_t)bytes), "hipMalloc(loop)");
    hip_check(hipMemset(p, 0, (size_t)bytes), "hipMemset(loop)");
    return reinterpret_cast<int64_t>(p);
  });
  m.def("loop_dev_free", [](int64_t p) { hipFree(reinterpret_cast<void*>(p)); });
  m.def("loop_ipc_handle", [](int64_t p) {
    hipIpcMemHandle_t h;
    hip_check(hipIpcGetMemHandle(&h, reinterpret_cast<void*>(p)), "hipIpcGetMemHandle");
    return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
  });
  m.def("loop_ipc_open", [](py::bytes hb) {
    const std::string s = hb;
    if (s.size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("bad IPC handle");
    hipIpcMemHandle_t h;
    std::memcpy(&h, s.data(), sizeof(h));
    void* p = nullptr;
    hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    return reinterpret_cast<int64_t>(p);
  });
  m.def("loop_shm_map", [](const std::string& name, int64_t bytes, bool create) {
    int fd = shm_open(name.c_str(), create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("shm_open(" + name + "): " + std::strerror(errno));
    if (create) {  // pages reserved now (no SIGBUS later on a full /dev/shm)
      const int rc = ftruncate(fd, (off_t)bytes) != 0 ? errno : posix_fallocate(fd, 0, (off_t)bytes);
      if (rc != 0) {
        close(fd);
        shm_unlink(name.c_str());
        throw std::runtime_error("reserving shared memory " + name + ": " + std::strerror(rc));
      }
    }
    void* p = mmap(nullptr, (size_t)bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("mmap(" + name + "): " + std::strerror(errno));
    return reinterpret_cast<int64_t>(p);  // mapped for the life of the process
  });
  m.def("loop_shm_unlink", [](const std::string& name) { shm_unlink(name.c_str()); });
  // A channel over given device pointers and a shared mirror slot; the
  // receiving end initialises the device state and the mirror (before any
  // sender attaches).
  m.def("loop_chan_attach", [](int64_t fab, int64_t state, int64_t ring, int64_t cap, int64_t id,
                               int64_t mirror, bool init, double spin_limit_s) {
    Fabric* f = as_fab(fab);
    if (!state || !ring || !mirror || cap <= 0 || (ring & 255))
      throw std::invalid_argument("loop_chan_attach: bad pointers");
    std::lock_guard<std::mutex> g(f->mu);
    auto c = std::make_unique<Chan>();
    c->fab = f;
    c->m = reinterpret_cast<Mirror*>(mirror);
    c->dev = reinterpret_cast<LoopChan*>(state);
    c->ring = reinterpret_cast<uint8_t*>(ring);
    c->cap = (uint64_t)cap;
    c->id = (uint32_t)id;
    if (init) {
      LoopChan st;
      std::memset(&st, 0, sizeof(st));
      st.cap = c->cap;
      st.spin_limit = (uint64_t)(spin_limit_s * 1e8);
      st.ring = reinterpret_cast<uint8_t*>(ring);
      st.id = c->id;
      st.stall_from = ~0ull;
      hip_check(hipMemcpy(c->dev, &st, sizeof(st), hipMemcpyHostToDevice), "hipMemcpy(chan init)");
      lsd_rt::loop_mirror_init(c->m);
    }
    Chan* raw = c.get();
    f->chans.push_back(std::move(c));
    return reinterpret_cast<int64_t>(raw);
  });
}
