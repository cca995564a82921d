// Single-producer / multi-reader broadcast ring in POSIX shared memory: the
// control plane of a one-node multi-GPU engine (runtime/plan.py records,
// parallel/comm.py ShmPlanChannel).
//
// Every step rank 0's scheduler sends each follower rank the step plan.  Over
// gloo that is one socket message per follower per step (~20 us of host time
// each on rank 0, ~150 us at P = 8: profiles/r4_plan_wire.log); all ranks of
// an 8-GPU MI355X node share one host, so here the plan is written ONCE into
// a slot of a shared ring and every follower of the pipeline replica reads it
// from there.  The reference's equivalent is a JSON POST per token per shard
// (`/root/reference/server.py:172-181`).
//
// Layout: Header (cache-line separated counters) + `slots` slots of
// `slot_bytes` bytes, each [u32 length][payload].  The producer publishes
// message k into slot k % slots once every reader's cursor is > k - slots
// (no overwrite of unread data), then release-stores head = k + 1; reader i
// acquire-loads head, copies the slot and release-stores cursor[i] = k + 1.
// Waits spin briefly, then sleep with backoff, and give up at their timeout.
// The producer stores its pid (and its pid namespace) in the header: a reader
// whose wait times out can tell a quiet producer from a dead one
// (producer_alive; a reader in another pid namespace -- another container of
// the pod sharing /dev/shm -- cannot signal-probe that pid and takes the
// producer as alive, relying on close_ring()), and close_ring() ends every
// reader's wait once the ring is drained.
#pragma once

#include <signal.h>

#include <cerrno>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

namespace lsd_rt {

class ShmRing {
 public:
  static constexpr uint64_t kMagic = 0x4C53445348524E47ull;  // "LSDSHRNG"
  static constexpr int kMaxReaders = 64;

  // Producer: create (and size) the segment.
  static ShmRing* create(const std::string& name, int slots, int slot_bytes, int readers) {
    if (slots < 2 || slot_bytes < 64 || readers < 1 || readers > kMaxReaders)
      throw std::invalid_argument("ShmRing: bad geometry");
    const size_t bytes = sizeof(Header) + (size_t)slots * slot_bytes;
    int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("shm_open(create " + name + "): " + std::strerror(errno));
    // reserve every page now: a sparse tmpfs file that later outgrows
    // /dev/shm (64 MiB in a default container) faults the writer with SIGBUS
    // mid-run; a reservation that does not fit fails here, and the caller
    // falls back to the gloo plan records
    int rc = ftruncate(fd, (off_t)bytes) != 0 ? errno : posix_fallocate(fd, 0, (off_t)bytes);
    if (rc != 0) {
      close(fd);
      shm_unlink(name.c_str());
      throw std::runtime_error("reserving " + std::to_string(bytes) + " B for " + name + ": " + std::strerror(rc));
    }
    auto* r = new ShmRing(name, fd, bytes, -1);
    Header* h = r->hdr_;
    h->slots = (uint32_t)slots;
    h->slot_bytes = (uint32_t)slot_bytes;
    h->readers = (uint32_t)readers;
    h->head.store(0, std::memory_order_relaxed);
    h->closed.store(0, std::memory_order_relaxed);
    h->producer_pid.store((int64_t)getpid(), std::memory_order_relaxed);
    h->producer_pidns = pid_ns();
    for (int i = 0; i < kMaxReaders; ++i) h->cursor[i].v.store(0, std::memory_order_relaxed);
    // publishes the geometry above: attach() acquire-loads the magic first
    h->magic.store(kMagic, std::memory_order_release);
    return r;
  }

  // Reader `index` (0-based) of an existing segment.
  static ShmRing* attach(const std::string& name, int index) {
    int fd = shm_open(name.c_str(), O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("shm_open(attach " + name + "): " + std::strerror(errno));
    struct stat st;
    if (fstat(fd, &st) != 0) {
      close(fd);
      throw std::runtime_error("fstat(" + name + ")");
    }
    auto* r = new ShmRing(name, fd, (size_t)st.st_size, index);
    if ((size_t)st.st_size < sizeof(Header) || r->hdr_->magic.load(std::memory_order_acquire) != kMagic ||
        index < 0 || index >= (int)r->hdr_->readers) {
      delete r;
      throw std::runtime_error("ShmRing: " + name + " is not a ring or reader index out of range");
    }
    return r;
  }

  ~ShmRing() {
    if (base_) munmap(base_, bytes_);
    if (fd_ >= 0) close(fd_);
  }

  void unlink() { shm_unlink(name_.c_str()); }

  // Producer: publish one message; false on timeout (slowest reader too far behind).
  bool publish(const char* data, size_t n, double timeout_s) {
    Header* h = hdr_;
    if (n + 4 > h->slot_bytes) throw std::length_error("ShmRing: message larger than a slot");
    const uint64_t k = h->head.load(std::memory_order_relaxed);
    auto room = [&] {
      for (uint32_t i = 0; i < h->readers; ++i)
        if (k - h->cursor[i].v.load(std::memory_order_acquire) >= h->slots) return false;
      return true;
    };
    if (!wait(room, timeout_s)) return false;
    char* slot = slot_ptr(k);
    const uint32_t len = (uint32_t)n;
    std::memcpy(slot, &len, 4);
    std::memcpy(slot + 4, data, n);
    h->head.store(k + 1, std::memory_order_release);
    return true;
  }

  // Reader: next message, or false on timeout / close.
  bool read(std::string* out, double timeout_s) {
    Header* h = hdr_;
    auto& cur = h->cursor[index_].v;
    const uint64_t k = cur.load(std::memory_order_relaxed);
    if (!wait([&] { return h->head.load(std::memory_order_acquire) > k || h->closed.load(); }, timeout_s))
      return false;
    if (h->head.load(std::memory_order_acquire) <= k) return false;  // closed, drained
    const char* slot = slot_ptr(k);
    uint32_t len;
    std::memcpy(&len, slot, 4);
    out->assign(slot + 4, len);
    cur.store(k + 1, std::memory_order_release);
    return true;
  }

  void close_ring() { hdr_->closed.store(1, std::memory_order_release); }
  bool closed() const { return hdr_->closed.load(std::memory_order_acquire) != 0; }
  // Is the producing process still there?  (EPERM: alive, owned by another user.)
  bool producer_alive() const {
    const pid_t pid = (pid_t)hdr_->producer_pid.load(std::memory_order_relaxed);
    const uint64_t ns = hdr_->producer_pidns;
    if (ns == 0 || ns != pid_ns()) return true;  // not our pid namespace: no probe possible
    return pid > 0 && (kill(pid, 0) == 0 || errno == EPERM);
  }
  // Inode of this process's pid namespace (0 when /proc does not tell).
  static uint64_t pid_ns() {
    struct stat st;
    return stat("/proc/self/ns/pid", &st) == 0 ? (uint64_t)st.st_ino : 0;
  }
  uint64_t head() const { return hdr_->head.load(std::memory_order_acquire); }
  uint64_t cursor(int i) const { return hdr_->cursor[i].v.load(std::memory_order_acquire); }
  int slots() const { return (int)hdr_->slots; }
  int slot_bytes() const { return (int)hdr_->slot_bytes; }

 private:
  struct alignas(64) Counter {
    std::atomic<uint64_t> v;
  };
  struct Header {
    std::atomic<uint64_t> magic;
    uint32_t slots, slot_bytes, readers, pad;
    std::atomic<int64_t> producer_pid;
    uint64_t producer_pidns;  // written before the magic's release store
    alignas(64) std::atomic<uint64_t> head;
    alignas(64) std::atomic<uint64_t> closed;
    Counter cursor[kMaxReaders];
  };

  ShmRing(std::string name, int fd, size_t bytes, int index) : name_(std::move(name)), fd_(fd), bytes_(bytes), index_(index) {
    base_ = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (base_ == MAP_FAILED) {
      base_ = nullptr;
      throw std::runtime_error("mmap(" + name_ + "): " + std::strerror(errno));
    }
    hdr_ = static_cast<Header*>(base_);
  }

  char* slot_ptr(uint64_t k) const {
    return static_cast<char*>(base_) + sizeof(Header) + (size_t)(k % hdr_->slots) * hdr_->slot_bytes;
  }

  template <typename Cond>
  static bool wait(Cond cond, double timeout_s) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    int sleep_us = 2;
    for (uint64_t spins = 0;; ++spins) {
      if (cond()) return true;
      if (spins < 4000) continue;  // ~tens of us of spinning: the common case
      if (std::chrono::duration<double>(clk::now() - t0).count() > timeout_s) return false;
      std::this_thread::sleep_for(std::chrono::microseconds(sleep_us));
      sleep_us = sleep_us < 200 ? sleep_us * 2 : 200;
    }
  }

  std::string name_;
  int fd_ = -1;
  size_t bytes_ = 0;
  int index_ = -1;
  void* base_ = nullptr;
  Header* hdr_ = nullptr;
};

}  // namespace lsd_rt
