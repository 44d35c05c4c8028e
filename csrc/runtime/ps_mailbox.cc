// Intra-node parameter-server control channel: a POSIX shared-memory mailbox with futex doorbells.
//
// The reference moves every gradient push / parameter pull through TF's gRPC Send/Recv rendezvous
// (reference trainer/task.py:236 [TF-RT]). On one node the bytes themselves move by direct copies
// between the trainers' and the PS's memory (HIP IPC-mapped HBM between GPUs over xGMI, or a shared-memory
// region for a CPU PS — parallel/ps_shm.py); this file is the small control plane around those copies:
//
//   * one mailbox per PS task, one 64-B slot per trainer: the trainer writes the request (op, arg), bumps the
//     slot's `req` sequence number (release) and rings the box's doorbell (futex wake); the PS's single serve
//     loop waits on the doorbell, scans the slots for req > done, handles them in arrival order, stores the
//     status and bumps `done` (release) + futex-wakes the trainer waiting on that word.
//   * no per-trainer threads, no sockets, no GPU kernels spinning: a PS serves any number of trainers from one
//     thread, and the RCCL hardware queues stay free for the collectives.
//   * `dtfrt_shmem_*`: named shared-memory regions (the CPU PS's published parameters / gradient inboxes).
// Futex words are 32-bit atomics in the shared mapping (no FUTEX_PRIVATE_FLAG: they are cross-process).
#include <errno.h>
#include <fcntl.h>
#include <linux/futex.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <string>
#include <thread>

#include "runtime.h"

using namespace dtfrt;

namespace {

constexpr uint32_t MAGIC = 0x44544d42;  // "DTMB"

struct alignas(64) Slot {
  std::atomic<uint32_t> req;   // requests posted by the trainer
  std::atomic<uint32_t> done;  // requests completed by the PS
  std::atomic<int32_t> op;
  std::atomic<int32_t> status;
  std::atomic<uint64_t> arg;
};
static_assert(sizeof(Slot) == 64, "slot = one cache line");

struct alignas(64) BoxHeader {
  std::atomic<uint32_t> magic;
  uint32_t nslots;
  std::atomic<uint32_t> doorbell;
  std::atomic<uint32_t> closed;
};

struct Box {
  std::string name;
  size_t bytes;
  char* base;
  bool owner;
  uint32_t cursor = 0;  // PS scan position (round robin over slots)
  BoxHeader* hdr() { return (BoxHeader*)base; }
  Slot* slot(int i) { return (Slot*)(base + 64) + i; }
};

long futex(std::atomic<uint32_t>* addr, int op, uint32_t val, const struct timespec* ts) {
  return syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), op, val, ts, nullptr, 0);
}

void wake_all(std::atomic<uint32_t>* w) { futex(w, FUTEX_WAKE, 0x7fffffff, nullptr); }

// Wait until *w != seen or timeout (a short spin first: requests on one node are answered in microseconds).
void wait_change(std::atomic<uint32_t>* w, uint32_t seen, int timeout_ms) {
  for (int i = 0; i < 256; ++i) {
    if (w->load(std::memory_order_acquire) != seen) return;
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
  }
  struct timespec ts;
  const int ms = timeout_ms < 0 ? 1000 : std::min(timeout_ms, 1000);
  ts.tv_sec = ms / 1000;
  ts.tv_nsec = (long)(ms % 1000) * 1000000L;
  futex(w, FUTEX_WAIT, seen, &ts);
}

std::string shm_name(const char* name) { return name[0] == '/' ? std::string(name) : "/" + std::string(name); }

char* map_fd(int fd, size_t bytes) {
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  return p == MAP_FAILED ? nullptr : (char*)p;
}

}  // namespace

// ---- mailbox -------------------------------------------------------------------------------------------------
DTF_RT void* dtfrt_mbox_create(const char* name, int nslots) {
  const std::string n = shm_name(name);
  const size_t bytes = 64 + (size_t)nslots * sizeof(Slot);
  shm_unlink(n.c_str());  // a stale box of a crashed run
  int fd = shm_open(n.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0 || ftruncate(fd, (off_t)bytes) != 0) {
    set_error("mbox create %s: %s", n.c_str(), strerror(errno));
    if (fd >= 0) close(fd);
    return nullptr;
  }
  char* p = map_fd(fd, bytes);
  close(fd);
  if (!p) {
    set_error("mbox mmap %s: %s", n.c_str(), strerror(errno));
    return nullptr;
  }
  memset(p, 0, bytes);
  auto* b = new Box{n, bytes, p, true};
  b->hdr()->nslots = (uint32_t)nslots;
  b->hdr()->magic.store(MAGIC, std::memory_order_release);
  return b;
}

DTF_RT void* dtfrt_mbox_open(const char* name, int timeout_ms) {
  const std::string n = shm_name(name);
  auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    int fd = shm_open(n.c_str(), O_RDWR, 0600);
    if (fd >= 0) {
      struct stat st;
      if (fstat(fd, &st) == 0 && st.st_size >= 64) {
        char* p = map_fd(fd, (size_t)st.st_size);
        close(fd);
        if (p && ((BoxHeader*)p)->magic.load(std::memory_order_acquire) == MAGIC)
          return new Box{n, (size_t)st.st_size, p, false};
        if (p) munmap(p, (size_t)st.st_size);
      } else {
        close(fd);
      }
    }
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms)) {
      set_error("mbox open %s: timed out", n.c_str());
      return nullptr;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
}

// Trainer: post a request on `slot`; returns its sequence number (> 0).
DTF_RT int64_t dtfrt_mbox_post(void* h, int slot, int op, uint64_t arg) {
  auto* b = (Box*)h;
  if (slot < 0 || (uint32_t)slot >= b->hdr()->nslots) return -1;
  Slot* s = b->slot(slot);
  s->op.store(op, std::memory_order_relaxed);
  s->arg.store(arg, std::memory_order_relaxed);
  const uint32_t seq = s->req.fetch_add(1, std::memory_order_acq_rel) + 1;
  b->hdr()->doorbell.fetch_add(1, std::memory_order_acq_rel);
  wake_all(&b->hdr()->doorbell);
  return seq;
}

// Trainer: wait for request `seq` of `slot` to complete. Returns its status, or -1000 on timeout / closed box.
DTF_RT int dtfrt_mbox_wait(void* h, int slot, int64_t seq, int timeout_ms) {
  auto* b = (Box*)h;
  Slot* s = b->slot(slot);
  auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const uint32_t d = s->done.load(std::memory_order_acquire);
    if ((int32_t)(d - (uint32_t)seq) >= 0) return s->status.load(std::memory_order_relaxed);
    if (b->hdr()->closed.load(std::memory_order_acquire)) {
      set_error("mbox %s closed while waiting", b->name.c_str());
      return -1000;
    }
    if (timeout_ms >= 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms)) {
      set_error("mbox %s slot %d: request %lld timed out", b->name.c_str(), slot, (long long)seq);
      return -1000;
    }
    wait_change(&s->done, d, timeout_ms);
  }
}

// PS: next pending request (round robin over slots). Returns 1 and fills the outputs, 0 on timeout.
DTF_RT int dtfrt_mbox_next(void* h, int timeout_ms, int* slot, int* op, int64_t* seq, uint64_t* arg) {
  auto* b = (Box*)h;
  const uint32_t n = b->hdr()->nslots;
  auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const uint32_t bell = b->hdr()->doorbell.load(std::memory_order_acquire);
    for (uint32_t k = 0; k < n; ++k) {
      const uint32_t i = (b->cursor + k) % n;
      Slot* s = b->slot((int)i);
      const uint32_t r = s->req.load(std::memory_order_acquire), d = s->done.load(std::memory_order_relaxed);
      if (r != d) {  // one request per slot in flight: it is number d + 1
        *slot = (int)i;
        *op = s->op.load(std::memory_order_relaxed);
        *arg = s->arg.load(std::memory_order_relaxed);
        *seq = (int64_t)(d + 1);
        b->cursor = (i + 1) % n;
        return 1;
      }
    }
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms)) return 0;
    wait_change(&b->hdr()->doorbell, bell, timeout_ms);
  }
}

// PS: complete request `seq` of `slot` with `status` and wake the trainer.
DTF_RT int dtfrt_mbox_complete(void* h, int slot, int64_t seq, int status) {
  auto* b = (Box*)h;
  Slot* s = b->slot(slot);
  s->status.store(status, std::memory_order_relaxed);
  s->done.store((uint32_t)seq, std::memory_order_release);
  wake_all(&s->done);
  return 0;
}

DTF_RT void dtfrt_mbox_close(void* h, int unlink_it) {
  auto* b = (Box*)h;
  if (b->owner) {
    b->hdr()->closed.store(1, std::memory_order_release);
    for (uint32_t i = 0; i < b->hdr()->nslots; ++i) wake_all(&b->slot((int)i)->done);
  }
  munmap(b->base, b->bytes);
  if (unlink_it) shm_unlink(b->name.c_str());
  delete b;
}

// ---- named shared-memory regions ---------------------------------------------------------------------------------
DTF_RT void* dtfrt_shmem_create(const char* name, uint64_t bytes) {
  const std::string n = shm_name(name);
  shm_unlink(n.c_str());
  int fd = shm_open(n.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0 || ftruncate(fd, (off_t)bytes) != 0) {
    set_error("shmem create %s: %s", n.c_str(), strerror(errno));
    if (fd >= 0) close(fd);
    return nullptr;
  }
  char* p = map_fd(fd, (size_t)bytes);
  close(fd);
  if (!p) set_error("shmem mmap %s: %s", n.c_str(), strerror(errno));
  return p;
}

DTF_RT void* dtfrt_shmem_open(const char* name, uint64_t bytes, int timeout_ms) {
  const std::string n = shm_name(name);
  auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    int fd = shm_open(n.c_str(), O_RDWR, 0600);
    if (fd >= 0) {
      struct stat st;
      if (fstat(fd, &st) == 0 && (uint64_t)st.st_size >= bytes) {
        char* p = map_fd(fd, (size_t)bytes);
        close(fd);
        if (!p) set_error("shmem mmap %s: %s", n.c_str(), strerror(errno));
        return p;
      }
      close(fd);
    }
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms)) {
      set_error("shmem open %s: timed out", n.c_str());
      return nullptr;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
}

DTF_RT void dtfrt_shmem_close(void* p, uint64_t bytes, const char* name, int unlink_it) {
  if (p) munmap(p, (size_t)bytes);
  if (unlink_it && name) shm_unlink(shm_name(name).c_str());
}
