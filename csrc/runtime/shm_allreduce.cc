// CPU all-reduce across the processes of one host through POSIX shared memory.
//
// The BASELINE plumbing config "MNIST MLP MirroredStrategy on CPU:0,CPU:1, world_size=2" and the
// multi-process CPU tests reduce gradients here instead of over loopback TCP: every rank copies
// its buffer into its slot, a sense-reversing barrier, each rank sums its 1/world chunk across
// all slots into the result area (reduce-scatter), barrier, every rank copies the full result
// (all-gather), barrier. Slots are reused call after call.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <string>
#include <thread>

#include "runtime.h"

using namespace dtfrt;

namespace {

struct Header {
  std::atomic<int> count;
  std::atomic<int> sense;
  std::atomic<int> ready;
  int world;
  uint64_t slot_bytes;
};

struct Shm {
  std::string name;
  int rank, world;
  uint64_t slot_bytes;
  size_t total;
  char* base;
  int local_sense = 0;
  Header* hdr() { return (Header*)base; }
  float* slot(int r) { return (float*)(base + 4096 + (size_t)r * slot_bytes); }
  float* result() { return (float*)(base + 4096 + (size_t)world * slot_bytes); }
};

bool barrier(Shm* s, int timeout_ms = 600000) {
  Header* h = s->hdr();
  s->local_sense ^= 1;
  if (h->count.fetch_add(1) + 1 == s->world) {
    h->count.store(0);
    h->sense.store(s->local_sense);
    return true;
  }
  auto t0 = std::chrono::steady_clock::now();
  int spins = 0;
  while (h->sense.load() != s->local_sense) {
    if (++spins > 1000) {
      std::this_thread::sleep_for(std::chrono::microseconds(20));
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms)) return false;
    }
  }
  return true;
}

}  // namespace

DTF_RT void* dtfrt_shm_open(const char* name, int rank, int world, uint64_t max_bytes) {
  auto* s = new Shm;
  s->name = std::string("/dtf_") + name;
  s->rank = rank;
  s->world = world;
  s->slot_bytes = (max_bytes + 4095) / 4096 * 4096;
  s->total = 4096 + (size_t)(world + 1) * s->slot_bytes;
  int fd = -1;
  if (rank == 0) {
    shm_unlink(s->name.c_str());
    fd = shm_open(s->name.c_str(), O_CREAT | O_RDWR, 0600);
    if (fd >= 0 && ftruncate(fd, (off_t)s->total) != 0) {
      close(fd);
      fd = -1;
    }
  } else {
    for (int i = 0; i < 20000 && fd < 0; ++i) {
      fd = shm_open(s->name.c_str(), O_RDWR, 0600);
      if (fd < 0) std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
  }
  if (fd < 0) {
    set_error("shm_open %s failed", s->name.c_str());
    delete s;
    return nullptr;
  }
  // wait until the creator has sized the segment
  for (int i = 0; i < 20000; ++i) {
    struct stat st;
    if (fstat(fd, &st) == 0 && (size_t)st.st_size >= s->total) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  s->base = (char*)mmap(nullptr, s->total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (s->base == MAP_FAILED) {
    set_error("mmap failed");
    delete s;
    return nullptr;
  }
  Header* h = s->hdr();
  if (rank == 0) {
    h->world = world;
    h->slot_bytes = s->slot_bytes;
    h->count.store(0);
    h->sense.store(0);
    h->ready.store(1);
  } else {
    while (h->ready.load() != 1) std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  return s;
}

DTF_RT int dtfrt_shm_barrier(void* hp) { return barrier((Shm*)hp) ? 0 : -1; }

DTF_RT int dtfrt_shm_allreduce_f32(void* hp, void* data, uint64_t n) {
  auto* s = (Shm*)hp;
  uint64_t chunk_max = s->slot_bytes / 4;
  float* x = (float*)data;
  for (uint64_t base = 0; base < n; base += chunk_max) {
    uint64_t m = std::min<uint64_t>(chunk_max, n - base);
    memcpy(s->slot(s->rank), x + base, m * 4);
    if (!barrier(s)) return -1;
    uint64_t per = (m + s->world - 1) / s->world;
    uint64_t lo = per * s->rank, hi = std::min<uint64_t>(m, lo + per);
    float* res = s->result();
    for (uint64_t i = lo; i < hi; ++i) {
      float acc = 0.f;
      for (int r = 0; r < s->world; ++r) acc += s->slot(r)[i];
      res[i] = acc;
    }
    if (!barrier(s)) return -1;
    memcpy(x + base, res, m * 4);
    if (!barrier(s)) return -1;
  }
  return 0;
}

DTF_RT void dtfrt_shm_close(void* hp, int unlink_it) {
  auto* s = (Shm*)hp;
  munmap(s->base, s->total);
  if (unlink_it) shm_unlink(s->name.c_str());
  delete s;
}
