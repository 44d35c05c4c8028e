// RCCL communicator owned by the framework: the GPU collective data plane driven from C++ (SURVEY §1.2 "RCCL over
// xGMI"; the reference's CollectiveAllReduce is TF's C++ NCCL manager, /root/reference/trainer/task.py:150-175 builds
// MirroredStrategy / MultiWorkerMirroredStrategy on top of it).
//
// librccl is bound at run time (dlopen/dlsym), not at link time:
//   * the process usually has PyTorch's bundled librccl.so.1 loaded already; RTLD_NOLOAD picks that copy first, so
//     one RCCL (one set of proxy threads, one topology probe) serves both torch.distributed and this communicator;
//   * the runtime library still loads on hosts without ROCm (CPU tests, the gloo paths).
// The ABI pieces used here (opaque communicator, 128-byte unique id, the ncclConfig_t prefix, the data type and
// reduction enums) are stable across RCCL 2.2x.
//
// Channel configuration: every collective kernel runs one CTA per channel and a ring channel drives one xGMI link in
// each direction, so the communicator is created with minCTAs >= 8 (all 7 point-to-point links of an MI355X busy on
// an 8-GPU ring set) and a maxCTAs cap (the CUs a collective may take from the overlapped backward pass).
#include <dlfcn.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <string>

#define DTF_API extern "C" __attribute__((visibility("default")))

namespace {

typedef int nres_t;  // ncclResult_t
typedef void* ncomm_t;
struct NUid {
  char internal[128];
};
// ncclConfig_t as laid out by RCCL 2.26 and 2.27 (fields after nvlsCTAs are not used). The layout is NOT a stable ABI
// across releases: load() refuses any other version (kMinVersion..kMaxVersion), and the framework then falls back
// to torch.distributed's process group.
constexpr int kMinVersion = 22600, kMaxVersion = 22799;
struct NConfig {
  size_t size;
  unsigned int magic;
  unsigned int version;
  int blocking;
  int cgaClusterSize;
  int minCTAs;
  int maxCTAs;
  const char* netName;
  int splitShare;
  int trafficClass;
  const char* commName;
  int collnetEnable;
  int CTAPolicy;
  int shrinkShare;
  int nvlsCTAs;
};
constexpr int kUndefInt = (int)0x80000000;  // NCCL_CONFIG_UNDEF_INT

struct Api {
  void* lib = nullptr;
  nres_t (*GetVersion)(int*) = nullptr;
  nres_t (*GetUniqueId)(NUid*) = nullptr;
  nres_t (*CommInitRankConfig)(ncomm_t*, int, NUid, int, NConfig*) = nullptr;
  nres_t (*CommDestroy)(ncomm_t) = nullptr;
  nres_t (*CommAbort)(ncomm_t) = nullptr;
  nres_t (*CommFinalize)(ncomm_t) = nullptr;
  nres_t (*CommGetAsyncError)(ncomm_t, nres_t*) = nullptr;
  nres_t (*CommCount)(ncomm_t, int*) = nullptr;
  nres_t (*CommUserRank)(ncomm_t, int*) = nullptr;
  nres_t (*AllReduce)(const void*, void*, size_t, int, int, ncomm_t, void*) = nullptr;
  nres_t (*ReduceScatter)(const void*, void*, size_t, int, int, ncomm_t, void*) = nullptr;
  nres_t (*AllGather)(const void*, void*, size_t, int, ncomm_t, void*) = nullptr;
  nres_t (*Broadcast)(const void*, void*, size_t, int, int, ncomm_t, void*) = nullptr;
  nres_t (*Send)(const void*, size_t, int, int, ncomm_t, void*) = nullptr;
  nres_t (*Recv)(void*, size_t, int, int, ncomm_t, void*) = nullptr;
  nres_t (*GroupStart)() = nullptr;
  nres_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(nres_t) = nullptr;
  int version = 0;
  std::string where;
};

Api g_api;
std::once_flag g_once;
std::string g_err;

template <typename F>
bool sym(void* lib, const char* name, F& out) {
  out = reinterpret_cast<F>(dlsym(lib, name));
  return out != nullptr;
}

void load() {
  static const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
  void* lib = nullptr;
  for (const char* n : names) {  // an RCCL the process already has (PyTorch's) first
    lib = dlopen(n, RTLD_NOW | RTLD_NOLOAD | RTLD_GLOBAL);
    if (lib) { g_api.where = std::string(n) + " (already loaded)"; break; }
  }
  for (int i = 0; !lib && i < 3; ++i) {
    lib = dlopen(names[i], RTLD_NOW | RTLD_GLOBAL);
    if (lib) g_api.where = names[i];
  }
  if (!lib) {
    const char* e = dlerror();
    g_err = std::string("librccl not loadable: ") + (e ? e : "?");
    return;
  }
  Api& a = g_api;
  bool ok = sym(lib, "ncclGetVersion", a.GetVersion) && sym(lib, "ncclGetUniqueId", a.GetUniqueId) &&
            sym(lib, "ncclCommInitRankConfig", a.CommInitRankConfig) && sym(lib, "ncclCommDestroy", a.CommDestroy) &&
            sym(lib, "ncclCommAbort", a.CommAbort) && sym(lib, "ncclCommGetAsyncError", a.CommGetAsyncError) &&
            sym(lib, "ncclCommCount", a.CommCount) && sym(lib, "ncclCommUserRank", a.CommUserRank) &&
            sym(lib, "ncclAllReduce", a.AllReduce) && sym(lib, "ncclReduceScatter", a.ReduceScatter) &&
            sym(lib, "ncclAllGather", a.AllGather) && sym(lib, "ncclBroadcast", a.Broadcast) &&
            sym(lib, "ncclSend", a.Send) && sym(lib, "ncclRecv", a.Recv) && sym(lib, "ncclGroupStart", a.GroupStart) &&
            sym(lib, "ncclGroupEnd", a.GroupEnd) && sym(lib, "ncclGetErrorString", a.GetErrorString);
  sym(lib, "ncclCommFinalize", a.CommFinalize);  // optional
  if (!ok) {
    g_err = "librccl lacks an expected symbol";
    return;
  }
  if (a.GetVersion(&a.version) != 0) a.version = 0;
  if (a.version < kMinVersion || a.version > kMaxVersion) {
    g_err = "RCCL version " + std::to_string(a.version) + " outside the ncclConfig_t layouts this binding knows (" +
            std::to_string(kMinVersion) + ".." + std::to_string(kMaxVersion) + ")";
    return;
  }
  a.lib = lib;
}

bool ready() {
  std::call_once(g_once, load);
  return g_api.lib != nullptr;
}

struct Comm {
  ncomm_t c = nullptr;
  int nranks = 0, rank = 0, min_ctas = 0, max_ctas = 0;
  long calls = 0;
  long long bytes = 0;
};

int dsize(int dt) {  // ncclDataType_t element size
  switch (dt) {
    case 0: case 1: return 1;            // int8, uint8
    case 2: case 3: case 7: return 4;    // int32, uint32, float32
    case 4: case 5: case 8: return 8;    // int64, uint64, float64
    case 6: case 9: return 2;            // float16, bfloat16
    default: return 1;                   // fp8 formats
  }
}

}  // namespace

// 0 when librccl is usable; else -1 and *msg (optional) names the reason.
DTF_API int dtfrt_rccl_available(const char** msg) {
  const bool ok = ready();
  if (msg) *msg = ok ? g_api.where.c_str() : g_err.c_str();
  return ok ? 0 : -1;
}

DTF_API int dtfrt_rccl_version() { return ready() ? g_api.version : -1; }

DTF_API const char* dtfrt_rccl_error_string(int code) {
  if (!ready()) return g_err.c_str();
  return g_api.GetErrorString(code);
}

// A fresh unique id (rank 0 of a communicator draws it and publishes the 128 bytes through the rendezvous store).
DTF_API int dtfrt_rccl_unique_id(char* out128) {
  if (!ready()) return -1;
  NUid id;
  const nres_t r = g_api.GetUniqueId(&id);
  if (r == 0) memcpy(out128, id.internal, 128);
  return r;
}

// Create this rank's communicator on the CURRENT HIP device (the caller binds it). min_ctas / max_ctas <= 0 leave
// RCCL's choice. Returns the handle or null (*err = the ncclResult_t).
DTF_API void* dtfrt_rccl_comm_init(const char* id128, int nranks, int rank, int min_ctas, int max_ctas,
                                 const char* name, int* err) {
  if (err) *err = -1;
  if (!ready() || nranks < 1 || rank < 0 || rank >= nranks) return nullptr;
  NUid id;
  memcpy(id.internal, id128, 128);
  NConfig cfg;
  memset(&cfg, 0, sizeof(cfg));
  cfg.size = sizeof(NConfig);
  cfg.magic = 0xcafebeef;
  cfg.version = (unsigned)(g_api.version > 0 ? g_api.version : 22600);
  cfg.blocking = 1;
  cfg.cgaClusterSize = kUndefInt;
  cfg.minCTAs = min_ctas > 0 ? min_ctas : kUndefInt;
  cfg.maxCTAs = max_ctas > 0 ? max_ctas : kUndefInt;
  cfg.netName = nullptr;
  cfg.splitShare = kUndefInt;
  cfg.trafficClass = kUndefInt;
  cfg.commName = name;
  cfg.collnetEnable = kUndefInt;
  cfg.CTAPolicy = kUndefInt;
  cfg.shrinkShare = kUndefInt;
  cfg.nvlsCTAs = kUndefInt;
  Comm* c = new Comm();
  const nres_t r = g_api.CommInitRankConfig(&c->c, nranks, id, rank, &cfg);
  if (err) *err = r;
  if (r != 0) {
    delete c;
    return nullptr;
  }
  c->nranks = nranks;
  c->rank = rank;
  c->min_ctas = min_ctas;
  c->max_ctas = max_ctas;
  return c;
}

// abort = 1: ncclCommAbort (a peer died / a collective will never complete), else finalize + destroy.
DTF_API int dtfrt_rccl_comm_destroy(void* h, int abort) {
  Comm* c = static_cast<Comm*>(h);
  if (!c) return 0;
  nres_t r = 0;
  if (ready() && c->c) {
    if (abort) {
      r = g_api.CommAbort(c->c);
    } else {
      if (g_api.CommFinalize) r = g_api.CommFinalize(c->c);
      const nres_t r2 = g_api.CommDestroy(c->c);
      if (r == 0) r = r2;
    }
  }
  delete c;
  return r;
}

DTF_API int dtfrt_rccl_comm_info(void* h, int* nranks, int* rank, long* calls, long long* bytes) {
  Comm* c = static_cast<Comm*>(h);
  if (!c || !ready()) return -1;
  int n = 0, r = 0;
  nres_t e = g_api.CommCount(c->c, &n);
  if (e == 0) e = g_api.CommUserRank(c->c, &r);
  if (nranks) *nranks = n;
  if (rank) *rank = r;
  if (calls) *calls = c->calls;
  if (bytes) *bytes = c->bytes;
  return e;
}

// Asynchronous error state of the communicator (0 = fine; a peer failure surfaces here without a host hang).
DTF_API int dtfrt_rccl_async_error(void* h) {
  Comm* c = static_cast<Comm*>(h);
  if (!c || !ready()) return -1;
  nres_t a = 0;
  const nres_t e = g_api.CommGetAsyncError(c->c, &a);
  return e != 0 ? e : a;
}

// Collectives, stream-ordered on `stream` (a hipStream_t; null = the legacy default stream). dtype / op are the
// ncclDataType_t / ncclRedOp_t values (7 float32, 9 bfloat16; 0 sum, 2 max, 3 min, 4 avg).
DTF_API int dtfrt_rccl_all_reduce(void* h, const void* send, void* recv, long count, int dtype, int op, void* stream) {
  Comm* c = static_cast<Comm*>(h);
  if (!c || !ready()) return -1;
  c->calls++;
  c->bytes += (long long)count * dsize(dtype);
  return g_api.AllReduce(send, recv, (size_t)count, dtype, op, c->c, stream);
}

// recv (count elements) = the reduced chunk `rank` of send (nranks * count elements)
DTF_API int dtfrt_rccl_reduce_scatter(void* h, const void* send, void* recv, long count, int dtype, int op,
                                    void* stream) {
  Comm* c = static_cast<Comm*>(h);
  if (!c || !ready()) return -1;
  c->calls++;
  c->bytes += (long long)count * c->nranks * dsize(dtype);
  return g_api.ReduceScatter(send, recv, (size_t)count, dtype, op, c->c, stream);
}

// recv (nranks * count elements) = every rank's send (count elements) in rank order
DTF_API int dtfrt_rccl_all_gather(void* h, const void* send, void* recv, long count, int dtype, void* stream) {
  Comm* c = static_cast<Comm*>(h);
  if (!c || !ready()) return -1;
  c->calls++;
  c->bytes += (long long)count * c->nranks * dsize(dtype);
  return g_api.AllGather(send, recv, (size_t)count, dtype, c->c, stream);
}

DTF_API int dtfrt_rccl_broadcast(void* h, const void* send, void* recv, long count, int dtype, int root, void* stream) {
  Comm* c = static_cast<Comm*>(h);
  if (!c || !ready()) return -1;
  c->calls++;
  c->bytes += (long long)count * dsize(dtype);
  return g_api.Broadcast(send, recv, (size_t)count, dtype, root, c->c, stream);
}

// Point-to-point (pipeline / parameter-server style transfers); wrap several in group_start / group_end.
DTF_API int dtfrt_rccl_send(void* h, const void* buf, long count, int dtype, int peer, void* stream) {
  Comm* c = static_cast<Comm*>(h);
  if (!c || !ready()) return -1;
  c->calls++;
  c->bytes += (long long)count * dsize(dtype);
  return g_api.Send(buf, (size_t)count, dtype, peer, c->c, stream);
}

DTF_API int dtfrt_rccl_recv(void* h, void* buf, long count, int dtype, int peer, void* stream) {
  Comm* c = static_cast<Comm*>(h);
  if (!c || !ready()) return -1;
  c->calls++;
  return g_api.Recv(buf, (size_t)count, dtype, peer, c->c, stream);
}

DTF_API int dtfrt_rccl_group_start() { return ready() ? g_api.GroupStart() : -1; }
DTF_API int dtfrt_rccl_group_end() { return ready() ? g_api.GroupEnd() : -1; }
