// HIP IPC for the intra-node parameter-server data plane (parallel/ps_shm.py).
//
// A PS task keeps its variable shard, optimizer slots and one gradient inbox per trainer in its own GPU's HBM
// and exports them with IPC handles; trainers map them (hipIpcOpenMemHandle, peer access enabled lazily) and
// move gradients in / parameters out with device-to-device copies over xGMI on their own streams — the
// SURVEY T4 design (hipMemcpyPeerAsync into IPC-mapped HBM) replacing TF's gRPC Send/Recv of the reference
// (trainer/task.py:236). Requires HSA_ENABLE_IPC_MODE_LEGACY=0 (dmabuf IPC) on this driver.
#include <hip/hip_runtime.h>
#include <string.h>

#include "common.h"

// Export the allocation holding `ptr`: 64-byte IPC handle + byte offset of ptr inside the allocation (the caching
// allocator sub-allocates, so the handle names the whole segment).
DTF_API int dtf_ipc_export(void* ptr, void* handle_out, long* offset_out) {
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  hipError_t e = hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr);
  if (e != hipSuccess) return (int)e;
  hipIpcMemHandle_t h;
  e = hipIpcGetMemHandle(&h, (void*)base);
  if (e != hipSuccess) return (int)e;
  static_assert(sizeof(hipIpcMemHandle_t) <= 64, "IPC handle larger than 64 bytes");
  memset(handle_out, 0, 64);
  memcpy(handle_out, &h, sizeof(h));
  *offset_out = (long)((char*)ptr - (char*)base);
  return 0;
}

// Map a peer allocation into this process (current device): *ptr_out = its base address.
DTF_API int dtf_ipc_open(const void* handle, void** ptr_out) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr_out, h, hipIpcMemLazyEnablePeerAccess);
}

DTF_API int dtf_ipc_close(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }

// Stream-ordered copy between any two device addresses of this process (local or IPC-mapped peer memory).
DTF_API int dtf_memcpy_async(void* dst, const void* src, long bytes, void* stream) {
  if (bytes <= 0) return 0;
  return (int)hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream);
}

// A non-blocking HIP stream created NOW (not taken from PyTorch's lazily created stream pool): the framework's
// weight-gradient / collective side stream is created before the process group initialises RCCL, so it takes its
// own hardware queue ahead of RCCL's streams at HIP's default of 4 queues per process (round 3 measured the side
// stream landing on the main stream's queue when it was created after RCCL: profiles/r3_hw_queues.txt).
DTF_API void* dtf_stream_create(int priority) {
  hipStream_t s = nullptr;
  if (hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority) != hipSuccess) return nullptr;
  return (void*)s;
}
