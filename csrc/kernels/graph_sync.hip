// Cross-stream ordering for the per-stream hipGraph executor (graphs.py "split" capture): a train step whose kernels
// run on several streams (main dgrad chain, weight-gradient side stream, communication stream, update stream) is
// captured as ONE graph PER STREAM and replayed by launching each graph into its own stream, so the kernels keep the
// hardware queue they had eagerly and overlap exactly as they do eagerly (a single multi-branch graph lets the HIP
// runtime re-map its branches onto queues of its own choice: 7% slower on ResNet-50, profiles/r4_negative_results.txt).
//
// The graphs are launched in a fixed order (main first). An edge from an EARLIER-launched stream's graph to a later
// one is an event record/wait node pair added to the two graphs by hand (the wait binds at enqueue time to the record
// the earlier graph just enqueued). An edge the other way (a later graph's work that an
// earlier graph waits for: the joins at the end of backward) cannot bind at enqueue time, so it is a device-side flag:
//   * every graph starts with xs_epoch_inc (its replay counter += 1; all graphs replay once per step, so the
//     counters agree),
//   * the producer stream runs xs_signal (flag[slot] = its counter, release) after the work the edge orders,
//   * the consumer stream runs xs_wait (one wave spins until flag[slot] >= its own counter, acquire).
// Every spin is bounded (timeout_ms of s_memrealtime): on a timeout *err is set and the kernel returns, so a broken
// edge can never hang the GPU; the executor checks err and raises. Vector memory only (agent-scope atomics).
#include "common.h"

namespace {

__global__ void xs_epoch_inc_kernel(int* epochs, int idx) {
  if (threadIdx.x == 0) {
    const int v = __hip_atomic_load(epochs + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(epochs + idx, v + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void xs_signal_kernel(int* flags, int slot, const int* epochs, int idx) {
  if (threadIdx.x == 0) {
    const int e = __hip_atomic_load(epochs + idx, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_store(flags + slot, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void xs_wait_kernel(const int* flags, int slot, const int* epochs, int idx, int* err, long timeout) {
  if (threadIdx.x == 0) {
    const int e = __hip_atomic_load(epochs + idx, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const long t0 = (long)__builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(flags + slot, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < e) {
      __builtin_amdgcn_s_sleep(4);
      if ((long)__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
        __hip_atomic_store(err, slot + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
}

}  // namespace

DTF_API int dtf_xs_epoch_inc(int* epochs, int idx, void* stream) {
  hipLaunchKernelGGL(xs_epoch_inc_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, epochs, idx);
  return (int)hipGetLastError();
}

DTF_API int dtf_xs_signal(int* flags, int slot, const int* epochs, int idx, void* stream) {
  hipLaunchKernelGGL(xs_signal_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, flags, slot, epochs, idx);
  return (int)hipGetLastError();
}

DTF_API int dtf_xs_wait(const int* flags, int slot, const int* epochs, int idx, int* err, int timeout_ms,
                        void* stream) {
  hipLaunchKernelGGL(xs_wait_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, flags, slot, epochs, idx, err,
                     (long)timeout_ms * 100000L);  // s_memrealtime: 100 MHz
  return (int)hipGetLastError();
}

// Events for the external record/wait node pairs (no timing: a record is a marker packet).
DTF_API void* dtf_event_create() {
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
  return e;
}

DTF_API int dtf_event_destroy(void* e) { return e ? (int)hipEventDestroy((hipEvent_t)e) : 0; }

// Append an event node to a capturing stream's graph by hand (hipEventRecordWithFlags(External) is refused under
// capture by this HIP): the node depends on the stream's current capture frontier and becomes the new frontier.
static int add_event_node(hipStream_t s, hipEvent_t e, bool record) {
  hipStreamCaptureStatus st;
  unsigned long long id = 0;
  hipGraph_t g = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t nd = 0;
  hipError_t r = hipStreamGetCaptureInfo_v2(s, &st, &id, &g, &deps, &nd);
  if (r != hipSuccess) return (int)r;
  if (st != hipStreamCaptureStatusActive || !g) return -100;
  hipGraphNode_t node = nullptr;
  r = record ? hipGraphAddEventRecordNode(&node, g, deps, nd, e) : hipGraphAddEventWaitNode(&node, g, deps, nd, e);
  if (r != hipSuccess) return (int)r;
  return (int)hipStreamUpdateCaptureDependencies(s, &node, 1, hipStreamSetCaptureDependencies);
}

// Record `e` on `stream`: an event-record node of the stream's graph while it captures, a plain record otherwise.
DTF_API int dtf_event_record_external(void* e, void* stream) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing((hipStream_t)stream, &st) == hipSuccess && st == hipStreamCaptureStatusActive)
    return add_event_node((hipStream_t)stream, (hipEvent_t)e, true);
  return (int)hipEventRecord((hipEvent_t)e, (hipStream_t)stream);
}

// `stream` waits for the last record of `e`: an event-wait node while it captures, a plain wait otherwise.
DTF_API int dtf_stream_wait_external(void* stream, void* e) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing((hipStream_t)stream, &st) == hipSuccess && st == hipStreamCaptureStatusActive)
    return add_event_node((hipStream_t)stream, (hipEvent_t)e, false);
  return (int)hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)e, 0);
}
