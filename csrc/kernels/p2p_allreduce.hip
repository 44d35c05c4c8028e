// One-shot peer-to-peer all-reduce of a small f32 gradient bucket over IPC-mapped HBM (xGMI between the GPUs of a
// node), for the buckets where RCCL's per-collective latency dominates (SURVEY §2.6 "custom one-shot P2P all-reduce
// over IPC-mapped HBM for small buckets", §5).
//
// Every rank exports its gradient arena, a reduction scratch and a flag array once (parallel/p2p.py); a call then
// runs ONE kernel per rank, `nblk` blocks, block b owning the interleaved slice {b*256*4 + k*nblk*256*4 ...}:
//   1. arrival: lane 0 makes the rank's gradient (written by earlier kernels, possibly still dirty in this GPU's L2)
//      visible system-wide (release fence, system scope), then stores the call's epoch into flag [0][b][rank] of
//      EVERY rank (system-scope relaxed stores into the IPC-mapped flag arrays) and polls its own [0][b][p] until
//      every rank arrived, then acquires (system scope: this CU's caches no longer hold stale peer lines);
//   2. reduce: the block sums its slice over the ranks IN RANK ORDER (every rank computes the identical f32 value:
//      bitwise-identical replicas) into its own scratch;
//   3. departure: after every wave's loads completed (vmcnt(0) + barrier) lane 0 stores the epoch into [1][b][rank]
//      of every rank and polls its own [1][b][p]: no rank may overwrite its gradient while a peer still reads it;
//   4. the block copies its scratch slice into its own gradient.
// Epochs are monotonic per (rank, communicator) and every rank issues the same calls in the same stream order, so
// the flag arrays are reused without resets. Every spin is bounded (~`timeout_ms` of s_memrealtime, 100 MHz): on a
// timeout the block sets *err and runs to completion (the result is then garbage; the host raises).
// Vector memory only: flags are written with system-scope vector atomics/stores.
#include <algorithm>

#include "common.h"

namespace {

constexpr int P2P_MAX_RANKS = 8;
constexpr int P2P_NT = 256;

struct P2PArgs {
  float* dst;                              // this rank's bucket (receives the sum)
  const float* src[P2P_MAX_RANKS];         // every rank's bucket (this rank's own pointer at [rank])
  float* red;                              // this rank's scratch (bucket-sized)
  int* flags_local;                        // this rank's flags [2][nblk][P2P_MAX_RANKS]
  int* flags_peer[P2P_MAX_RANKS];          // every rank's flag array (IPC-mapped; own at [rank])
  long n;                                  // floats
  int head;                                // leading floats before the 16-B aligned body (same on every rank)
  int world, rank, epoch, nblk;
  long timeout_ticks;
  int* err;
};

__device__ __forceinline__ bool wait_flags(const int* f, int world, int epoch, long timeout, int* err) {
  const long t0 = (long)__builtin_amdgcn_s_memrealtime();
  for (int p = 0; p < world; ++p) {
    while (__hip_atomic_load(f + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      __builtin_amdgcn_s_sleep(2);
      if ((long)__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return false;
      }
    }
  }
  return true;
}

__global__ void __launch_bounds__(P2P_NT) p2p_allreduce_kernel(P2PArgs a) {
  const int b = blockIdx.x, t = threadIdx.x;
  __shared__ int ok;
  // 1. arrival
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: this rank's gradient leaves the L2
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int p = 0; p < a.world; ++p)
      __hip_atomic_store(a.flags_peer[p] + b * P2P_MAX_RANKS + a.rank, a.epoch, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    ok = wait_flags(a.flags_local + b * P2P_MAX_RANKS, a.world, a.epoch, a.timeout_ticks, a.err);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // 2. reduce this block's slice in rank order (16-B aligned float4 body; head and tail floats by the last block)
  const long h = a.head, n4 = (a.n - h) >> 2;
  const long step = (long)a.nblk * P2P_NT;
  for (long i = (long)b * P2P_NT + t; i < n4; i += step) {
    float4 s = reinterpret_cast<const float4*>(a.src[0] + h)[i];
    for (int p = 1; p < a.world; ++p) {
      const float4 v = reinterpret_cast<const float4*>(a.src[p] + h)[i];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    reinterpret_cast<float4*>(a.red + h)[i] = s;
  }
  auto scalar = [&](long i) {
    float s = a.src[0][i];
    for (int p = 1; p < a.world; ++p) s += a.src[p][i];
    a.red[i] = s;
  };
  if (b == a.nblk - 1) {
    if (t < h) scalar(t);
    for (long i = h + n4 * 4 + t; i < a.n; i += P2P_NT) scalar(i);
  }
  // 3. departure: every peer finished reading this rank's bucket before it is overwritten
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    for (int p = 0; p < a.world; ++p)
      __hip_atomic_store(a.flags_peer[p] + (a.nblk + b) * P2P_MAX_RANKS + a.rank, a.epoch, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    if (!wait_flags(a.flags_local + (a.nblk + b) * P2P_MAX_RANKS, a.world, a.epoch, a.timeout_ticks, a.err)) ok = 0;
  }
  __syncthreads();
  // 4. the sum into this rank's bucket (the block's own scratch writes: same CU)
  for (long i = (long)b * P2P_NT + t; i < n4; i += step)
    reinterpret_cast<float4*>(a.dst + h)[i] = reinterpret_cast<const float4*>(a.red + h)[i];
  if (b == a.nblk - 1) {
    if (t < h) a.dst[t] = a.red[t];
    for (long i = h + n4 * 4 + t; i < a.n; i += P2P_NT) a.dst[i] = a.red[i];
  }
}

}  // namespace

// srcs / peer_flags: arrays of `world` device pointers (this rank's own at [rank]). dst, every src and red must share
// their address modulo 16 (the same arena offset on 16-B aligned bases); flags_local has >= 2 * nblk * 8 ints.
// Returns 0 when launched.
DTF_API int dtf_p2p_allreduce_f32(float* dst, const void* const* srcs, float* red, int* flags_local,
                                  void* const* peer_flags, long n, int world, int rank, int epoch, int nblk,
                                  int timeout_ms, int* err, void* stream) {
  if (world < 1 || world > P2P_MAX_RANKS || rank < 0 || rank >= world || nblk < 1 || n < 0) return -1;
  const uintptr_t mis = (uintptr_t)dst & 15;
  if ((mis & 3) || ((uintptr_t)red & 15) != mis) return -2;
  P2PArgs a{};
  a.dst = dst;
  a.red = red;
  a.flags_local = flags_local;
  for (int p = 0; p < world; ++p) {
    a.src[p] = (const float*)srcs[p];
    a.flags_peer[p] = (int*)peer_flags[p];
    if (((uintptr_t)a.src[p] & 15) != mis) return -2;
  }
  a.n = n;
  a.head = (int)std::min<long>(n, (long)((16 - mis) & 15) / 4);
  a.world = world;
  a.rank = rank;
  a.epoch = epoch;
  a.nblk = nblk;
  a.timeout_ticks = (long)timeout_ms * 100000L;  // s_memrealtime: 100 MHz
  a.err = err;
  hipLaunchKernelGGL(p2p_allreduce_kernel, dim3(nblk), dim3(P2P_NT), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}
