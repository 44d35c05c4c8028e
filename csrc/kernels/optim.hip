// Fused optimizer kernels over flat parameter arenas (SURVEY §2.4.a K10–K15).
//
// The framework keeps every trainable variable of a model as a view into ONE
// contiguous f32 master arena (plus one f32 gradient arena and one slot arena
// per optimizer slot), so each optimizer update is a single streaming launch
// over the whole model instead of one TF Apply* kernel per variable
// (reference: trainer/task.py:41-56 builds the six TF1 optimizers; their Apply
// ops run once per variable on the PS). The kernel also
//   * scales the gradient (1/replicas, loss-scale, global-norm clip factor),
//   * writes the bf16 compute copy of each updated weight (mixed precision),
//   * optionally zeroes the gradient for the next step,
// all in the same pass: 3-5 f32 streams read once, written once.
//
// Hyper-parameters that change per step (bias-corrected Adam lr, lr schedule)
// are read from a small device array `hp` so a hipGraph-captured train step
// picks up new values without re-capture:
//   hp[0] = lr (already bias corrected for Adam), hp[1] = grad scale,
//   hp[2] = global-norm clip threshold (<=0: off); sumsq (optional) = sum g^2.
#include "common.h"

namespace {

enum OptKind : int {
  OPT_SGD = 0,       // p -= lr*g ; momentum: m = mu*m + g, p -= lr*m (nesterov: p -= lr*(g + mu*m))
  OPT_ADAM = 1,      // TF1/Keras eps-hat Adam (+ decoupled weight decay = AdamW)
  OPT_ADAGRAD = 2,   // a += g^2 ; p -= lr*g/(sqrt(a) + eps)   (TF1: eps = 0)
  OPT_ADADELTA = 3,  // TF1 Adadelta
  OPT_FTRL = 4,      // TF1 FTRL-proximal (lr_power = -0.5)
  OPT_RMSPROP = 5,   // TF1 RMSProp: ms = rho*ms + (1-rho) g^2; mom = m*mom + lr*g/sqrt(ms+eps); p -= mom
  OPT_LAMB = 6,      // (per-arena trust ratio not fused; treated as AdamW here)
};

struct OptArgs {
  float* p;
  float* g;
  float* s1;
  float* s2;
  bf16_t* p16;
  long n;
  int kind;
  float b1, b2, eps, wd, mom, l1, l2;
  int nesterov, zero_grad;
  const float* hp;
  const float* sumsq;
  const int* abort;  // per-stream hipGraph replay: nonzero after a timed-out cross-stream wait -> apply nothing
};

template <int KIND>
__device__ __forceinline__ void upd1(const OptArgs& a, float lr, float gs, float& p, float g, float& s1,
                                     float& s2) {
  g *= gs;
  if constexpr (KIND == OPT_SGD) {
    if (a.wd != 0.f) g += a.wd * p;
    if (a.mom != 0.f) {
      s1 = a.mom * s1 + g;
      p -= lr * (a.nesterov ? g + a.mom * s1 : s1);
    } else {
      p -= lr * g;
    }
  } else if constexpr (KIND == OPT_ADAM || KIND == OPT_LAMB) {
    s1 = a.b1 * s1 + (1.f - a.b1) * g;
    s2 = a.b2 * s2 + (1.f - a.b2) * g * g;
    p -= lr * (s1 / (sqrtf(s2) + a.eps) + a.wd * p);
  } else if constexpr (KIND == OPT_ADAGRAD) {
    s1 += g * g;
    p -= lr * g / (sqrtf(s1) + a.eps);
  } else if constexpr (KIND == OPT_ADADELTA) {
    s1 = a.b1 * s1 + (1.f - a.b1) * g * g;                 // accum
    float d = sqrtf(s2 + a.eps) / sqrtf(s1 + a.eps) * g;  // update
    s2 = a.b1 * s2 + (1.f - a.b1) * d * d;                 // accum_update
    p -= lr * d;
  } else if constexpr (KIND == OPT_FTRL) {
    // s1 = accumulator n, s2 = linear z
    float n_new = s1 + g * g;
    float sigma = (sqrtf(n_new) - sqrtf(s1)) / lr;
    s2 += g - sigma * p;
    s1 = n_new;
    float quad = sqrtf(n_new) / lr + 2.f * a.l2;
    p = fabsf(s2) > a.l1 ? (copysignf(a.l1, s2) - s2) / quad : 0.f;
  } else {  // OPT_RMSPROP
    s1 = a.b1 * s1 + (1.f - a.b1) * g * g;
    s2 = a.mom * s2 + lr * g / sqrtf(s1 + a.eps);
    p -= s2;
  }
}

// streaming loads/stores: every byte of the arenas is touched exactly once per step, so keep them out of the
// L2/MALL working set of the kernels around the update
typedef float nt4f __attribute__((ext_vector_type(4)));
typedef unsigned int nt2u __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float4 ld_nt(const float* p, long i) {
  const nt4f v = __builtin_nontemporal_load(reinterpret_cast<const nt4f*>(p) + i);
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_nt(float* p, long i, float4 v) {
  __builtin_nontemporal_store((nt4f){v.x, v.y, v.z, v.w}, reinterpret_cast<nt4f*>(p) + i);
}

// U float4 groups per thread per trip, all loads issued before any math (4-5 streams x U x 16 B in flight per
// lane); the kernel kind and the slot count are template parameters so the loop body is branch-free
template <int KIND, int NS>
__global__ void __launch_bounds__(256) optim_kernel(OptArgs a) {
  constexpr int U = 2;
  // a join of this step timed out (graph_sync.hip xs_wait): its gradients may be incomplete, so the weights must not
  // move; the host raises at its next check (graphs.CapturedStep)
  if (a.abort && __hip_atomic_load(a.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const float lr = a.hp[0];
  float gs = a.hp[1];
  if (a.sumsq && a.hp[2] > 0.f) {
    float nrm = sqrtf(*a.sumsq) * gs;
    if (nrm > a.hp[2]) gs *= a.hp[2] / nrm;
  }
  const long n4 = a.n / 4;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x; i0 < n4; i0 += U * stride) {
    float4 p[U], g[U], s1[U], s2[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * stride;
      if (i < n4) {
        p[u] = ld_nt(a.p, i);
        g[u] = ld_nt(a.g, i);
        s1[u] = NS > 0 ? ld_nt(a.s1, i) : make_float4(0, 0, 0, 0);
        s2[u] = NS > 1 ? ld_nt(a.s2, i) : make_float4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * stride;
      if (i >= n4) break;
      upd1<KIND>(a, lr, gs, p[u].x, g[u].x, s1[u].x, s2[u].x);
      upd1<KIND>(a, lr, gs, p[u].y, g[u].y, s1[u].y, s2[u].y);
      upd1<KIND>(a, lr, gs, p[u].z, g[u].z, s1[u].z, s2[u].z);
      upd1<KIND>(a, lr, gs, p[u].w, g[u].w, s1[u].w, s2[u].w);
      st_nt(a.p, i, p[u]);
      if (NS > 0) st_nt(a.s1, i, s1[u]);
      if (NS > 1) st_nt(a.s2, i, s2[u]);
      if (a.zero_grad) st_nt(a.g, i, make_float4(0, 0, 0, 0));
      if (a.p16) {
        __builtin_nontemporal_store((nt2u){pack2bf(p[u].x, p[u].y), pack2bf(p[u].z, p[u].w)},
                                    reinterpret_cast<nt2u*>(a.p16) + i);
      }
    }
  }
  // tail
  if (blockIdx.x == 0 && threadIdx.x < (a.n & 3)) {
    long i = n4 * 4 + threadIdx.x;
    float p = a.p[i], g = a.g[i], s1 = NS > 0 ? a.s1[i] : 0.f, s2 = NS > 1 ? a.s2[i] : 0.f;
    upd1<KIND>(a, lr, gs, p, g, s1, s2);
    a.p[i] = p;
    if (NS > 0) a.s1[i] = s1;
    if (NS > 1) a.s2[i] = s2;
    if (a.zero_grad) a.g[i] = 0.f;
    if (a.p16) a.p16[i] = f2bf(p);
  }
}

template <int KIND>
void launch_optim(const OptArgs& a, hipStream_t st) {
  const dim3 grid(stream_grid(a.n / 8 + 1, 256)), block(256);
  if (a.s2) hipLaunchKernelGGL((optim_kernel<KIND, 2>), grid, block, 0, st, a);
  else if (a.s1) hipLaunchKernelGGL((optim_kernel<KIND, 1>), grid, block, 0, st, a);
  else hipLaunchKernelGGL((optim_kernel<KIND, 0>), grid, block, 0, st, a);
}

__global__ void __launch_bounds__(256) sumsq_kernel(const float* __restrict__ x, long n, float* __restrict__ out) {
  __shared__ float red[16];
  float s = 0.f;
  const long n4 = n / 4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 v = reinterpret_cast<const float4*>(x)[i];
    s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    float v = x[n4 * 4 + threadIdx.x];
    s += v * v;
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) atomicAdd(out, s);
}

// hipGraph replays: hp = table[ctr % R], then ctr += 1. The host fills slot k % R of the (pinned) table before
// replay k and reuses a slot only after the replay that read it has finished, so consecutive replays need no
// host synchronisation (graphs.CapturedStep; the captured table copy reads the pinned ring at replay time).
__global__ void hp_ring_select_kernel(const float* __restrict__ table, int R, int n, int* ctr,
                                      float* __restrict__ hp) {
  const int k = *ctr;
  if ((int)threadIdx.x < n) hp[threadIdx.x] = table[(k % R) * n + threadIdx.x];
  __syncthreads();
  if (threadIdx.x == 0) *ctr = k + 1;
}

}  // namespace

DTF_API int dtf_hp_ring_select(const float* table, int R, int n, int* ctr, float* hp, void* stream) {
  if (R < 1 || n < 1 || n > 64) return -1;
  hipLaunchKernelGGL(hp_ring_select_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, table, R, n, ctr, hp);
  return (int)hipGetLastError();
}

DTF_API int dtf_optim_apply(int kind, float* p, float* g, float* s1, float* s2, void* p16, long n, float b1,
                            float b2, float eps, float wd, float mom, float l1, float l2, int nesterov,
                            int zero_grad, const float* hp, const float* sumsq, const int* abort, void* stream) {
  if (n <= 0) return 0;
  OptArgs a;
  a.p = p; a.g = g; a.s1 = s1; a.s2 = s2; a.p16 = (bf16_t*)p16; a.n = n; a.kind = kind;
  a.b1 = b1; a.b2 = b2; a.eps = eps; a.wd = wd; a.mom = mom; a.l1 = l1; a.l2 = l2;
  a.nesterov = nesterov; a.zero_grad = zero_grad; a.hp = hp; a.sumsq = sumsq; a.abort = abort;
  hipStream_t st = (hipStream_t)stream;
  switch (kind) {
    case OPT_SGD: launch_optim<OPT_SGD>(a, st); break;
    case OPT_ADAM: case OPT_LAMB: launch_optim<OPT_ADAM>(a, st); break;
    case OPT_ADAGRAD: launch_optim<OPT_ADAGRAD>(a, st); break;
    case OPT_ADADELTA: launch_optim<OPT_ADADELTA>(a, st); break;
    case OPT_FTRL: launch_optim<OPT_FTRL>(a, st); break;
    case OPT_RMSPROP: launch_optim<OPT_RMSPROP>(a, st); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

DTF_API int dtf_sumsq(const float* x, long n, float* out, int zero, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (zero) (void)hipMemsetAsync(out, 0, sizeof(float), st);
  int grid = stream_grid(n / 4 + 1, 256);
  if (grid > 1024) grid = 1024;
  hipLaunchKernelGGL(sumsq_kernel, dim3(grid), dim3(256), 0, st, x, n, out);
  return (int)hipGetLastError();
}
