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
};

__device__ __forceinline__ void upd1(const OptArgs& a, float lr, float gs, float& p, float g, float& s1,
                                     float& s2) {
  g *= gs;
  switch (a.kind) {
    case OPT_SGD:
      if (a.wd != 0.f) g += a.wd * p;
      if (a.mom != 0.f) {
        s1 = a.mom * s1 + g;
        p -= lr * (a.nesterov ? g + a.mom * s1 : s1);
      } else {
        p -= lr * g;
      }
      break;
    case OPT_ADAM:
    case OPT_LAMB:
      s1 = a.b1 * s1 + (1.f - a.b1) * g;
      s2 = a.b2 * s2 + (1.f - a.b2) * g * g;
      p -= lr * (s1 / (sqrtf(s2) + a.eps) + a.wd * p);
      break;
    case OPT_ADAGRAD:
      s1 += g * g;
      p -= lr * g / (sqrtf(s1) + a.eps);
      break;
    case OPT_ADADELTA: {
      s1 = a.b1 * s1 + (1.f - a.b1) * g * g;                 // accum
      float d = sqrtf(s2 + a.eps) / sqrtf(s1 + a.eps) * g;  // update
      s2 = a.b1 * s2 + (1.f - a.b1) * d * d;                 // accum_update
      p -= lr * d;
      break;
    }
    case OPT_FTRL: {
      // s1 = accumulator n, s2 = linear z
      float n_new = s1 + g * g;
      float sigma = (sqrtf(n_new) - sqrtf(s1)) / lr;
      s2 += g - sigma * p;
      s1 = n_new;
      float quad = sqrtf(n_new) / lr + 2.f * a.l2;
      p = fabsf(s2) > a.l1 ? (copysignf(a.l1, s2) - s2) / quad : 0.f;
      break;
    }
    case OPT_RMSPROP:
      s1 = a.b1 * s1 + (1.f - a.b1) * g * g;
      s2 = a.mom * s2 + lr * g / sqrtf(s1 + a.eps);
      p -= s2;
      break;
  }
}

__global__ void __launch_bounds__(256) optim_kernel(OptArgs a) {
  const float lr = a.hp[0];
  float gs = a.hp[1];
  if (a.sumsq && a.hp[2] > 0.f) {
    float nrm = sqrtf(*a.sumsq) * gs;
    if (nrm > a.hp[2]) gs *= a.hp[2] / nrm;
  }
  const long n4 = a.n / 4;
  const bool has1 = a.s1 != nullptr, has2 = a.s2 != nullptr;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 p = reinterpret_cast<float4*>(a.p)[i];
    float4 g = reinterpret_cast<float4*>(a.g)[i];
    float4 s1 = has1 ? reinterpret_cast<float4*>(a.s1)[i] : make_float4(0, 0, 0, 0);
    float4 s2 = has2 ? reinterpret_cast<float4*>(a.s2)[i] : make_float4(0, 0, 0, 0);
    upd1(a, lr, gs, p.x, g.x, s1.x, s2.x);
    upd1(a, lr, gs, p.y, g.y, s1.y, s2.y);
    upd1(a, lr, gs, p.z, g.z, s1.z, s2.z);
    upd1(a, lr, gs, p.w, g.w, s1.w, s2.w);
    reinterpret_cast<float4*>(a.p)[i] = p;
    if (has1) reinterpret_cast<float4*>(a.s1)[i] = s1;
    if (has2) reinterpret_cast<float4*>(a.s2)[i] = s2;
    if (a.zero_grad) reinterpret_cast<float4*>(a.g)[i] = make_float4(0, 0, 0, 0);
    if (a.p16) {
      uint2 o;
      o.x = pack2bf(p.x, p.y);
      o.y = pack2bf(p.z, p.w);
      reinterpret_cast<uint2*>(a.p16)[i] = o;
    }
  }
  // tail
  if (blockIdx.x == 0 && threadIdx.x < (a.n & 3)) {
    long i = n4 * 4 + threadIdx.x;
    float p = a.p[i], g = a.g[i], s1 = has1 ? a.s1[i] : 0.f, s2 = has2 ? a.s2[i] : 0.f;
    upd1(a, lr, gs, p, g, s1, s2);
    a.p[i] = p;
    if (has1) a.s1[i] = s1;
    if (has2) a.s2[i] = s2;
    if (a.zero_grad) a.g[i] = 0.f;
    if (a.p16) a.p16[i] = f2bf(p);
  }
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
                            int zero_grad, const float* hp, const float* sumsq, void* stream) {
  if (n <= 0) return 0;
  OptArgs a;
  a.p = p; a.g = g; a.s1 = s1; a.s2 = s2; a.p16 = (bf16_t*)p16; a.n = n; a.kind = kind;
  a.b1 = b1; a.b2 = b2; a.eps = eps; a.wd = wd; a.mom = mom; a.l1 = l1; a.l2 = l2;
  a.nesterov = nesterov; a.zero_grad = zero_grad; a.hp = hp; a.sumsq = sumsq;
  hipLaunchKernelGGL(optim_kernel, dim3(stream_grid(n / 4 + 1, 256)), dim3(256), 0, (hipStream_t)stream, a);
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
