// Linear BatchNorm backward of a 1x1 convolution (ops.conv _lbb): the small per-channel / per-filter finalize between
// the two concatenated-operand GEMMs of gemm.hip (dtf_conv1x1_wgrad_cat, dtf_conv1x1_dgrad_cat).
//
// Forward: yc = X W^T (X [M][C] bf16, W [K][C] bf16), BN over the K channels of yc with batch mean mu and invstd is,
// z = gamma * (yc - mu) * is + beta, then (+ residual, ReLU: the caller's mask pass turns the incoming gradient into
// dz). The usual backward dyc = a*dz + b*yc + c (bn_bwd_finalize_kernel's coefficients) is LINEAR in yc = X W^T, so
// with P = dz^T X [K][C], G = X^T X [C][C] and s = 1^T X [C] (one GEMM over [dz | X]):
//   sum dz * yc  = rowdot(W, P)                          (the BN reduction, no read of yc)
//   dW           = diag(a) P + diag(b) W G + c s^T        (lbb_dw_kernel)
//   dX           = [dz | X] . Bd^T + bias,  Bd = [ (diag(a) W)^T | W^T diag(b) W ],  bias = W^T c   (lbb_bmat_kernel)
// Neither yc nor dyc is ever written or read: the BN backward apply pass and the conv output's storage disappear.
// (SURVEY §2.4.b K4/K5, §7.4 hard part 1; the reference's hot loop: trainer/task.py:232-236.)
#include "common.h"

namespace {

// One wave per output channel k: sdz = rsum[k] (sum dz, from the GEMM's row sums), sdzy = rowdot(W[k], P[k]) (fixed
// lane order and shuffle tree: deterministic); the BN-backward coefficients and dgamma / dbeta (accumulated into the
// gradients when accumulate).
__global__ void __launch_bounds__(256) lbb_coef_kernel(const float* __restrict__ rsum, const bf16_t* __restrict__ W,
                                                       const float* __restrict__ P, const float* __restrict__ gamma,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ invstd, long M, int K, int C,
                                                       float* dgamma, float* dbeta, int accumulate,
                                                       float* __restrict__ coef) {
  const int lane = threadIdx.x & 63;
  const int k = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (k >= K) return;
  float d = 0.f;
  for (int c = lane; c < C; c += 64) d = fmaf(bf2f(W[(long)k * C + c]), P[(long)k * C + c], d);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
  if (lane != 0) return;
  const float sdz = rsum[k];
  const float is = invstd[k], mu = mean[k];
  const float sdzx = d - mu * sdz;  // sum dz * (yc - mu)
  const float sdx = sdzx * is;      // sum dz * xhat
  if (dgamma) dgamma[k] = (accumulate ? dgamma[k] : 0.f) + sdx;
  if (dbeta) dbeta[k] = (accumulate ? dbeta[k] : 0.f) + sdz;
  const float gm = gamma ? gamma[k] : 1.f;
  const float k1 = gm * is, k2 = sdz / (float)M, k3 = sdx / (float)M;
  coef[k] = k1;
  coef[K + k] = -k1 * k3 * is;
  coef[2 * K + k] = k1 * (mu * is * k3 - k2);
}

// dW[k][c] (+)= a_k P[k][c] + b_k sum_c' W[k][c'] G[c'][c] + c_k s[c]: 32 x 64 (k, c) tile per block, c' in chunks of
// 32 staged through LDS; thread (ty, tx) owns rows 2 ty, 2 ty + 1 and columns 4 tx .. 4 tx + 3.
__global__ void __launch_bounds__(256) lbb_dw_kernel(const float* __restrict__ P, const float* __restrict__ G,
                                                     const float* __restrict__ s, const bf16_t* __restrict__ W,
                                                     const float* __restrict__ coef, int K, int C,
                                                     float* __restrict__ dW, int accumulate) {
  __shared__ float wt[32][33];
  __shared__ float gt[32][64];
  const int k0 = blockIdx.y * 32, c0 = blockIdx.x * 64;
  const int t = threadIdx.x, ty = t >> 4, tx = t & 15;
  float acc[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  for (int cp = 0; cp < C; cp += 32) {
    for (int i = t; i < 32 * 32; i += 256) {
      const int r = i >> 5, q = i & 31;
      wt[r][q] = (k0 + r < K && cp + q < C) ? bf2f(W[(long)(k0 + r) * C + cp + q]) : 0.f;
    }
    for (int i = t; i < 32 * 64; i += 256) {
      const int r = i >> 6, q = i & 63;
      gt[r][q] = (cp + r < C && c0 + q < C) ? G[(long)(cp + r) * C + c0 + q] : 0.f;
    }
    __syncthreads();
#pragma unroll 8
    for (int q = 0; q < 32; ++q) {
      const float w0 = wt[2 * ty][q], w1 = wt[2 * ty + 1][q];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float gv = gt[q][4 * tx + j];
        acc[0][j] = fmaf(w0, gv, acc[0][j]);
        acc[1][j] = fmaf(w1, gv, acc[1][j]);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int k = k0 + 2 * ty + i;
    if (k >= K) continue;
    const float ca = coef[k], cb = coef[K + k], cc = coef[2 * K + k];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = c0 + 4 * tx + j;
      if (c >= C) continue;
      const long e = (long)k * C + c;
      const float v = fmaf(ca, P[e], fmaf(cb, acc[i][j], cc * s[c]));
      dW[e] = accumulate ? dW[e] + v : v;
    }
  }
}

// The data-gradient GEMM's B operand Bd [C][K + C] (bf16) and bias [C]:
//   part 0: Bd[c][k] = a_k W[k][c] (a 32 x 32 transpose through LDS per block, grid (K/32, C/32));
//   part 1: Bd[c][K + c'] = sum_k b_k W[k][c'] W[k][c], a 32 x 32 (c', c) tile per block (grid (C/32, C/32)),
//                    k in chunks of 32 through LDS; the blocks with c' tile 0 also write bias[c] = sum_k c_k W[k][c].
__global__ void __launch_bounds__(256) lbb_bmat_kernel(const bf16_t* __restrict__ W, const float* __restrict__ coef,
                                                       int K, int C, bf16_t* __restrict__ Bd,
                                                       float* __restrict__ bias, int part) {
  __shared__ float ta[32][33];
  __shared__ float tb[32][33];
  const int t = threadIdx.x;
  const long ldb = (long)K + C;
  if (part == 0) {
    const int kb = blockIdx.x * 32, cb = blockIdx.y * 32;
    if (kb >= K || cb >= C) return;
    for (int i = t; i < 32 * 32; i += 256) {
      const int r = i >> 5, q = i & 31;  // r: k, q: c
      ta[r][q] = (kb + r < K && cb + q < C) ? coef[kb + r] * bf2f(W[(long)(kb + r) * C + cb + q]) : 0.f;
    }
    __syncthreads();
    for (int i = t; i < 32 * 32; i += 256) {
      const int r = i >> 5, q = i & 31;  // r: c, q: k
      if (cb + r < C && kb + q < K) Bd[(long)(cb + r) * ldb + kb + q] = f2bf(ta[q][r]);
    }
    return;
  }
  const int pb = blockIdx.x * 32, cb = blockIdx.y * 32;  // c' tile, c tile
  if (pb >= C || cb >= C) return;
  const int ty = t >> 3, tx = t & 7;  // thread: c' row pb + ty, c columns cb + 4 tx .. + 3
  float acc[4] = {0.f, 0.f, 0.f, 0.f}, bsum[4] = {0.f, 0.f, 0.f, 0.f};
  for (int kc = 0; kc < K; kc += 32) {
    for (int i = t; i < 32 * 32; i += 256) {
      const int r = i >> 5, q = i & 31;  // r: k in chunk, q: column
      const bool kv = kc + r < K;
      const float bk = kv ? coef[K + kc + r] : 0.f;
      ta[r][q] = (kv && pb + q < C) ? bk * bf2f(W[(long)(kc + r) * C + pb + q]) : 0.f;
      tb[r][q] = (kv && cb + q < C) ? bf2f(W[(long)(kc + r) * C + cb + q]) : 0.f;
    }
    __syncthreads();
#pragma unroll 8
    for (int r = 0; r < 32; ++r) {
      const float av = ta[r][ty];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = fmaf(av, tb[r][4 * tx + j], acc[j]);
    }
    if (blockIdx.x == 0 && ty == 0) {  // bias over this k chunk (fixed order)
      for (int r = 0; r < 32; ++r) {
        const float ck = kc + r < K ? coef[2 * K + kc + r] : 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) bsum[j] = fmaf(ck, tb[r][4 * tx + j], bsum[j]);
      }
    }
    __syncthreads();
  }
  const int p = pb + ty;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = cb + 4 * tx + j;
    if (p < C && c < C) Bd[(long)c * ldb + K + p] = f2bf(acc[j]);
    if (blockIdx.x == 0 && ty == 0 && c < C) bias[c] = bsum[j];
  }
}

}  // namespace

// After dtf_conv1x1_wgrad_cat: P2 = [P ; G] ([K + C][C] f32), rsum = [sum dz ; s] ([K + C]). Writes the BN-backward
// coefficients (coef, 3K floats), dgamma / dbeta (accumulated when accumulate_bn), dW (K x C f32, accumulated when
// accumulate), the data-gradient operand Bd ([C][K + C] bf16) and bias ([C] f32). W: the bf16 filter the forward used.
DTF_API int dtf_lbb_finalize(const float* P2, const float* rsum, const void* W, const float* gamma, const float* mean,
                             const float* invstd, long M, int K, int C, float* dgamma, float* dbeta, int accumulate_bn,
                             float* dW, int accumulate, float* coef, void* Bd, float* bias, void* stream) {
  if ((K & 31) || (C & 31) || !coef || !dW || !Bd || !bias) return -1;
  hipStream_t st = (hipStream_t)stream;
  const float* P = P2;
  const float* G = P2 + (long)K * C;
  const float* s = rsum + K;
  hipLaunchKernelGGL(lbb_coef_kernel, dim3((K + 3) / 4), dim3(256), 0, st, rsum, (const bf16_t*)W, P, gamma, mean,
                     invstd, M, K, C, dgamma, dbeta, accumulate_bn, coef);
  hipLaunchKernelGGL(lbb_dw_kernel, dim3((C + 63) / 64, (K + 31) / 32), dim3(256), 0, st, P, G, s, (const bf16_t*)W,
                     (const float*)coef, K, C, dW, accumulate);
  hipLaunchKernelGGL(lbb_bmat_kernel, dim3((K + 31) / 32, (C + 31) / 32), dim3(256), 0, st, (const bf16_t*)W,
                     (const float*)coef, K, C, (bf16_t*)Bd, bias, 0);
  hipLaunchKernelGGL(lbb_bmat_kernel, dim3((C + 31) / 32, (C + 31) / 32), dim3(256), 0, st, (const bf16_t*)W,
                     (const float*)coef, K, C, (bf16_t*)Bd, bias, 1);
  return (int)hipGetLastError();
}
