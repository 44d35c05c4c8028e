// FusedBatchNorm (NHWC, training + inference) and LayerNorm for gfx950.
//
// TF's FusedBatchNormV3 / FusedBatchNormGradV3 and LayerNorm equivalents
// (SURVEY §2.4.b K5/K6). Layout is channels-last [M = N*H*W][C], bf16 I/O,
// f32 statistics. The forward statistics are normally produced for free by the
// conv epilogue (gemm.hip `stats`), so the standalone path here is:
//   bn_stats (only when no conv produced them) -> bn_finalize (per channel,
//   also updates running stats TF-style) -> bn_apply (scale/shift [+res] [+relu]).
// Backward: bn_bwd_reduce (sum dz, sum dz*xhat with the ReLU mask applied
//   on the fly) -> bn_bwd_finalize -> bn_bwd_apply (dx, optional dz for the
//   residual branch). All passes are 16-B vectorized and grid-stride; reductions
//   write one partial row per block (no same-address atomics: deterministic).
#include "common.h"
#include "dropout_mask.h"
#include <algorithm>
#include <cmath>
#include <cstdlib>

namespace {

// Column-reduction geometry: TPR threads per row (8 channels each), RPB rows per pass.
struct ColGeo {
  int cols8, TPR, RPB;
};
__host__ __device__ inline ColGeo colgeo(int C) {
  ColGeo g;
  g.cols8 = C / 8;
  g.TPR = g.cols8 < 256 ? g.cols8 : 256;
  g.RPB = 256 / g.TPR;
  return g;
}

// Block-level column reduction of per-thread 8-channel partial sums -> one partial row per block.
// s/q: this thread's sums for channels [cc*8, cc*8+8); rows of the block with equal cc are combined in LDS.
__device__ __forceinline__ void block_col_partials(float (&s)[8], float (&q)[8], int cc0, int TPR, int RPB, int C,
                                                   float* __restrict__ part_row, float* red) {
  const int t = threadIdx.x;
  const bool act = t < TPR * RPB;
  __syncthreads();
  if (act) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { red[t * 8 + j] = s[j]; red[2048 + t * 8 + j] = q[j]; }
  }
  __syncthreads();
  for (int o = t; o < TPR * 8; o += blockDim.x) {
    const int c = cc0 * 8 + o;
    if (c >= C) continue;
    float a = 0.f, b = 0.f;
    for (int r = 0; r < RPB; ++r) {
      a += red[(r * TPR + (o >> 3)) * 8 + (o & 7)];
      b += red[2048 + (r * TPR + (o >> 3)) * 8 + (o & 7)];
    }
    part_row[c] = a;
    part_row[C + c] = b;
  }
}

// Standalone BN statistics: partial [gridDim.x][2C] rows (no atomics; summed by bn_finalize).
__global__ void __launch_bounds__(256) bn_stats_kernel(const bf16_t* __restrict__ x, long M, int C,
                                                       float* __restrict__ part) {
  __shared__ float red[4096];
  ColGeo g = colgeo(C);
  const int t = threadIdx.x;
  const int rsub = t / g.TPR;
  for (int cc0 = 0; cc0 < g.cols8; cc0 += g.TPR) {
    const int cc = cc0 + t % g.TPR;
    float s[8] = {0}, q[8] = {0};
    if (t < g.TPR * g.RPB && cc < g.cols8) {
      for (long r = (long)blockIdx.x * g.RPB + rsub; r < M; r += (long)gridDim.x * g.RPB) {
        float f[8];
        load8(x + r * C + cc * 8, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) { s[j] += f[j]; q[j] += f[j] * f[j]; }
      }
    }
    block_col_partials(s, q, cc0, g.TPR, g.RPB, C, part + (long)blockIdx.x * 2 * C, red);
  }
}

// Per-channel: sum T partial rows, mean/var, scale = gamma*invstd, shift = beta - mean*scale.
// Running stats follow Keras BatchNormalization: r = r*momentum + batch*(1-momentum),
// with the unbiased variance, as TF's FusedBatchNormV3 does.
// grid: ceil(C/64) blocks of FIN_NT threads (FIN_G row-groups x 64 channels): up to ~256 partial rows are summed
// here directly (16 rows per thread, 4 loads in flight), so the row-grouping launch only runs for larger T.
constexpr int FIN_G = 16, FIN_NT = 64 * FIN_G;

// this thread's strided share of the T partial rows of channel c (sum half and sum-of-squares / x-weighted half),
// combined over the FIN_G row groups in a fixed order (deterministic)
__device__ __forceinline__ void fin_rows(const float* __restrict__ part, int T, long rs, int C, int c, bool cv,
                                         float (&red)[2][FIN_G][64], float& A, float& B) {
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  float a = 0.f, b = 0.f;
  if (cv) {
#pragma unroll 4
    for (int r = grp; r < T; r += FIN_G) { a += part[(long)r * rs + c]; b += part[(long)r * rs + C + c]; }
  }
  red[0][grp][cl] = a;
  red[1][grp][cl] = b;
  __syncthreads();
  A = B = 0.f;
  if (grp == 0) {
#pragma unroll
    for (int g = 0; g < FIN_G; ++g) { A += red[0][g][cl]; B += red[1][g][cl]; }
  }
}

__global__ void __launch_bounds__(FIN_NT) bn_finalize_kernel(const float* __restrict__ part, int T, long rs,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float* running_mean,
                                                          float* running_var, long M, int C, float momentum,
                                                          float eps, float* __restrict__ scale,
                                                          float* __restrict__ shift, float* __restrict__ mean_out,
                                                          float* __restrict__ invstd_out) {
  __shared__ float red[2][FIN_G][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float a, b;
  fin_rows(part, T, rs, C, c, c < C, red, a, b);
  if (grp != 0 || c >= C) return;
  float mean = a / (float)M;
  float var = fmaxf(b / (float)M - mean * mean, 0.f);
  float inv = rsqrtf(var + eps);
  float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  scale[c] = gm * inv;
  shift[c] = bt - mean * gm * inv;
  if (mean_out) mean_out[c] = mean;
  if (invstd_out) invstd_out[c] = inv;
  if (running_mean) {
    float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
    running_mean[c] = running_mean[c] * momentum + mean * (1.f - momentum);
    running_var[c] = running_var[c] * momentum + unb * (1.f - momentum);
  }
}

__device__ __forceinline__ void bn_finalize_channel(int c, float a, float b, const float* __restrict__ gamma,
                                                    const float* __restrict__ beta, float* running_mean,
                                                    float* running_var, long M, float momentum, float eps,
                                                    float* __restrict__ scale, float* __restrict__ shift,
                                                    float* __restrict__ mean_out, float* __restrict__ invstd_out) {
  float mean = a / (float)M;
  float var = fmaxf(b / (float)M - mean * mean, 0.f);
  float inv = rsqrtf(var + eps);
  float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  scale[c] = gm * inv;
  shift[c] = bt - mean * gm * inv;
  if (mean_out) mean_out[c] = mean;
  if (invstd_out) invstd_out[c] = inv;
  if (running_mean) {
    float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
    running_mean[c] = running_mean[c] * momentum + mean * (1.f - momentum);
    running_var[c] = running_var[c] * momentum + unb * (1.f - momentum);
  }
}

__device__ __forceinline__ void bn_bwd_finalize_channel(int c, int C, float sdz, float sdxm,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ invstd, long M, float* dgamma,
                                                        float* dbeta, int accumulate, float* __restrict__ coef) {
  const float is = invstd[c];
  const float sdx = sdxm * is;
  if (dgamma) dgamma[c] = (accumulate ? dgamma[c] : 0.f) + sdx;
  if (dbeta) dbeta[c] = (accumulate ? dbeta[c] : 0.f) + sdz;
  const float gm = gamma ? gamma[c] : 1.f;
  const float k1 = gm * is, k2 = sdz / (float)M, k3 = sdx / (float)M;
  coef[c] = k1;
  coef[C + c] = -k1 * k3 * is;
  coef[2 * C + c] = k1 * (mean[c] * is * k3 - k2);
}

// Inference: scale/shift from running statistics.
__global__ void bn_infer_coeff_kernel(const float* gamma, const float* beta, const float* rmean,
                                      const float* rvar, int C, float eps, float* scale, float* shift) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float inv = rsqrtf(rvar[c] + eps);
  float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  scale[c] = gm * inv;
  shift[c] = bt - rmean[c] * gm * inv;
}

// Channels-last elementwise passes (apply / backward apply) use the reduction geometry: a thread owns one
// fixed 8-channel chunk, so its per-channel coefficients sit in registers for the whole launch (no per-element
// channel index division or coefficient reloads), and walks rows with a grid stride, EU rows per trip with all
// loads issued before any use (memory-level parallelism for the HBM-bound pass).
constexpr int EU = 4;

__device__ __forceinline__ void load_coef8(const float* __restrict__ p, float* f) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

// y = [relu](x*scale + shift [+ res]); optional 1-bit ReLU mask of the stored (bf16) values
__device__ __forceinline__ void bn_apply_row(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                             bf16_t* __restrict__ y, uint8_t* __restrict__ mbits, long i8,
                                             const float* f, const float* r, const float* sc, const float* sh,
                                             int relu) {
  float o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float v = fmaf(f[j], sc[j], sh[j]);
    if (res) v += r[j];
    if (relu) v = fmaxf(v, 0.f);
    o[j] = v;
  }
  store8(y + i8 * 8, o);
  if (mbits) {
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) bits |= (uint32_t)(f2bf(o[j]) != 0 && o[j] > 0.f) << j;
    mbits[i8] = (uint8_t)bits;
  }
}

// rscale/rshift (optional): the residual is itself a BatchNorm input (a projection shortcut's conv output) whose
// affine normalisation is applied here, so the shortcut's BN output is never materialised.
template <int NU = EU>  // rows per trip (all loads of a trip issued before the first use)
__global__ void __launch_bounds__(256) bn_apply_kernel(const bf16_t* __restrict__ x, const float* __restrict__ scale,
                                                       const float* __restrict__ shift,
                                                       const bf16_t* __restrict__ res, bf16_t* __restrict__ y,
                                                       long M, int C, int relu, uint8_t* __restrict__ mbits,
                                                       const float* __restrict__ rscale,
                                                       const float* __restrict__ rshift, int rev) {
  const ColGeo g = colgeo(C);
  const int t = threadIdx.x;
  if (t >= g.TPR * g.RPB) return;
  const int rsub = t / g.TPR;
  const long rstep = (long)gridDim.x * g.RPB;
  for (int cc = t % g.TPR; cc < g.cols8; cc += g.TPR) {
    float sc[8], sh[8], rsc[8], rsh[8];
    load_coef8(scale + cc * 8, sc);
    load_coef8(shift + cc * 8, sh);
    if (rscale) {
      load_coef8(rscale + cc * 8, rsc);
      load_coef8(rshift + cc * 8, rsh);
    }
    auto raff = [&](float* rv) {
      if (rscale) {
#pragma unroll
        for (int j = 0; j < 8; ++j) rv[j] = fmaf(rv[j], rsc[j], rsh[j]);
      }
    };
    long r = (long)blockIdx.x * g.RPB + rsub;
    for (; r + (NU - 1) * rstep < M; r += NU * rstep) {
      float f[NU][8], rv[NU][8];
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const long i8 = (rev ? M - 1 - (r + u * rstep) : r + u * rstep) * g.cols8 + cc;
        load8(x + i8 * 8, f[u]);
        if (res) load8(res + i8 * 8, rv[u]);
      }
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        if (res) raff(rv[u]);
        bn_apply_row(x, res, y, mbits, (rev ? M - 1 - (r + u * rstep) : r + u * rstep) * g.cols8 + cc, f[u], rv[u],
                     sc, sh, relu);
      }
    }
    for (; r < M; r += rstep) {
      float f[8], rv[8];
      const long i8 = (rev ? M - 1 - r : r) * g.cols8 + cc;
      load8(x + i8 * 8, f);
      if (res) {
        load8(res + i8 * 8, rv);
        raff(rv);
      }
      bn_apply_row(x, res, y, mbits, i8, f, rv, sc, sh, relu);
    }
  }
}

// dz = dy masked by ReLU: from the 1-bit mask or the bf16 output (sign/zero test)
__device__ __forceinline__ void relu_mask8(float* d, const bf16_t* ymask, const uint8_t* mbits, long i8) {
  if (mbits) {
    const uint32_t b = mbits[i8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (!((b >> j) & 1u)) d[j] = 0.f;
  } else if (ymask) {
    uint4 mv = *reinterpret_cast<const uint4*>(ymask + i8 * 8);
    uint32_t w[4] = {mv.x, mv.y, mv.z, mv.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // bf16 > 0  <=>  sign bit clear and value bits non-zero
      uint32_t lo = w[j] & 0xffffu, hi = w[j] >> 16;
      if (!(lo != 0 && !(lo & 0x8000u))) d[2 * j] = 0.f;
      if (!(hi != 0 && !(hi & 0x8000u))) d[2 * j + 1] = 0.f;
    }
  }
}

// Backward reduce: dz = dy * (y > 0 if relu-mask given); partial rows [gridDim.x][2C]:
// [0,C) sum dz, [C,2C) sum dz*xhat. No atomics; bn_bwd_finalize sums the rows.
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(const bf16_t* __restrict__ dy,
                                                            const bf16_t* __restrict__ ymask,
                                                            const uint8_t* __restrict__ mbits,
                                                            const bf16_t* __restrict__ x,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ invstd, long M, int C,
                                                            float* __restrict__ part) {
  __shared__ float red[4096];
  ColGeo g = colgeo(C);
  const int t = threadIdx.x;
  const int rsub = t / g.TPR;
  for (int cc0 = 0; cc0 < g.cols8; cc0 += g.TPR) {
    const int cc = cc0 + t % g.TPR;
    float s[8] = {0}, q[8] = {0};
    if (t < g.TPR * g.RPB && cc < g.cols8) {
      float mu[8];
      load_coef8(mean + cc * 8, mu);
      // sum dz*(x - mean) here; the invstd factor is applied once per channel in bn_bwd_finalize
      const long rstep = (long)gridDim.x * g.RPB;
      long r = (long)blockIdx.x * g.RPB + rsub;
      for (; r + (EU - 1) * rstep < M; r += EU * rstep) {
        float d[EU][8], xv[EU][8];
#pragma unroll
        for (int u = 0; u < EU; ++u) {
          const long i8 = (r + u * rstep) * g.cols8 + cc;
          load8(dy + i8 * 8, d[u]);
          load8(x + i8 * 8, xv[u]);
          relu_mask8(d[u], ymask, mbits, i8);
        }
#pragma unroll
        for (int u = 0; u < EU; ++u)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            s[j] += d[u][j];
            q[j] = fmaf(d[u][j], xv[u][j] - mu[j], q[j]);
          }
      }
      for (; r < M; r += rstep) {
        float d[8], xv[8];
        const long i8 = r * g.cols8 + cc;
        load8(dy + i8 * 8, d);
        load8(x + i8 * 8, xv);
        relu_mask8(d, ymask, mbits, i8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s[j] += d[j];
          q[j] = fmaf(d[j], xv[j] - mu[j], q[j]);
        }
      }
    }
    block_col_partials(s, q, cc0, g.TPR, g.RPB, C, part + (long)blockIdx.x * 2 * C, red);
  }
}

// Sum T partial rows; dgamma = sum dz*xhat, dbeta = sum dz; coefficients for the apply pass:
//   dx = k1 * (dz - k2 - xhat * k3)   with k1 = gamma*invstd, k2 = sum_dz/M, k3 = sum_dzxhat/M
// folded into dx = a*dz + b*x + c (a = k1, b = -k1*k3*invstd, c = k1*(mean*invstd*k3 - k2)).
__global__ void __launch_bounds__(FIN_NT) bn_bwd_finalize_kernel(const float* __restrict__ part, int T, long rs,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ invstd, long M, int C,
                                                              float* dgamma, float* dbeta, int accumulate,
                                                              float* __restrict__ coef) {
  __shared__ float red[2][FIN_G][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float sa, sb;
  fin_rows(part, T, rs, C, c, c < C, red, sa, sb);
  if (grp != 0 || c >= C) return;
  const float sdz = sa;
  const float is = invstd[c];
  const float sdx = sb * is;
  if (dgamma) dgamma[c] = (accumulate ? dgamma[c] : 0.f) + sdx;
  if (dbeta) dbeta[c] = (accumulate ? dbeta[c] : 0.f) + sdz;
  const float gm = gamma ? gamma[c] : 1.f;
  const float k1 = gm * is, k2 = sdz / (float)M, k3 = sdx / (float)M;
  coef[c] = k1;
  coef[C + c] = -k1 * k3 * is;
  coef[2 * C + c] = k1 * (mean[c] * is * k3 - k2);
}

__device__ __forceinline__ void bn_bwd_apply_row(const float* d, const float* xv, const float* ka, const float* kb,
                                                 const float* kc, bf16_t* __restrict__ dx, bf16_t* __restrict__ dz_out,
                                                 long i8) {
  if (dz_out) store8(dz_out + i8 * 8, d);
  float o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = fmaf(ka[j], d[j], fmaf(kb[j], xv[j], kc[j]));
  store8(dx + i8 * 8, o);
}

// dx = a*dz + b*x + c per channel (coefficients from bn_bwd_finalize); dz_out: the masked dz for the
// residual branch (only when a ReLU mask is given)
// SC: the masked dz (dz_out, the residual gradient) also feeds a projection shortcut's BatchNorm whose input is
// x2 (mean2): its backward reduction (sum dz, sum dz*(x2 - mean2), over the bf16-rounded dz that is stored) is
// taken here as one partial row per block into part2 — the shortcut's own reduce pass disappears.
// (host: C/8 <= 256 and 256 % (C/8) == 0, so every thread owns exactly one channel chunk)
// 16-B streaming load/store with the nontemporal hint (the pass reads and writes each byte once)
__device__ __forceinline__ void load8s(const bf16_t* p, float* f, bool nt) {
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  const u4 v = nt ? __builtin_nontemporal_load(reinterpret_cast<const u4*>(p)) : *reinterpret_cast<const u4*>(p);
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}
__device__ __forceinline__ void store8s(bf16_t* p, const float* f, bool nt) {
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  const u4 v = {pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]), pack2bf(f[6], f[7])};
  if (nt) __builtin_nontemporal_store(v, reinterpret_cast<u4*>(p));
  else *reinterpret_cast<u4*>(p) = v;
}

// dx = a*dz + b*x + c per channel (coefficients from bn_bwd_finalize); dz_out: the masked dz for the
// residual branch (only when a ReLU mask is given)
// SC: the masked dz (dz_out, the residual gradient) also feeds a projection shortcut's BatchNorm whose input is
// x2 (mean2): its backward reduction (sum dz, sum dz*(x2 - mean2), over the bf16-rounded dz that is stored) is
// taken here as one partial row per block into part2 — the shortcut's own reduce pass disappears.
// (host: C/8 <= 256 and 256 % (C/8) == 0, so every thread owns exactly one channel chunk)
// NU rows per trip, all of their loads (dy, x, mask bytes) issued before the first use; NT: nontemporal hints.
template <bool SC, int NU = EU, bool NT = false>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(const bf16_t* __restrict__ dy,
                                                           const bf16_t* __restrict__ ymask,
                                                           const uint8_t* __restrict__ mbits,
                                                           const bf16_t* __restrict__ x,
                                                           const float* __restrict__ coef, long M, int C,
                                                           bf16_t* __restrict__ dx, bf16_t* __restrict__ dz_out,
                                                           const bf16_t* __restrict__ x2,
                                                           const float* __restrict__ mean2,
                                                           float* __restrict__ part2, int rev) {
  const ColGeo g = colgeo(C);
  const int t = threadIdx.x;
  if (!SC && t >= g.TPR * g.RPB) return;
  const int rsub = t / g.TPR;
  const long rstep = (long)gridDim.x * g.RPB;
  if (!ymask && !mbits) dz_out = nullptr;
  float s2[8] = {0}, q2[8] = {0}, mu2[8];
  auto sc_acc = [&](const float* d, long i8) {
    if constexpr (SC) {
      float x2v[8];
      load8(x2 + i8 * 8, x2v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float dz = bf2f(f2bf(d[j]));
        s2[j] += dz;
        q2[j] = fmaf(dz, x2v[j] - mu2[j], q2[j]);
      }
    }
  };
  auto row_out = [&](const float* d, const float* xv, const float* ka, const float* kb, const float* kc, long i8) {
    if (dz_out) store8s(dz_out + i8 * 8, d, NT);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = fmaf(ka[j], d[j], fmaf(kb[j], xv[j], kc[j]));
    store8s(dx + i8 * 8, o, NT);
  };
  for (int cc = t % g.TPR; cc < g.cols8; cc += g.TPR) {
    float ka[8], kb[8], kc[8];
    load_coef8(coef + cc * 8, ka);
    load_coef8(coef + C + cc * 8, kb);
    load_coef8(coef + 2 * C + cc * 8, kc);
    if constexpr (SC) load_coef8(mean2 + cc * 8, mu2);
    long r = (long)blockIdx.x * g.RPB + rsub;
    for (; r + (NU - 1) * rstep < M; r += NU * rstep) {
      float d[NU][8], xv[NU][8];
      uint32_t mb[NU];
      long i8[NU];
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        i8[u] = (rev ? M - 1 - (r + u * rstep) : r + u * rstep) * g.cols8 + cc;
        load8s(dy + i8[u] * 8, d[u], NT);
        load8s(x + i8[u] * 8, xv[u], NT);
        if (mbits) mb[u] = mbits[i8[u]];
      }
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        if (mbits) {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (!((mb[u] >> j) & 1u)) d[u][j] = 0.f;
        } else {
          relu_mask8(d[u], ymask, nullptr, i8[u]);
        }
        row_out(d[u], xv[u], ka, kb, kc, i8[u]);
        sc_acc(d[u], i8[u]);
      }
    }
    for (; r < M; r += rstep) {
      float d[8], xv[8];
      const long i8 = (rev ? M - 1 - r : r) * g.cols8 + cc;
      load8(dy + i8 * 8, d);
      load8(x + i8 * 8, xv);
      relu_mask8(d, ymask, mbits, i8);
      row_out(d, xv, ka, kb, kc, i8);
      sc_acc(d, i8);
    }
  }
  if constexpr (SC) {
    __shared__ float red[4096];
    block_col_partials(s2, q2, 0, g.TPR, g.RPB, C, part2 + (long)blockIdx.x * 2 * C, red);
  }
}

// ---------------- BatchNorm + ReLU + MaxPool (the ResNet stem) ----------------
// Forward: one pass over the conv output yc produces the pooled BN+ReLU output and a 1-byte argmax per
// (pixel, channel) — the BN output is never written. Argmax byte = window tap (r*S+s) | 0x80 when the pooled
// value is > 0: a tap's value IS the pooled value of every window it wins, so bit 7 doubles as the BN's
// ReLU mask in the backward. Backward: the pooled gradient is gathered back per input pixel on the fly (no
// materialised maxpool gradient) by two passes: reduce (sum dz, sum dz*(x-mean)) and apply (dx of the BN).
struct PoolGeo {
  int N, H, W, C, P, Q, R, S, sh, sw, ph, pw;
  FastDiv c8, dQ, dP, dW, dHW;  // forward: C/8, Q, P; backward: W, H*W
};

__global__ void __launch_bounds__(256) bn_relu_maxpool_fwd_kernel(const bf16_t* __restrict__ x,
                                                                  const float* __restrict__ scale,
                                                                  const float* __restrict__ shift,
                                                                  bf16_t* __restrict__ y, uint8_t* __restrict__ arg,
                                                                  PoolGeo pg) {
  const uint32_t total = (uint32_t)pg.N * pg.P * pg.Q * (pg.C / 8);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    uint32_t pix, cc, t, q, n, p;
    fdivmod(i, pg.c8, pix, cc);
    fdivmod(pix, pg.dQ, t, q);
    fdivmod(t, pg.dP, n, p);
    float sc[8], sh[8], best[8];
    uint32_t bi[8];
    load_coef8(scale + cc * 8, sc);
    load_coef8(shift + cc * 8, sh);
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
    for (int r = 0; r < pg.R; ++r) {
      const int hi = (int)p * pg.sh - pg.ph + r;
      if ((unsigned)hi >= (unsigned)pg.H) continue;
      for (int s = 0; s < pg.S; ++s) {
        const int wi = (int)q * pg.sw - pg.pw + s;
        if ((unsigned)wi >= (unsigned)pg.W) continue;
        float f[8];
        load8(x + (((long)n * pg.H + hi) * pg.W + wi) * pg.C + cc * 8, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          // the value the unfused BN apply would have stored (bf16), compared as the unfused pool does
          const float v = bf2f(f2bf(fmaxf(fmaf(f[j], sc[j], sh[j]), 0.f)));
          if (v > best[j]) { best[j] = v; bi[j] = (uint32_t)(r * pg.S + s); }
        }
      }
    }
    store8(y + (long)i * 8, best);
    uint32_t b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) b[j] = bi[j] | (best[j] > 0.f ? 0x80u : 0u);
    uint2 a;
    a.x = b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24);
    a.y = b[4] | (b[5] << 8) | (b[6] << 16) | (b[7] << 24);
    *reinterpret_cast<uint2*>(arg + (long)i * 8) = a;
  }
}

// dz of input pixel (n, h, w), channels [8cc, 8cc+8): the pooled gradients of the windows this pixel won with a
// positive value, summed in tap order and rounded to bf16 (what the unfused pool backward stored). Any geometry.
__device__ __forceinline__ void pool_grad8(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                                           uint32_t n, int h, int w, int cc, const PoolGeo& pg, float* dz) {
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int rr = 0; rr < pg.R; ++rr) {
    const int th = h + pg.ph - rr;
    if (th < 0 || th % pg.sh) continue;
    const int p = th / pg.sh;
    if (p >= pg.P) continue;
    for (int ss = 0; ss < pg.S; ++ss) {
      const int tw = w + pg.pw - ss;
      if (tw < 0 || tw % pg.sw) continue;
      const int q = tw / pg.sw;
      if (q >= pg.Q) continue;
      const long o = (((long)n * pg.P + p) * pg.Q + q) * pg.C + cc * 8;
      const uint2 a = *reinterpret_cast<const uint2*>(arg + o);
      float g[8];
      load8(dy + o, g);
      const uint32_t me = (uint32_t)(rr * pg.S + ss) | 0x80u;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t bj = ((j < 4 ? a.x : a.y) >> (8 * (j & 3))) & 0xffu;
        if (bj == me) acc[j] += g[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) dz[j] = bf2f(f2bf(acc[j]));
}

// 3x3 / stride 2 / pad 1 windows over an input of exactly 2P x 2Q: the 2x2 input block (rows 2i, 2i+1; cols 2j,
// 2j+1) is covered by the 4 windows (i|i+1, j|j+1) only, so one thread gathers all four windows once (4 regular
// loads, no per-tap branching) and hands out dz for the block's pixels [(2i,2j), (2i,2j+1), (2i+1,2j),
// (2i+1,2j+1)], each summed in the same tap order as pool_grad8 (bitwise the same result).
struct Win8 {
  uint2 a;
  float g[8];
};
__device__ __forceinline__ void load_win(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ arg, long o,
                                         bool valid, Win8& w) {
  if (valid) {
    w.a = *reinterpret_cast<const uint2*>(arg + o);
    load8(dy + o, w.g);
  } else {
    w.a = make_uint2(0u, 0u);  // no bit 7: never selected
#pragma unroll
    for (int j = 0; j < 8; ++j) w.g[j] = 0.f;
  }
}
__device__ __forceinline__ void win_add(const Win8& w, uint32_t tap, float* acc) {
  const uint32_t me = tap | 0x80u;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t bj = ((j < 4 ? w.a.x : w.a.y) >> (8 * (j & 3))) & 0xffu;
    if (bj == me) acc[j] += w.g[j];
  }
}
__device__ __forceinline__ void pool_grad8_2x2(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                                               uint32_t n, int i, int j, int cc, const PoolGeo& pg,
                                               float (&dz)[4][8]) {
  const bool vi = i + 1 < pg.P, vj = j + 1 < pg.Q;
  const long o00 = (((long)n * pg.P + i) * pg.Q + j) * pg.C + cc * 8;
  const long rowq = (long)pg.Q * pg.C;
  Win8 w00, w01, w10, w11;
  load_win(dy, arg, o00, true, w00);
  load_win(dy, arg, o00 + pg.C, vj, w01);
  load_win(dy, arg, o00 + rowq, vi, w10);
  load_win(dy, arg, o00 + rowq + pg.C, vi && vj, w11);
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int c = 0; c < 8; ++c) dz[k][c] = 0.f;
  win_add(w00, 4, dz[0]);                                                       // (2i, 2j): tap (1,1)
  win_add(w01, 3, dz[1]); win_add(w00, 5, dz[1]);                               // (2i, 2j+1)
  win_add(w10, 1, dz[2]); win_add(w00, 7, dz[2]);                               // (2i+1, 2j)
  win_add(w11, 0, dz[3]); win_add(w10, 2, dz[3]); win_add(w01, 6, dz[3]); win_add(w00, 8, dz[3]);
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int c = 0; c < 8; ++c) dz[k][c] = bf2f(f2bf(dz[k][c]));
}

// Reduce pass. B2: rows are 2x2 input blocks (pool_grad8_2x2 geometry; dHW divides by P*Q, dW by Q);
// otherwise rows are input pixels (pool_grad8; dHW = H*W, dW = W).
template <bool B2>
__global__ void __launch_bounds__(256) maxpool_bn_bwd_reduce_kernel(const bf16_t* __restrict__ dy,
                                                                    const uint8_t* __restrict__ arg,
                                                                    const bf16_t* __restrict__ x,
                                                                    const float* __restrict__ mean, PoolGeo pg,
                                                                    float* __restrict__ part) {
  __shared__ float red[4096];
  const int C = pg.C;
  const long M = B2 ? (long)pg.N * pg.P * pg.Q : (long)pg.N * pg.H * pg.W;
  ColGeo g = colgeo(C);
  const int t = threadIdx.x;
  const int rsub = t / g.TPR;
  for (int cc0 = 0; cc0 < g.cols8; cc0 += g.TPR) {
    const int cc = cc0 + t % g.TPR;
    float s[8] = {0}, q[8] = {0};
    if (t < g.TPR * g.RPB && cc < g.cols8) {
      float mu[8];
      load_coef8(mean + cc * 8, mu);
      for (long r = (long)blockIdx.x * g.RPB + rsub; r < M; r += (long)gridDim.x * g.RPB) {
        uint32_t n, hw, h, w;
        fdivmod((uint32_t)r, pg.dHW, n, hw);
        fdivmod(hw, pg.dW, h, w);
        if constexpr (B2) {
          float d[4][8], xv[4][8];
#pragma unroll
          for (int k = 0; k < 4; ++k)
            load8(x + ((((long)n * pg.H + 2 * h + (k >> 1)) * pg.W + 2 * w + (k & 1)) * g.cols8 + cc) * 8, xv[k]);
          pool_grad8_2x2(dy, arg, n, (int)h, (int)w, cc, pg, d);
#pragma unroll
          for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              s[j] += d[k][j];
              q[j] = fmaf(d[k][j], xv[k][j] - mu[j], q[j]);
            }
        } else {
          float d[8], xv[8];
          load8(x + (r * g.cols8 + cc) * 8, xv);
          pool_grad8(dy, arg, n, (int)h, (int)w, cc, pg, d);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            s[j] += d[j];
            q[j] = fmaf(d[j], xv[j] - mu[j], q[j]);
          }
        }
      }
    }
    block_col_partials(s, q, cc0, g.TPR, g.RPB, C, part + (long)blockIdx.x * 2 * C, red);
  }
}

template <bool B2>
__global__ void __launch_bounds__(256) maxpool_bn_bwd_apply_kernel(const bf16_t* __restrict__ dy,
                                                                   const uint8_t* __restrict__ arg,
                                                                   const bf16_t* __restrict__ x,
                                                                   const float* __restrict__ coef, PoolGeo pg,
                                                                   bf16_t* __restrict__ dx) {
  const int C = pg.C;
  const long M = B2 ? (long)pg.N * pg.P * pg.Q : (long)pg.N * pg.H * pg.W;
  const ColGeo g = colgeo(C);
  const int t = threadIdx.x;
  if (t >= g.TPR * g.RPB) return;
  const int rsub = t / g.TPR;
  for (int cc = t % g.TPR; cc < g.cols8; cc += g.TPR) {
    float ka[8], kb[8], kc[8];
    load_coef8(coef + cc * 8, ka);
    load_coef8(coef + C + cc * 8, kb);
    load_coef8(coef + 2 * C + cc * 8, kc);
    for (long r = (long)blockIdx.x * g.RPB + rsub; r < M; r += (long)gridDim.x * g.RPB) {
      uint32_t n, hw, h, w;
      fdivmod((uint32_t)r, pg.dHW, n, hw);
      fdivmod(hw, pg.dW, h, w);
      if constexpr (B2) {
        float d[4][8], xv[4][8];
        long i8[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          i8[k] = (((long)n * pg.H + 2 * h + (k >> 1)) * pg.W + 2 * w + (k & 1)) * g.cols8 + cc;
          load8(x + i8[k] * 8, xv[k]);
        }
        pool_grad8_2x2(dy, arg, n, (int)h, (int)w, cc, pg, d);
#pragma unroll
        for (int k = 0; k < 4; ++k) bn_bwd_apply_row(d[k], xv[k], ka, kb, kc, dx, nullptr, i8[k]);
      } else {
        float d[8], xv[8];
        const long i8 = r * g.cols8 + cc;
        load8(x + i8 * 8, xv);
        pool_grad8(dy, arg, n, (int)h, (int)w, cc, pg, d);
        bn_bwd_apply_row(d, xv, ka, kb, kc, dx, nullptr, i8);
      }
    }
  }
}

// ---------------- LayerNorm: one wave per row, D % 8 == 0, D <= 512 * NC ----------------
// The row lives in registers (NC 16-byte chunks per lane): one HBM read, one write.
template <int NC>
// fb (optional): the LayerNorm input is the residual sum x + dropout(fb) of ops.add_dropout, formed here (same mask,
// same roundings as elementwise.hip add_dropout_kernel) and stored to ysum for the backward — one pass instead of
// the add kernel's write and this kernel's re-read of the sum.
__global__ void __launch_bounds__(256) ln_fwd_kernel(const bf16_t* __restrict__ x, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, bf16_t* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     long M, int D, float eps, const bf16_t* __restrict__ fb,
                                                     bf16_t* __restrict__ ysum, uint32_t thr, uint64_t seed,
                                                     const uint64_t* ctr) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const bf16_t* xr = x + row * D;
  const int d8 = D / 8;
  const uint64_t sd = fb ? step_seed(seed, ctr) : 0ull;
  const float dinv = 65536.f / (float)thr;
  float f[NC][8];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    const int c = lane + 64 * k;
    if (c < d8) {
      load8(xr + c * 8, f[k]);
      if (fb) {
        float b[8];
        load8(fb + row * D + c * 8, b);
        const uint32_t kb = keep_bits8(sd, row * d8 + c, thr);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          f[k][j] = bf2f(f2bf(f[k][j] + (((kb >> j) & 1u) ? bf2f(f2bf(b[j] * dinv)) : 0.f)));
        store8(ysum + row * D + c * 8, f[k]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += f[k][j];
    }
  }
  const float mu = wave_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NC; ++k)
    if (lane + 64 * k < d8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { float t = f[k][j] - mu; q += t * t; }
    }
  const float rs = rsqrtf(wave_sum(q) / D + eps);
  if (lane == 0) { mean_out[row] = mu; rstd_out[row] = rs; }
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    const int c = lane + 64 * k;
    if (c < d8) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (f[k][j] - mu) * rs * gamma[c * 8 + j] + beta[c * 8 + j];
      store8(y + row * D + c * 8, o);
    }
  }
}

// dx = rstd * (g*dy - mean(g*dy) - xhat*mean(g*dy*xhat)). Every lane owns the same columns in every row it
// visits, so dgamma/dbeta accumulate in registers across rows; the 4 waves combine through LDS and each
// block writes one partial row part[block][2D] (dgamma | dbeta) for a deterministic dtf_sum_rows.
template <int NC>
__global__ void __launch_bounds__(256) ln_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, bf16_t* __restrict__ dx,
                                                     float* __restrict__ part, long M, int D,
                                                     const bf16_t* __restrict__ res, bf16_t* __restrict__ dfo,
                                                     uint32_t thr, uint64_t seed, const uint64_t* ctr) {
  extern __shared__ float sred[];  // [4][2D]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int d8 = D / 8;
  // dfo: the input x was y = x0 + dropout(f) (ops.add_dropout); the branch gradient df = dropout(dx) with that mask
  // (elementwise.hip dropout_kernel: same chunk hashes, same roundings) is written in the same store pass
  const uint64_t sd = dfo ? step_seed(seed, ctr) : 0ull;
  const float dinv = 65536.f / (float)thr;
  float gm[NC][8], ag[NC][8], ab[NC][8];
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    const int c = lane + 64 * k;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      gm[k][j] = c < d8 ? gamma[c * 8 + j] : 0.f;
      ag[k][j] = 0.f;
      ab[k][j] = 0.f;
    }
  }
  // software-pipelined over the wave's rows: the next row's x / dy / statistics are loaded while this row's
  // two wave reductions run (a row per wave is otherwise one exposed memory latency + two reduction chains)
  const long stride = (long)gridDim.x * 4;
  long row = (long)blockIdx.x * 4 + w;
  uint4 nx[NC], ng[NC];
  float nmu = 0.f, nrs = 0.f;
  auto fetch = [&](long r) {
    if (r >= M) return;
    nmu = mean[r];
    nrs = rstd[r];
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const int c = lane + 64 * k;
      if (c < d8) {
        nx[k] = *reinterpret_cast<const uint4*>(x + r * D + c * 8);
        ng[k] = *reinterpret_cast<const uint4*>(dy + r * D + c * 8);
      }
    }
  };
  fetch(row);
  for (; row < M; row += stride) {
    const float mu = nmu, rs = nrs;
    float xh[NC][8], g[NC][8];
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const uint32_t xw[4] = {nx[k].x, nx[k].y, nx[k].z, nx[k].w}, gw[4] = {ng[k].x, ng[k].y, ng[k].z, ng[k].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        xh[k][2 * q] = __uint_as_float(xw[q] << 16); xh[k][2 * q + 1] = __uint_as_float(xw[q] & 0xffff0000u);
        g[k][2 * q] = __uint_as_float(gw[q] << 16); g[k][2 * q + 1] = __uint_as_float(gw[q] & 0xffff0000u);
      }
    }
    fetch(row + stride);
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const int c = lane + 64 * k;
      if (c < d8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[k][j] = (xh[k][j] - mu) * rs;
          const float gd = g[k][j] * gm[k][j];
          a += gd;
          b += gd * xh[k][j];
          ag[k][j] += g[k][j] * xh[k][j];
          ab[k][j] += g[k][j];
        }
      }
    }
    a = wave_sum(a) / D;
    b = wave_sum(b) / D;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const int c = lane + 64 * k;
      if (c < d8) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rs * (g[k][j] * gm[k][j] - a - xh[k][j] * b);
        if (res) {  // residual gradient joined in the store: round(round(dx) + res), as LN backward + an add
          float rv[8];
          load8(res + row * D + c * 8, rv);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = bf2f(f2bf(o[j])) + rv[j];
        }
        store8(dx + row * D + c * 8, o);
        if (dfo) {
          const uint32_t kb = keep_bits8(sd, row * d8 + c, thr);
          float q[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) q[j] = ((kb >> j) & 1u) ? bf2f(f2bf(o[j])) * dinv : 0.f;
          store8(dfo + row * D + c * 8, q);
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    const int c = lane + 64 * k;
    if (c < d8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sred[w * 2 * D + c * 8 + j] = ag[k][j];
        sred[w * 2 * D + D + c * 8 + j] = ab[k][j];
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * D; i += blockDim.x)
    part[(long)blockIdx.x * 2 * D + i] = sred[i] + sred[2 * D + i] + sred[4 * D + i] + sred[6 * D + i];
}

int red_grid(long M, int C) {
  ColGeo g = colgeo(C);
  long rows_per_thread = 32;
  long blocks = (M + (long)g.RPB * rows_per_thread - 1) / ((long)g.RPB * rows_per_thread);
  if (blocks > 1024) blocks = 1024;
  if (blocks < 256 && M >= 256L * g.RPB) blocks = 256;
  if (blocks < 1) blocks = 1;
  return (int)blocks;
}

// leader rows left by the first (grouping) pass of a BN statistics reduction, which the finalize kernel then sums:
// the grouping pass runs one block per leader row (more rows = more blocks reading the partials in parallel)
static int bn_group_target() { return 256; }  // (the finalize kernels sum up to ~256 rows themselves)

// Elementwise passes that consume a GEMM output sweep the rows last-to-first: the GEMM wrote them first-to-last,
// so the most recently written rows (still in the 256 MiB Infinity Cache) are read first; the next GEMM then
// reads this pass's output in its own first-to-last order, again most recent first. Measured: no effect on
// ResNet-50 (b256): off.
static int ew_reverse() { return 0; }

// Variant of the streaming BN passes (tools/bench_bnb.py sweeps it; dtf_set_ew_variant): 0 = EU rows per trip,
// 1 = + nontemporal hints, 2 = 8 rows per trip, 3 = 8 rows + nontemporal, 4 = 2 rows per trip
// Measured (tools/bench_bnb.py, MI355X, ResNet-50 b256 shapes): 2 rows per trip is 3-9% faster than 4 on the
// tensors that miss the Infinity Cache; nontemporal hints and 8 rows are not faster.
int g_ew_variant = 4;
int g_ew_apply_nu = 2;  // rows per trip of the forward apply pass (2, 4 or 8; 4 measured -0.4%)

// elementwise channels-last passes: enough blocks to fill the chip, each with >= nu row trips when possible
int ew_grid(long M, int C, int nu = EU) {
  ColGeo g = colgeo(C);
  long blocks = (M + (long)g.RPB * nu - 1) / ((long)g.RPB * nu);
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  return (int)blocks;
}

}  // namespace

// Statistics of x: writes G partial rows into `part` (capacity >= 1024*2*C floats), returns G via *rows.
DTF_API int dtf_bn_stats(const void* x, long M, int C, float* part, int* rows, void* stream) {
  if (C & 7) return -1;
  int G = red_grid(M, C);
  hipLaunchKernelGGL(bn_stats_kernel, dim3(G), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, M, C, part);
  *rows = G;
  return (int)hipGetLastError();
}

DTF_API void dtf_sum_rows(float* rows, long stride, int nrows, long W, float* out, int accumulate, void* stream);
DTF_API int dtf_group_rows_once(float* rows, long stride, int nrows, long W, int target, long* out_stride,
                                void* stream);

DTF_API int dtf_bn_finalize(float* part, int T, const float* gamma, const float* beta, float* running_mean,
                            float* running_var, long M, int C, float momentum, float eps, float* scale,
                            float* shift, float* mean_out, float* invstd_out, void* stream) {
  long rs = 2L * C;
  T = dtf_group_rows_once(part, rs, T, 2L * C, bn_group_target(), &rs, stream);  // <= target leader rows, one launch
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(cdiv(C, 64)), dim3(FIN_NT), 0, (hipStream_t)stream, part, T, rs, gamma,
                     beta,
                     running_mean, running_var, M, C, momentum, eps, scale, shift, mean_out, invstd_out);
  return (int)hipGetLastError();
}

DTF_API int dtf_set_ew_variant(int v) {
  g_ew_variant = v;
  return 0;
}
DTF_API int dtf_set_ew_apply_nu(int nu) {
  g_ew_apply_nu = nu;
  return 0;
}

DTF_API int dtf_bn_infer_coeff(const float* gamma, const float* beta, const float* rmean, const float* rvar, int C,
                               float eps, float* scale, float* shift, void* stream) {
  hipLaunchKernelGGL(bn_infer_coeff_kernel, dim3(cdiv(C, 256)), dim3(256), 0, (hipStream_t)stream, gamma, beta,
                     rmean, rvar, C, eps, scale, shift);
  return (int)hipGetLastError();
}

// mbits (optional, relu only): 1-bit ReLU mask, M*C/8 bytes, consumed by dtf_bn_bwd instead of re-reading y
// rscale/rshift (optional, with res): res is a BN input; res * rscale + rshift is added (see bn_apply_kernel)
DTF_API int dtf_bn_apply(const void* x, const float* scale, const float* shift, const void* res, void* y, long M,
                         int C, int relu, void* mbits, const float* rscale, const float* rshift, void* stream) {
  if ((C & 7) || ((rscale == nullptr) != (rshift == nullptr))) return -1;
  const int nu = g_ew_apply_nu;
  hipLaunchKernelGGL((nu == 2 ? bn_apply_kernel<2> : nu == 8 ? bn_apply_kernel<8> : bn_apply_kernel<4>),
                     dim3(ew_grid(M, C, nu == 2 || nu == 8 ? nu : 4)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)x, scale, shift, (const bf16_t*)res, (bf16_t*)y, M, C, relu,
                     relu ? (uint8_t*)mbits : nullptr, res ? rscale : nullptr, res ? rshift : nullptr, ew_reverse());
  return (int)hipGetLastError();
}

struct ShortcutStats {  // optional fused projection-shortcut BN reduction (bn_bwd_apply_kernel<true>)
  const void* x2;
  const float* mean2;
  float* part2;
  int* rows2;
};
static int bn_bwd_tail(const void* dy, const void* ymask, const void* mbits, const void* x, const float* mean,
                       const float* invstd, const float* gamma, long M, int C, void* dx, void* dz_out, float* dgamma,
                       float* dbeta, int accumulate, float* part, int G, float* coef, hipStream_t st,
                       const ShortcutStats* sc = nullptr);

// work: (2*1024 + 3) * C floats (partials + coefficients)
// ReLU mask from mbits (1 bit/element, preferred) or from the bf16 output ymask; neither = no ReLU
DTF_API int dtf_bn_bwd(const void* dy, const void* ymask, const void* mbits, const void* x, const float* mean,
                       const float* invstd,
                       const float* gamma, long M, int C, void* dx, void* dz_out, float* dgamma, float* dbeta,
                       int accumulate, float* work, const void* x2, const float* mean2, float* part2, int* rows2,
                       void* stream) {
  if (C & 7) return -1;
  const ShortcutStats sc{x2, mean2, part2, rows2};
  hipStream_t st = (hipStream_t)stream;
  float* coef = work;
  float* part = work + 3 * C;
  int G = red_grid(M, C);
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(G), dim3(256), 0, st, (const bf16_t*)dy, (const bf16_t*)ymask,
                     (const uint8_t*)mbits, (const bf16_t*)x, mean, invstd, M, C, part);
  return bn_bwd_tail(dy, ymask, mbits, x, mean, invstd, gamma, M, C, dx, dz_out, dgamma, dbeta, accumulate, part, G,
                     coef, st, &sc);
}

// Backward with the reduction already done by the GEMM that produced dy (dtf_conv_dgrad's fused BN-backward
// statistics): `part` holds T partial rows [T][2C] (used as scratch); coef: 3*C floats.
DTF_API int dtf_bn_bwd_partials(const void* dy, const void* mbits, const void* x, const float* mean,
                                const float* invstd, const float* gamma, long M, int C, void* dx, void* dz_out,
                                float* dgamma, float* dbeta, int accumulate, float* part, int T, float* coef,
                                const void* x2, const float* mean2, float* part2, int* rows2, void* stream) {
  if ((C & 7) || T < 1) return -1;
  const ShortcutStats sc{x2, mean2, part2, rows2};
  return bn_bwd_tail(dy, nullptr, mbits, x, mean, invstd, gamma, M, C, dx, dz_out, dgamma, dbeta, accumulate, part, T,
                     coef, (hipStream_t)stream, &sc);
}

// Backward apply only: the coefficients `coef` (3*C) were already finalized — by the data-gradient GEMM that produced
// dy (dtf_conv_dgrad_bn's fused finalize). Optional fused projection-shortcut statistics as in dtf_bn_bwd_partials.
DTF_API int dtf_bn_bwd_apply_coef(const void* dy, const void* mbits, const void* x, long M, int C, void* dx,
                                  void* dz_out, const float* coef, const void* x2, const float* mean2, float* part2,
                                  int* rows2, void* stream) {
  if (C & 7) return -1;
  const ShortcutStats sc{x2, mean2, part2, rows2};
  return bn_bwd_tail(dy, nullptr, mbits, x, nullptr, nullptr, nullptr, M, C, dx, dz_out, nullptr, nullptr, 0, nullptr,
                     0, const_cast<float*>(coef), (hipStream_t)stream, &sc);
}

// Sum the G partial rows [G][2C] of a BN backward reduction and finalize: dgamma/dbeta and the apply
// coefficients `coef` (3*C floats): a grouping launch, then the finalize launch.
static void bn_bwd_finalize_launch(float* part, int G, const float* mean, const float* invstd, const float* gamma,
                                   long M, int C, float* dgamma, float* dbeta, int accumulate, float* coef,
                                   hipStream_t st) {
  long rs = 2L * C;
  int T = dtf_group_rows_once(part, rs, G, 2L * C, bn_group_target(), &rs, (void*)st);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(cdiv(C, 64)), dim3(FIN_NT), 0, st, part, T, rs, gamma, mean, invstd, M, C,
                     dgamma, dbeta, accumulate, coef);
}

// Finalize only: sum the T partial rows [T][2C] in `part` (scratch) into dgamma/dbeta and the apply coefficients
// coef (3*C) — for a consumer that applies them itself (pwbwd.hip dtf_pw_conv_bwd_bn).
DTF_API int dtf_bn_bwd_coef(float* part, int T, const float* mean, const float* invstd, const float* gamma, long M,
                            int C, float* dgamma, float* dbeta, int accumulate, float* coef, void* stream) {
  if ((C & 7) || T < 1 || !part || !coef) return -1;
  bn_bwd_finalize_launch(part, T, mean, invstd, gamma, M, C, dgamma, dbeta, accumulate, coef, (hipStream_t)stream);
  return (int)hipGetLastError();
}

static int bn_bwd_tail(const void* dy, const void* ymask, const void* mbits, const void* x, const float* mean,
                       const float* invstd, const float* gamma, long M, int C, void* dx, void* dz_out, float* dgamma,
                       float* dbeta, int accumulate, float* part, int G, float* coef, hipStream_t st,
                       const ShortcutStats* sc) {
  if (part) bn_bwd_finalize_launch(part, G, mean, invstd, gamma, M, C, dgamma, dbeta, accumulate, coef, st);
  const ColGeo geo = colgeo(C);
  const int grid = ew_grid(M, C, g_ew_variant == 4 ? 2 : EU);  // (the shortcut-fused launch: one partial row per block)
  const bool fuse_sc = sc && sc->x2 && sc->part2 && dz_out && (ymask || mbits) && geo.cols8 <= 256 &&
                       geo.TPR * geo.RPB == 256;
  if (sc && sc->rows2) *sc->rows2 = fuse_sc ? grid : 0;
  if (fuse_sc) {
    if (g_ew_variant == 4)
      hipLaunchKernelGGL((bn_bwd_apply_kernel<true, 2>), dim3(grid), dim3(256), 0, st, (const bf16_t*)dy,
                         (const bf16_t*)ymask, (const uint8_t*)mbits, (const bf16_t*)x, coef, M, C, (bf16_t*)dx,
                         (bf16_t*)dz_out, (const bf16_t*)sc->x2, sc->mean2, sc->part2, ew_reverse());
    else
      hipLaunchKernelGGL(bn_bwd_apply_kernel<true>, dim3(grid), dim3(256), 0, st, (const bf16_t*)dy,
                         (const bf16_t*)ymask, (const uint8_t*)mbits, (const bf16_t*)x, coef, M, C, (bf16_t*)dx,
                         (bf16_t*)dz_out, (const bf16_t*)sc->x2, sc->mean2, sc->part2, ew_reverse());
  } else {
#define BNB_LAUNCH(NU, NT)                                                                                        \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<false, NU, NT>), dim3(ew_grid(M, C, NU)), dim3(256), 0, st,            \
                     (const bf16_t*)dy, (const bf16_t*)ymask, (const uint8_t*)mbits, (const bf16_t*)x, coef, M, C, \
                     (bf16_t*)dx, (bf16_t*)dz_out, nullptr, nullptr, nullptr, ew_reverse())
    switch (g_ew_variant) {
      case 1: BNB_LAUNCH(EU, true); break;
      case 2: BNB_LAUNCH(8, false); break;
      case 3: BNB_LAUNCH(8, true); break;
      case 4: BNB_LAUNCH(2, false); break;
      default: BNB_LAUNCH(EU, false); break;
    }
#undef BNB_LAUNCH
  }
  return (int)hipGetLastError();
}

static bool pool_geo(int N, int H, int W, int C, int P, int Q, int R, int S, int sh, int sw, int ph, int pw,
                     PoolGeo* pg) {
  if ((C & 7) || R * S > 127 || sh < 1 || sw < 1) return false;
  if ((long)N * H * W * C >= (1L << 31) || (long)N * P * Q * C >= (1L << 31)) return false;
  *pg = PoolGeo{N, H, W, C, P, Q, R, S, sh, sw, ph, pw, make_fastdiv(C / 8), make_fastdiv(Q), make_fastdiv(P),
                make_fastdiv(W), make_fastdiv((uint32_t)(H * W))};
  return true;
}

// Fused BatchNorm(scale/shift) + ReLU + MaxPool forward over the conv output x [N,H,W,C] -> y [N,P,Q,C] and
// the argmax/mask bytes arg [N,P,Q,C] (see bn_relu_maxpool_fwd_kernel).
DTF_API int dtf_bn_relu_maxpool_fwd(const void* x, const float* scale, const float* shift, void* y, void* arg, int N,
                                    int H, int W, int C, int P, int Q, int R, int S, int sh, int sw, int ph, int pw,
                                    void* stream) {
  PoolGeo pg;
  if (!pool_geo(N, H, W, C, P, Q, R, S, sh, sw, ph, pw, &pg)) return -1;
  const long total = (long)N * P * Q * (C / 8);
  hipLaunchKernelGGL(bn_relu_maxpool_fwd_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)x, scale, shift, (bf16_t*)y, (uint8_t*)arg, pg);
  return (int)hipGetLastError();
}

// Backward of dtf_bn_relu_maxpool_fwd: dy = gradient of the pooled output; writes dx (gradient of the conv
// output x), dgamma/dbeta (+= when accumulate). work: (2*1024 + 3) * C floats.
DTF_API int dtf_maxpool_bn_bwd(const void* dy, const void* arg, const void* x, const float* mean, const float* invstd,
                               const float* gamma, int N, int H, int W, int C, int P, int Q, int R, int S, int sh,
                               int sw, int ph, int pw, void* dx, float* dgamma, float* dbeta, int accumulate,
                               float* work, void* stream) {
  PoolGeo pg;
  if (!pool_geo(N, H, W, C, P, Q, R, S, sh, sw, ph, pw, &pg)) return -1;
  hipStream_t st = (hipStream_t)stream;
  const long M = (long)N * H * W;
  float* coef = work;
  float* part = work + 3 * C;
  // the stem's 3x3/2 pad-1 pool over an even-sized map: 2x2-block gathers (pool_grad8_2x2)
  const bool b2 = R == 3 && S == 3 && sh == 2 && sw == 2 && ph == 1 && pw == 1 && H == 2 * P && W == 2 * Q;
  if (b2) {
    pg.dHW = make_fastdiv((uint32_t)(P * Q));
    pg.dW = make_fastdiv((uint32_t)Q);
  }
  const long rows = b2 ? (long)N * P * Q : M;
  const int G = red_grid(rows, C);
  if (b2)
    hipLaunchKernelGGL((maxpool_bn_bwd_reduce_kernel<true>), dim3(G), dim3(256), 0, st, (const bf16_t*)dy,
                       (const uint8_t*)arg, (const bf16_t*)x, mean, pg, part);
  else
    hipLaunchKernelGGL((maxpool_bn_bwd_reduce_kernel<false>), dim3(G), dim3(256), 0, st, (const bf16_t*)dy,
                       (const uint8_t*)arg, (const bf16_t*)x, mean, pg, part);
  bn_bwd_finalize_launch(part, G, mean, invstd, gamma, M, C, dgamma, dbeta, accumulate, coef, st);
  if (!dx) return (int)hipGetLastError();  // coefficients only: the consumer applies them (dtf_stem_wgrad_fused)
  if (b2)
    hipLaunchKernelGGL((maxpool_bn_bwd_apply_kernel<true>), dim3(ew_grid(rows, C)), dim3(256), 0, st,
                       (const bf16_t*)dy, (const uint8_t*)arg, (const bf16_t*)x, coef, pg, (bf16_t*)dx);
  else
    hipLaunchKernelGGL((maxpool_bn_bwd_apply_kernel<false>), dim3(ew_grid(M, C)), dim3(256), 0, st,
                       (const bf16_t*)dy, (const uint8_t*)arg, (const bf16_t*)x, coef, pg, (bf16_t*)dx);
  return (int)hipGetLastError();
}

#define LN_DISPATCH(D, F) \
  if ((D) <= 512) F(1); else if ((D) <= 1024) F(2); else if ((D) <= 1536) F(3); else F(4)

static int ln_fwd_impl(const void* x, const float* gamma, const float* beta, void* y, float* mean, float* rstd,
                       long M, int D, float eps, const void* fb, void* ysum, uint32_t thr, unsigned long long seed,
                       const void* ctr, void* stream) {
  if ((D & 7) || D > 2048) return -1;
#define LNF(NC) \
  hipLaunchKernelGGL(ln_fwd_kernel<NC>, dim3(cdiv(M, 4)), dim3(256), 0, (hipStream_t)stream,             \
                      (const bf16_t*)x, gamma, beta, (bf16_t*)y, mean, rstd, M, D, eps, (const bf16_t*)fb,    \
                      (bf16_t*)ysum, thr, (uint64_t)seed, (const uint64_t*)ctr)
  LN_DISPATCH(D, LNF);
#undef LNF
  return (int)hipGetLastError();
}

DTF_API int dtf_layernorm_fwd(const void* x, const float* gamma, const float* beta, void* y, float* mean,
                              float* rstd, long M, int D, float eps, void* stream) {
  return ln_fwd_impl(x, gamma, beta, y, mean, rstd, M, D, eps, nullptr, nullptr, 65536u, 0ull, nullptr, stream);
}

// LayerNorm of ysum = x + dropout(f, keep, seed, ctr) (ops.add_dropout deferred to its LayerNorm): ysum is written
// too (the LayerNorm input the backward needs, the residual stream of pre-LN blocks).
DTF_API int dtf_add_dropout_layernorm_fwd(const void* x, const void* f, void* ysum, const float* gamma,
                                          const float* beta, void* y, float* mean, float* rstd, long M, int D,
                                          float eps, float keep, unsigned long long seed, const void* ctr,
                                          void* stream) {
  return ln_fwd_impl(x, gamma, beta, y, mean, rstd, M, D, eps, f, ysum, keep_threshold(keep), seed, ctr, stream);
}

DTF_API int dtf_layernorm_bwd2(const void* dy, const void* x, const float* gamma, const float* mean,
                               const float* rstd, void* dx, float* dgb, float* ws, long ws_elems, long M, int D,
                               int accumulate, const void* res, void* stream);
// dgb = [dgamma | dbeta] (2D floats, overwritten or accumulated); ws >= min(1024, M/16 + 1) * 2D floats.
DTF_API int dtf_layernorm_bwd(const void* dy, const void* x, const float* gamma, const float* mean, const float* rstd,
                              void* dx, float* dgb, float* ws, long ws_elems, long M, int D, int accumulate,
                              void* stream) {
  return dtf_layernorm_bwd2(dy, x, gamma, mean, rstd, dx, dgb, ws, ws_elems, M, D, accumulate, nullptr, stream);
}
// res (optional, bf16 [M][D]): another gradient of the LayerNorm's input (the residual branch), added to dx
static int ln_bwd_impl(const void* dy, const void* x, const float* gamma, const float* mean, const float* rstd,
                       void* dx, float* dgb, float* ws, long ws_elems, long M, int D, int accumulate, const void* res,
                       void* dfo, uint32_t thr, unsigned long long seed, const void* ctr, void* stream);
DTF_API int dtf_layernorm_bwd2(const void* dy, const void* x, const float* gamma, const float* mean,
                               const float* rstd, void* dx, float* dgb, float* ws, long ws_elems, long M, int D,
                               int accumulate, const void* res, void* stream) {
  return ln_bwd_impl(dy, x, gamma, mean, rstd, dx, dgb, ws, ws_elems, M, D, accumulate, res, nullptr, 65536u, 0ull,
                     nullptr, stream);
}
static int ln_bwd_impl(const void* dy, const void* x, const float* gamma, const float* mean, const float* rstd,
                       void* dx, float* dgb, float* ws, long ws_elems, long M, int D, int accumulate, const void* res,
                       void* dfo, uint32_t thr, unsigned long long seed, const void* ctr, void* stream) {
  if ((D & 7) || D > 2048) return -1;
  // ~48 rows (12 per wave) per block, 256..1024 blocks: long enough software-pipelined row walks per wave and a
  // smaller partial-row reduction; measured in the training step (the pass shares the CUs with the weight-gradient
  // GEMMs): BERT-base 19.60 -> 19.17 ms/step vs 16 rows per block.
  long blocks = std::max<long>(256, cdiv(M, 48));
  blocks = std::max<long>(1, std::min<long>(blocks, std::min<long>(1024, cdiv(M, 4))));
  blocks = std::min<long>(blocks, std::max<long>(1, ws_elems / (2L * D)));
  const size_t sh = sizeof(float) * 8 * D;
#define LNB(NC) \
  hipLaunchKernelGGL(ln_bwd_kernel<NC>, dim3((unsigned)blocks), dim3(256), sh, (hipStream_t)stream,       \
                      (const bf16_t*)dy, (const bf16_t*)x, gamma, mean, rstd, (bf16_t*)dx, ws, M, D,            \
                      (const bf16_t*)res, (bf16_t*)dfo, thr, (uint64_t)seed, (const uint64_t*)ctr)
  LN_DISPATCH(D, LNB);
#undef LNB
  if (dgb) dtf_sum_rows(ws, 2L * D, (int)blocks, 2L * D, dgb, accumulate, stream);
  return (int)hipGetLastError();
}

// The data-gradient half of dtf_layernorm_bwd2: dx and the per-block [dgamma | dbeta] partial rows in part (>= 2D
// floats per row, part_elems in all); *rows = the partial row count. The caller reduces the rows where it likes
// (ops/norm.py: on the weight-gradient side stream, off the dgrad chain).
// dfo (optional): also the gradient of a dropped-out branch that the LayerNorm input was the residual sum of
// (ops.add_dropout: x = x0 + dropout(f, keep, seed, ctr)): df = dropout(dx) with the same mask, in the same pass.
DTF_API int dtf_layernorm_bwd_part(const void* dy, const void* x, const float* gamma, const float* mean,
                                   const float* rstd, void* dx, float* part, long part_elems, long M, int D,
                                   const void* res, int* rows, void* dfo, float keep, unsigned long long seed,
                                   const void* ctr, void* stream) {
  if ((D & 7) || D > 2048 || part_elems < 2L * D) return -1;
  const long blocks = std::max<long>(
      1, std::min<long>(std::min<long>(std::max<long>(256, cdiv(M, 48)), std::min<long>(1024, cdiv(M, 4))),
                        part_elems / (2L * D)));
  *rows = (int)blocks;
  return ln_bwd_impl(dy, x, gamma, mean, rstd, dx, nullptr, part, blocks * 2L * D, M, D, 0, res, dfo,
                     dfo ? keep_threshold(keep) : 65536u, seed, ctr, stream);
}
