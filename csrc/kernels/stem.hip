// ResNet stem forward as its own kernel: the 7x7/2 pad-3 convolution in its space-to-depth form (a 4x4/1 conv over
// the [N, H/2+3, W/2+3, 16] s2d image, 64 output channels, ops/conv.py stem_s2d_filter) plus the training BatchNorm
// partial statistics of its output.
//
// Why not the implicit-GEMM conv: the reduction dimension is 16 taps x 16 channels, so the generic loader moves
// 32-byte pixel pieces and re-reads every input pixel once per tap through L2 (r1_stem_s2d_tiles: 261-309 us,
// ~400 TF, against a ~105 us HBM floor: 108 MB in, 411 MB out). Here a work unit is RG output rows of one image:
// the RG+3 input rows it needs are ONE contiguous span of the s2d image, copied to LDS with 16-B loads; every
// MFMA operand is then a 16-B LDS read, because a 32-wide k chunk of this filter is two horizontally adjacent
// pixels x 16 channels (32 contiguous bf16 in the row). The whole filter (64 x 256 bf16) sits in VGPRs as MFMA
// fragments, loaded once per (persistent) block.
//
// MFMA: v_mfma_f32_16x16x32_bf16 with the filter as the row operand: lane l ends up owning output channels
// nb*16 + 4*(l>>4) + i (i = 0..3) of pixel l&15 — one 8-B store per lane and fragment, merged into full lines in L2.
// Parity: the ResNet-50 conv1 7x7/2 3->64 at 112^2 + its training BatchNorm.
#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace {

constexpr int SC = 16;   // s2d channels
constexpr int SK = 64;   // output channels
constexpr int RG = 8;    // output rows per work unit
constexpr int WMAX = 120;  // widest s2d row staged (W/2 + 3 <= 120: images up to 234 wide)
constexpr int NT = 256;

__global__ void __launch_bounds__(NT, 2) stem_fwd_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wt,
                                                         bf16_t* __restrict__ Y, float* __restrict__ part, int N,
                                                         int Hs, int Ws, int P, int Q) {
  // RG + 3 rows + one row of slack: the last m-block of a row reads up to 3 pixels past Q (never used)
  __shared__ __attribute__((aligned(16))) bf16_t sx[(RG + 4) * WMAX * SC];
  __shared__ float red[4][2 * SK];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  const int QB = Q / 16, UPI = (P + RG - 1) / RG, units = N * UPI;

  v8bf wf[4][8];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int kc = 0; kc < 8; ++kc)
      wf[nb][kc] = *reinterpret_cast<const v8bf*>(Wt + (nb * 16 + (lane & 15)) * (16 * SC) + kc * 32 + 8 * g);

  float s[4][4], q2[4][4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int i = 0; i < 4; ++i) s[nb][i] = q2[nb][i] = 0.f;

  const int rowe = Ws * SC;  // elements per s2d row
  for (int u = blockIdx.x; u < units; u += gridDim.x) {
    const int img = u / UPI, p0 = (u - img * UPI) * RG;
    const int rows = min(RG, P - p0);
    const int n16 = (rows + 3) * rowe / 8;  // 16-B pieces of the contiguous input span
    const uint4* src = reinterpret_cast<const uint4*>(X + ((long)img * Hs + p0) * rowe);
    __syncthreads();  // the previous unit's operand reads are done
    for (int i = tid; i < n16; i += NT) reinterpret_cast<uint4*>(sx)[i] = src[i];
    __syncthreads();
    const int nmb = rows * QB;
    for (int mb = w; mb < nmb; mb += 4) {
      const int r = mb / QB, q = (mb - r * QB) * 16 + (lane & 15);
      const bf16_t* base = sx + (r * Ws + q) * SC + 8 * g;
      v4f acc[4];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[nb] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < 8; ++kc) {
        // chunk kc: filter row a = kc/2, taps b0 = 2*(kc&1) and b0+1 (16 channels each) = 32 contiguous bf16
        const v8bf xf = *reinterpret_cast<const v8bf*>(base + (kc >> 1) * rowe + (kc & 1) * 2 * SC);
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[nb][kc], xf, acc[nb], 0, 0, 0);
      }
      bf16_t* dst = Y + (((long)img * P + p0 + r) * Q + q) * SK + 4 * g;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const uint2 o = make_uint2(pack2bf(acc[nb][0], acc[nb][1]), pack2bf(acc[nb][2], acc[nb][3]));
        *reinterpret_cast<uint2*>(dst + nb * 16) = o;
        // statistics of the stored (bf16) values: what the BatchNorm apply will normalise
        const float f[4] = {__uint_as_float(o.x << 16), __uint_as_float(o.x & 0xffff0000u),
                            __uint_as_float(o.y << 16), __uint_as_float(o.y & 0xffff0000u)};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          s[nb][i] += f[i];
          q2[nb][i] = fmaf(f[i], f[i], q2[nb][i]);
        }
      }
    }
  }
  // per-channel partial sums of this block: over the 16 pixel lanes of each row (DPP), then over the 4 waves
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float a = row16_sum(s[nb][i]), b = row16_sum(q2[nb][i]);
      if ((lane & 15) == 0) {
        red[w][nb * 16 + 4 * g + i] = a;
        red[w][SK + nb * 16 + 4 * g + i] = b;
      }
    }
  __syncthreads();
  if (tid < 2 * SK) part[(long)blockIdx.x * 2 * SK + tid] = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
}

}  // namespace

// Eligible shapes: C = 16 (s2d), K = 64, 4x4/1, no padding, Q a multiple of 16, s2d row <= WMAX pixels.
// Returns -1 when not eligible (the caller keeps the implicit-GEMM path). part: >= grid rows of [2*64] floats
// (sum, sum of squares); *rows = that row count.
DTF_API int dtf_stem_fwd(const void* X, const void* Wt, void* Y, float* part, int* rows, int N, int Hs, int Ws, int C,
                         int K, int R, int S, int P, int Q, void* stream) {
  if (C != SC || K != SK || R != 4 || S != 4 || P != Hs - 3 || Q != Ws - 3 || (Q & 15) || Ws > WMAX || !part)
    return -1;
  if (((uintptr_t)X | (uintptr_t)Wt | (uintptr_t)Y) & 15) return -1;
  const int units = N * ((P + RG - 1) / RG);
  constexpr int grid_cap = 512;  // 2 blocks per CU (register-bound: the filter lives in VGPRs)
  // the callers size `part` for the conv stats contract: ceil(N*P*Q/64) rows — never write more rows than that
  // (the units loop is persistent, so a smaller grid only means more units per block)
  const long cap_rows = ((long)N * P * Q + 63) / 64;
  const int grid = (int)std::min<long>(std::min(units, std::max(1, grid_cap)), std::max<long>(1, cap_rows));
  hipLaunchKernelGGL(stem_fwd_kernel, dim3(grid), dim3(NT), 0, (hipStream_t)stream, (const bf16_t*)X,
                     (const bf16_t*)Wt, (bf16_t*)Y, part, N, Hs, Ws, P, Q);
  if (rows) *rows = grid;
  return (int)hipGetLastError();
}
