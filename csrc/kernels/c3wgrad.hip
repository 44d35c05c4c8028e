// Persistent weight gradient of a 64 -> 64 channel 3x3 / stride 1 / pad 1 convolution (ResNet-50 stage 1, 56 x 56):
//   dW[k][a][b][c] = sum over output pixels (n, h, w) of dY[n][h][w][k] * X[n][h + a - 1][w + b - 1][c].
//
// The general tiles run it as an implicit GEMM with split-K slabs (gemm_kernel<128,64,...,8,7>: ~0.66 ms alone at
// batch 1024, 357 TF/s; 1.5-1.75 ms beside the data-gradient chain on the side stream, three per step). The filter is
// small (64 x 576) and the reduction long (3.2 M pixels), so the stem kernel's structure (stemwgrad.hip) fits:
//  * one block per CU, persistent over a contiguous range of output rows; the whole filter gradient in the
//    accumulators (wave w owns input channels 16w..16w+15: 9 taps x 64 k x 16 c = 144 registers per lane), one f32
//    partial per block, summed in a fixed order by dtf_sum_rows;
//  * per output row one dY row image (W <= 64 pixels, zero past W) and the X rows it needs go through LDS by LDS-DMA,
//    three rows ahead. X rows sit in an 8-slot ring indexed by a virtual row number that counts each image's two
//    zero padding rows, so the rows of consecutive outputs — across image boundaries too — are consecutive and each X
//    row leaves HBM once per block; a padding row is an out-of-range DMA (zeros);
//  * each X row slot holds pixel x at position x + 1, positions 0 and W + 1.. stay zero (the left / right padding):
//    tap (a, b) is the transposed read of positions k + b of tap row a — no im2col, no masks.
// LDS layout: 128-B pixel rows with the kouter_swz<64> chunk swizzle by slot position (conflict-free for the shifted
// reads too). Waits follow the pwwgrad.hip discipline (inline-asm LDS reads / barrier, 8 DMA pieces per thread per
// row always, unneeded ones into a junk area with out-of-range offsets).
// Reference op: the Conv2D weight gradient of the model trainer/task.py:62-71 builds.
#include "gemm_core.h"

namespace dtf {
namespace {

constexpr int C3_SLOT = 72 * 128;  // X row slot: 72 positions x 64 channels bf16
constexpr int C3_NS = 8;           // X row slots (at most 8 in use: 4 output rows, one image boundary)
constexpr int C3_DY = 64 * 128;    // dY row image
constexpr int C3_NB = 4;           // dY ring (three rows in flight)
constexpr int C3_JUNK = 8192;
constexpr int C3_SMEM = C3_NS * C3_SLOT + C3_NB * C3_DY + C3_JUNK;
constexpr int C3_OUT = 64 * 9 * 64;

struct C3Args {
  const bf16_t* X;   // [N][H][W][64]
  const bf16_t* dY;  // [N][H][W][64]
  float* ws;         // [grid][64][3][3][64]
  int H, W;
  long rows;         // N * H output rows
  int rpb;
};

__device__ __forceinline__ v8bf c3_tr_pair(uint32_t a0, uint32_t a1) {
  v4s r0, r1;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r0) : "v"(a0));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r1) : "v"(a1));
  v8s both = __builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(v8bf, both);
}
// transposed fragment of a [pos][64] image: channels cb..cb+15, positions shift + (k-step ks's pixel slots)
__device__ __forceinline__ v8bf c3_frag(const char* img, int cb, int shift, int ks, int lane) {
  const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  uint32_t ad[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int pos = 32 * ks + 8 * G + 4 * h + q + shift;
    const int g = ((cb >> 2) + p) ^ (kouter_swz<64>(pos) << 2);
    ad[h] = (uint32_t)(uintptr_t)LDS_PTR(char, img + pos * 128 + g * 8);
  }
  return c3_tr_pair(ad[0], ad[1]);
}

__global__ void __launch_bounds__(256, 1) c3_wgrad_kernel(C3Args a) {
  __shared__ __attribute__((aligned(16))) char smem[C3_SMEM];
  char* xs = smem;
  char* dyi = smem + C3_NS * C3_SLOT;
  char* junk = dyi + C3_NB * C3_DY;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;

  // positions 0 and 65..71 of every X slot: never DMA'd (left padding, right of the widest row)
  for (int e = t; e < C3_NS * 64; e += 256) {
    const int s = e >> 6, r = e & 63;  // 64 16-B pieces per slot: position 0 (8) + positions 65..71 (56)
    const int off = r < 8 ? r * 16 : 65 * 128 + (r - 8) * 16;
    *reinterpret_cast<uint4*>(xs + s * C3_SLOT + off) = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();

  const long r0 = (long)blockIdx.x * a.rpb;
  const long r1 = r0 + a.rpb < a.rows ? r0 + a.rpb : a.rows;
  const int n_mine = r0 < r1 ? (int)(r1 - r0) : 0;
  const int VH = a.H + 2;  // virtual rows per image (two zero padding rows)

  // loop-invariant DMA state (2 pieces per thread per row image): dY pixel kr, X slot position 1 + kr
  int doff[2], xoff[2];
  bool dok[2], xok[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int pb = i * 4096 + t * 16, kr = pb >> 7, ch = (pb & 127) >> 4;
    doff[i] = kr * 128 + ((ch ^ (kouter_swz<64>(kr) << 1)) << 4);
    dok[i] = kr < a.W;
    xoff[i] = kr * 128 + ((ch ^ (kouter_swz<64>(kr + 1) << 1)) << 4);
    xok[i] = kr < a.W;
  }

  auto issue = [&](int it, int n, int h) {
    const long r = r0 + it;
    const __amdgpu_buffer_rsrc_t ry =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.dY + r * a.W * 64), (short)0, a.W * 128, 0x00020000);
    char* img = dyi + (it % C3_NB) * C3_DY;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ry, (__attribute__((address_space(3))) void*)(img + i * 4096 + wave * 1024),
                                               16, dok[i] ? (uint32_t)doff[i] : 0x80000000u, 0, 0, 0);
    // X rows h-1 .. h+1 (virtual rows h .. h+2): all three at the block's first row and an image's first row
    const int first = (it == 0 || h == 0) ? 0 : 2;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int y = h - 1 + j;
      const bool need = j >= first, real = y >= 0 && y < a.H;
      const int V = n * VH + h + j;
      const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(a.X + (need && real ? ((long)n * a.H + y) * a.W * 64 : 0)), (short)0, a.W * 128, 0x00020000);
      char* dst = need ? xs + (V & (C3_NS - 1)) * C3_SLOT + 128 : junk;
#pragma unroll
      for (int i = 0; i < 2; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rx, (__attribute__((address_space(3))) void*)(dst + i * 4096 + wave * 1024), 16,
            need && real && xok[i] ? (uint32_t)xoff[i] : 0x80000000u, 0, 0, 0);
    }
  };

  int n = (int)(r0 / a.H), h = (int)(r0 % a.H);
  int in = n, ih = h;
  auto next = [&](int& nn, int& hh) {
    if (++hh == a.H) {
      hh = 0;
      ++nn;
    }
  };
#pragma unroll
  for (int i = 0; i < C3_NB - 1; ++i) {
    if (i < n_mine) issue(i, in, ih);
    next(in, ih);
  }

  v4f acc[9][4];
#pragma unroll
  for (int u = 0; u < 9; ++u)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[u][j] = (v4f){0.f, 0.f, 0.f, 0.f};

  for (int it = 0; it < n_mine; ++it) {
    // row `it` landed: after it this thread issued rows it+1, it+2 (8 pieces each, when they exist)
    if (it + 2 < n_mine) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (it + 1 < n_mine) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (it + C3_NB - 1 < n_mine) issue(it + C3_NB - 1, in, ih);
    next(in, ih);
    const char* img = dyi + (it % C3_NB) * C3_DY;
    const char* xr[3];
#pragma unroll
    for (int ta = 0; ta < 3; ++ta) xr[ta] = xs + ((n * VH + h + ta) & (C3_NS - 1)) * C3_SLOT;
    // fragments double-buffered across the row's 2 pixel k-steps: k-step 1's reads land under k-step 0's MFMAs
    v8bf fx[2][9], fy[2][4];
    auto load = [&](int ks, v8bf(&x)[9], v8bf(&y)[4]) {
#pragma unroll
      for (int ta = 0; ta < 3; ++ta)
#pragma unroll
        for (int tb = 0; tb < 3; ++tb) x[ta * 3 + tb] = c3_frag(xr[ta], 16 * wave, tb, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) y[j] = c3_frag(img, 16 * j, 0, ks, lane);
    };
    load(0, fx[0], fy[0]);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int u = 0; u < 9; ++u) asm volatile("" : "+v"(fx[ks][u]));
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(fy[ks][j]));
      if (ks == 0) load(1, fx[1], fy[1]);
      // D[c][k]: src0 = X^T (rows c), src1 = dY (columns k)
#pragma unroll
      for (int u = 0; u < 9; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[u][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fx[ks][u], fy[ks][j], acc[u][j], 0, 0, 0);
    }
    next(n, h);
  }

  // lane: c = 16 wave + 4 (lane >> 4) .. + 3 of out channel k = 16 j + (lane & 15), tap u = 3 a + b  (KRSC)
  float* slab = a.ws + (long)blockIdx.x * C3_OUT;
#pragma unroll
  for (int u = 0; u < 9; ++u)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 16 * j + (lane & 15), c = 16 * wave + 4 * (lane >> 4);
      *reinterpret_cast<float4*>(slab + ((long)k * 9 + u) * 64 + c) =
          make_float4(acc[u][j][0], acc[u][j][1], acc[u][j][2], acc[u][j][3]);
    }
}

}  // namespace

// dW [64][3][3][64] f32 (+= when accumulate) of a 64 -> 64 channel 3x3 / stride 1 / pad 1 conv over X [N][H][W][64]
// with dY [N][H][W][64], W <= 64, on the persistent kernel. ws: >= 256 * 36864 floats. Returns 0, or -1 with nothing
// launched when the shape is not handled.
int c3_wgrad_try(const void* X, const void* dY, float* dW, int N, int H, int W, int accumulate, float* ws,
                 long ws_elems, hipStream_t st) {
  if (((uintptr_t)X & 15) || ((uintptr_t)dY & 15) || !ws || N < 1 || H < 1 || W < 1 || W > 64) return -1;
  if ((long)N * (H + 2) >= (1l << 31)) return -1;
  C3Args a{};
  a.X = (const bf16_t*)X; a.dY = (const bf16_t*)dY; a.ws = ws;
  a.H = H; a.W = W;
  a.rows = (long)N * H;
  int grid = 256;
  while (grid > 8 && (long)grid * C3_OUT > ws_elems) grid /= 2;
  if ((long)grid * C3_OUT > ws_elems) return -1;
  a.rpb = (int)((a.rows + grid - 1) / grid);
  grid = (int)((a.rows + a.rpb - 1) / a.rpb);
  hipLaunchKernelGGL(c3_wgrad_kernel, dim3(grid), dim3(256), 0, st, a);
  if (hipGetLastError() != hipSuccess) return -1;
  dtf_sum_rows(ws, C3_OUT, grid, C3_OUT, dW, accumulate, st);
  return (int)hipGetLastError();
}

}  // namespace dtf
