// Weight gradient of the ResNet-50 stem, run on its space-to-depth form (ops/conv.py stem_s2d_filter): the 7x7/2
// conv over a 3-channel 224^2 image is a VALID 4x4/1 conv over the [N, 115, 115, 16] s2d image S, so
//   dW[k][a][b][c] = sum over output pixels (n, h, w) of dY[n][h][w][k] * S[n][h + a][w + b][c]   (k < 64, c < 16).
//
// The general wgrad tiles ran this as a 64x64-tile implicit GEMM with split-K slabs at ~445 TF/s effective (0.95 ms
// per ResNet-50 b1024 step, the last kernel of the backward, nothing beside it: profiles/r6_resnet50_steady_kernel_
// stats.txt). Its floor is the dY read (1.64 GB at b1024). Here:
//  * one block per CU, persistent over a contiguous range of output rows (n, h); the whole 64 x 256 filter
//    gradient lives in the accumulators (wave a owns tap row a: 4 taps x 64 k x 16 c = 64 registers per lane), one
//    f32 partial per block is written at the end and dtf_sum_rows adds them in a fixed order (deterministic);
//  * per output row, ONE dY row image (112 -> 128 pixels x 64 channels, zero past Q) and the s2d rows it needs are
//    LDS-DMA'd three rows ahead; s2d rows go into a 16-slot ring indexed by the s2d row's linear index, so
//    consecutive output rows reuse 3 of their 4 input rows (each s2d row leaves HBM once per block);
//  * a tap (a, b) is a pixel shift: the B fragment of tap b is the transposed read of pixels k + b of the wave's s2d
//    row, so no im2col image exists anywhere. s2d row slots are 32-B pixel rows with bit 2 of the pixel index
//    flipped by its bit 3 (the rows k and k + 8 of a transposed read then sit on different banks).
// The LDS reads and the barrier are inline asm with explicit waits (the pwwgrad.hip discipline: hipcc must not drain
// the in-flight DMA before them); every thread issues exactly 8 DMA pieces per row (unneeded s2d rows go to a junk
// area with an out-of-range offset), so the vmcnt of "one row still in flight" is a constant.
// Reference op: the Conv2D weight gradient of the model trainer/task.py:62-71 builds.
#include "gemm_core.h"

namespace dtf {
namespace {

constexpr int SW_PX = 136;                 // s2d row slot: 128 DMA'd pixels + 8 zero pixels, 32 B each
constexpr int SW_SLOT = SW_PX * 32;
constexpr int SW_NS = 16;                  // s2d row slots
constexpr int SW_DY = 128 * 128;           // dY row image: 128 pixels x 64 channels bf16
constexpr int SW_NB = 4;                   // dY ring depth (three rows in flight)
constexpr int SW_JUNK = 4096;              // target of the unneeded s2d pieces
constexpr int SW_SMEM = SW_NS * SW_SLOT + SW_NB * SW_DY + SW_JUNK;
constexpr int SW_OUT = 64 * 16 * 16;       // filter gradient floats

struct SwArgs {
  const bf16_t* X;   // [N][Hs][Ws][16]
  const bf16_t* dY;  // [N][P][Q][64]
  float* ws;         // [grid][64][4][4][16]
  int Hs, Ws, P, Q;
  long rows;         // N * P output rows
  int rpb;           // output rows per block
};

__device__ __forceinline__ int sw_px(int x) { return x ^ ((x >> 1) & 4); }

__device__ __forceinline__ v8bf tr_pair(uint32_t a0, uint32_t a1) {
  v4s r0, r1;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r0) : "v"(a0));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r1) : "v"(a1));
  v8s both = __builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(v8bf, both);
}
// dY^T fragment: out channels cb..cb+15, pixels of k-step ks (frag_kouter's slot order, kouter_swz<64> image)
__device__ __forceinline__ v8bf dy_frag(const char* img, int cb, int ks, int lane) {
  const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  uint32_t ad[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = 32 * ks + 8 * G + 4 * h + q;
    const int g = ((cb >> 2) + p) ^ (kouter_swz<64>(k) << 2);
    ad[h] = (uint32_t)(uintptr_t)LDS_PTR(char, img + k * 128 + g * 8);
  }
  return tr_pair(ad[0], ad[1]);
}
// s2d fragment of tap column b: the 16 channels of pixels k + b (the same pixel slot order as dy_frag)
__device__ __forceinline__ v8bf s2d_frag(const char* srow, int b, int ks, int lane) {
  const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  uint32_t ad[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int x = 32 * ks + 8 * G + 4 * h + q + b;
    ad[h] = (uint32_t)(uintptr_t)LDS_PTR(char, srow + sw_px(x) * 32 + p * 8);
  }
  return tr_pair(ad[0], ad[1]);
}

__global__ void __launch_bounds__(256, 1) stem_wgrad_kernel(SwArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[SW_SMEM];
  char* s2d = smem;
  char* dyi = smem + SW_NS * SW_SLOT;
  char* junk = dyi + SW_NB * SW_DY;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;

  // pixels 128..135 of every s2d slot are read (k + b <= 130) but never DMA'd: zero them once, before any DMA
  {
    const int s = t >> 4, c = t & 15;
    *reinterpret_cast<uint4*>(s2d + s * SW_SLOT + 4096 + c * 16) = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();

  const long r0 = (long)blockIdx.x * a.rpb;
  const long r1 = r0 + a.rpb < a.rows ? r0 + a.rpb : a.rows;
  const int n_mine = r0 < r1 ? (int)(r1 - r0) : 0;

  // loop-invariant per-lane DMA state: dY pieces (pixel kr[i], swizzled 16-B chunk) and the s2d piece (slot pixel
  // t >> 1 holds source pixel sw_px(t >> 1), half t & 1)
  int dkr[4], doff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int pb = i * 4096 + t * 16;
    dkr[i] = pb >> 7;
    const int c = ((pb & 127) >> 4) ^ (kouter_swz<64>(dkr[i]) << 1);
    doff[i] = dkr[i] * 128 + c * 16;
  }
  const int sx = sw_px(t >> 1);
  const uint32_t soff = sx < a.Ws ? (uint32_t)(sx * 32 + (t & 1) * 16) : 0x80000000u;

  // output rows are walked with incremental (n, h) counters: no 64-bit division per row
  auto issue = [&](int it, int n, int h) {
    const long r = r0 + it;
    const __amdgpu_buffer_rsrc_t ry =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.dY + r * a.Q * 64), (short)0, a.Q * 128, 0x00020000);
    char* img = dyi + (it % SW_NB) * SW_DY;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t off = dkr[i] < a.Q ? (uint32_t)doff[i] : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          ry, (__attribute__((address_space(3))) void*)(img + i * 4096 + wave * 1024), 16, off, 0, 0, 0);
    }
    // s2d rows h .. h+3 of image n: all four at the block's first row and at an image's first row, else h + 3
    const int first = (it == 0 || h == 0) ? 0 : 3;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long L = (long)n * a.Hs + h + j;
      const bool need = j >= first;
      const __amdgpu_buffer_rsrc_t rx =
          __builtin_amdgcn_make_buffer_rsrc((void*)(a.X + L * a.Ws * 16), (short)0, a.Ws * 32, 0x00020000);
      char* dst = need ? s2d + (int)(L & (SW_NS - 1)) * SW_SLOT : junk;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rx, (__attribute__((address_space(3))) void*)(dst + wave * 1024), 16, need ? soff : 0x80000000u, 0, 0, 0);
    }
  };

  int n = (int)(r0 / a.P), h = (int)(r0 % a.P);  // row `it` (compute)
  int in = n, ih = h;                               // row `it + 2` (issue)
  auto next = [&](int& nn, int& hh) {
    if (++hh == a.P) {
      hh = 0;
      ++nn;
    }
  };
#pragma unroll
  for (int i = 0; i < SW_NB - 1; ++i) {
    if (i < n_mine) issue(i, in, ih);
    next(in, ih);
  }

  v4f acc[4][4];
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[b][j] = (v4f){0.f, 0.f, 0.f, 0.f};

  for (int it = 0; it < n_mine; ++it) {
    // row `it` landed: what this thread issued after it are rows it+1, it+2 (8 pieces each, when they exist)
    if (it + 2 < n_mine) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (it + 1 < n_mine) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // every wave's pieces landed; every wave is done reading the buffers row it+3 overwrites
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (it + SW_NB - 1 < n_mine) issue(it + SW_NB - 1, in, ih);
    next(in, ih);
    const char* srow = s2d + (int)(((long)n * a.Hs + h + wave) & (SW_NS - 1)) * SW_SLOT;
    const char* img = dyi + (it % SW_NB) * SW_DY;
    // fragments double-buffered across the 4 pixel k-steps: the reads of k-step ks+1 are issued right after
    // k-step ks's reads are waited for, and land under its MFMAs
    v8bf fx[2][4], fy[2][4];
    auto load = [&](int ks, v8bf(&x)[4], v8bf(&y)[4]) {
#pragma unroll
      for (int b = 0; b < 4; ++b) x[b] = s2d_frag(srow, b, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) y[j] = dy_frag(img, 16 * j, ks, lane);
    };
    load(0, fx[0], fy[0]);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      // (the asm reads' results exist only after that wait: tie the k-step's fragments to it)
#pragma unroll
      for (int b = 0; b < 4; ++b) asm volatile("" : "+v"(fx[ks & 1][b]));
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(fy[ks & 1][j]));
      if (ks < 3) load(ks + 1, fx[(ks + 1) & 1], fy[(ks + 1) & 1]);
      // D[c][k]: src0 = s2d^T (rows c), src1 = dY (columns k)
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[b][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fx[ks & 1][b], fy[ks & 1][j], acc[b][j], 0, 0, 0);
    }
    next(n, h);
  }

  // lane: c = 4 (lane >> 4) .. + 3 of out channel k = 16 j + (lane & 15), tap (wave, b)
  float* slab = a.ws + (long)blockIdx.x * SW_OUT;
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 16 * j + (lane & 15), c = 4 * (lane >> 4);
      *reinterpret_cast<float4*>(slab + ((k * 4 + wave) * 4 + b) * 16 + c) =
          make_float4(acc[b][j][0], acc[b][j][1], acc[b][j][2], acc[b][j][3]);
    }
}

}  // namespace
}  // namespace dtf

// dW [64][4][4][16] f32 (accumulated when `accumulate`) of the valid 4x4/1 conv of the s2d image X [N][Hs][Ws][16]
// producing dY [N][Hs-3][Ws-3][64]. ws: >= 256 * 16384 floats. Returns 0, or -1 (nothing launched) when the shape
// is not handled (Ws > 128) or an operand is misaligned.
DTF_API int dtf_stem_wgrad(const void* X, const void* dY, float* dW, int N, int Hs, int Ws, int accumulate,
                           float* ws, long ws_elems, void* stream) {
  using namespace dtf;
  if (((uintptr_t)X & 15) || ((uintptr_t)dY & 15) || !ws || N < 1 || Hs < 4 || Ws < 4 || Ws > 128) return -1;
  SwArgs a{};
  a.X = (const bf16_t*)X; a.dY = (const bf16_t*)dY; a.ws = ws;
  a.Hs = Hs; a.Ws = Ws; a.P = Hs - 3; a.Q = Ws - 3;
  a.rows = (long)N * a.P;
  int grid = 256;
  while (grid > 8 && (long)grid * SW_OUT > ws_elems) grid /= 2;
  if ((long)grid * SW_OUT > ws_elems) return -1;
  a.rpb = (int)((a.rows + grid - 1) / grid);
  grid = (int)((a.rows + a.rpb - 1) / a.rpb);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(stem_wgrad_kernel, dim3(grid), dim3(256), 0, st, a);
  if (hipGetLastError() != hipSuccess) return -1;
  dtf_sum_rows(ws, SW_OUT, grid, SW_OUT, dW, accumulate, st);
  return (int)hipGetLastError();
}
