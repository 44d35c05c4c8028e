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
#include <cstdlib>

#include "gemm_core.h"

namespace dtf {
namespace {

constexpr int SW_PX = 136;                 // s2d row slot: 128 DMA'd pixels + 8 zero pixels, 32 B each
constexpr int SW_SLOT = SW_PX * 32;
constexpr int SW_NS = 16;                  // s2d row slots
constexpr int SW_DY = 128 * 128;           // dY row image: 128 pixels x 64 channels bf16
constexpr int SW_JUNK = 4096;              // target of the unneeded s2d pieces
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

// NB: dY ring depth (NB - 1 rows in flight)
template <int NB>
__global__ void __launch_bounds__(256, 1) stem_wgrad_kernel(SwArgs a) {
  constexpr int SW_NB = NB;
  __shared__ __attribute__((aligned(16))) char smem[SW_NS * SW_SLOT + NB * SW_DY + SW_JUNK];
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
    // row `it` landed: what this thread issued after it are rows it+1 .. it+NB-2 (8 pieces each, when they exist)
    if (NB >= 5 && it + 3 < n_mine) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else if (NB >= 4 && it + 2 < n_mine) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
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


// ---- fused form: the stem's BatchNorm + ReLU + MaxPool backward applied while building the dY image ----
// dY[n][h][w] = a dz + b yc + c (per channel; bn_bwd_finalize's coefficients), dz = the pooled gradient of the
// 3x3/2 pad-1 windows the pixel won with a positive value (argmax byte, bit 7 = ReLU), summed in
// pool_grad8_2x2's tap order and rounded to bf16: bitwise the dx maxpool_bn_bwd_apply_kernel<true> stores, which
// is therefore never written (1.64 GB) nor re-read (1.64 GB) at batch 1024. The raw inputs of row it+1 (two yc
// pixels and four windows per 8-channel unit) are register-prefetched under the MFMAs of row it; the s2d rows keep
// the LDS-DMA ring (two rows ahead).
struct SwfArgs {
  SwArgs s;
  const bf16_t* yc;     // [N][P][Q][64] BN input (the stem conv output)
  const bf16_t* dyp;    // [N][P2][Q2][64] pooled gradient
  const uint8_t* arg;   // [N][P2][Q2][64] argmax tap | ReLU bit 7
  const float* coef;    // [3][64]
  int P2, Q2;
};

typedef int v4i_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void lds_write16(char* p, uint4 v) {
  const uint32_t ad = (uint32_t)(uintptr_t)LDS_PTR(char, p);
  const v4i_t x = __builtin_bit_cast(v4i_t, v);
  asm volatile("ds_write_b128 %0, %1" ::"v"(ad), "v"(x) : "memory");
}

struct SwWin {
  uint2 a;
  uint4 g;
};
struct SwUnit {
  uint4 x0, x1;
  SwWin w[4];  // windows (i, j), (i, j+1), (i+1, j), (i+1, j+1)
};

__device__ __forceinline__ void swin_add(const SwWin& w, bool valid, uint32_t tap, float* acc) {
  const uint32_t me = tap | 0x80u;
  const uint32_t gw[4] = {w.g.x, w.g.y, w.g.z, w.g.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t bj = ((j < 4 ? w.a.x : w.a.y) >> (8 * (j & 3))) & 0xffu;
    const float g = __uint_as_float((j & 1) ? (gw[j >> 1] & 0xffff0000u) : (gw[j >> 1] << 16));
    if (valid && bj == me) acc[j] += g;
  }
}

// unit u of output row (n, h): 8 channels (cc = u & 7) of pixels 2j, 2j+1 (j = u >> 3)
__device__ __forceinline__ void swf_load(const SwfArgs& f, int n, int h, int u, SwUnit& r) {
  const int j = u >> 3, cc = u & 7, i = h >> 1;
  const long px = ((long)n * f.s.P + h) * f.s.Q + 2 * j;
  r.x0 = *reinterpret_cast<const uint4*>(f.yc + px * 64 + cc * 8);
  r.x1 = *reinterpret_cast<const uint4*>(f.yc + (px + 1) * 64 + cc * 8);
  const bool vj = j + 1 < f.Q2, vi = (h & 1) && i + 1 < f.P2;
  const long o00 = (((long)n * f.P2 + i) * f.Q2 + j) * 64 + cc * 8;
  const long oo[4] = {o00, vj ? o00 + 64 : o00, vi ? o00 + (long)f.Q2 * 64 : o00,
                      vi && vj ? o00 + (long)f.Q2 * 64 + 64 : o00};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    r.w[k].a = *reinterpret_cast<const uint2*>(f.arg + oo[k]);
    r.w[k].g = *reinterpret_cast<const uint4*>(f.dyp + oo[k]);
  }
}

__device__ __forceinline__ void swf_transform(const SwfArgs& f, int h, int u, const SwUnit& r, const float* ka,
                                              const float* kb, const float* kc, char* img) {
  const int j = u >> 3, cc = u & 7, i = h >> 1;
  const bool vj = j + 1 < f.Q2, vi = i + 1 < f.P2;
  float d0[8], d1[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) d0[c] = d1[c] = 0.f;
  if (!(h & 1)) {  // (2i, 2j): w00 tap 4; (2i, 2j+1): w01 tap 3, w00 tap 5
    swin_add(r.w[0], true, 4, d0);
    swin_add(r.w[1], vj, 3, d1);
    swin_add(r.w[0], true, 5, d1);
  } else {  // (2i+1, 2j): w10 tap 1, w00 tap 7; (2i+1, 2j+1): w11 tap 0, w10 tap 2, w01 tap 6, w00 tap 8
    swin_add(r.w[2], vi, 1, d0);
    swin_add(r.w[0], true, 7, d0);
    swin_add(r.w[3], vi && vj, 0, d1);
    swin_add(r.w[2], vi, 2, d1);
    swin_add(r.w[1], vj, 6, d1);
    swin_add(r.w[0], true, 8, d1);
  }
  const uint32_t xa[4] = {r.x0.x, r.x0.y, r.x0.z, r.x0.w}, xb[4] = {r.x1.x, r.x1.y, r.x1.z, r.x1.w};
  float o0[8], o1[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const float x0 = __uint_as_float((c & 1) ? (xa[c >> 1] & 0xffff0000u) : (xa[c >> 1] << 16));
    const float x1 = __uint_as_float((c & 1) ? (xb[c >> 1] & 0xffff0000u) : (xb[c >> 1] << 16));
    o0[c] = fmaf(ka[c], bf2f(f2bf(d0[c])), fmaf(kb[c], x0, kc[c]));
    o1[c] = fmaf(ka[c], bf2f(f2bf(d1[c])), fmaf(kb[c], x1, kc[c]));
  }
  const uint4 v0 = make_uint4(pack2bf(o0[0], o0[1]), pack2bf(o0[2], o0[3]), pack2bf(o0[4], o0[5]),
                              pack2bf(o0[6], o0[7]));
  const uint4 v1 = make_uint4(pack2bf(o1[0], o1[1]), pack2bf(o1[2], o1[3]), pack2bf(o1[4], o1[5]),
                              pack2bf(o1[6], o1[7]));
  const int p0 = 2 * j, p1 = 2 * j + 1;
  lds_write16(img + p0 * 128 + ((cc ^ (kouter_swz<64>(p0) << 1)) << 4), v0);
  lds_write16(img + p1 * 128 + ((cc ^ (kouter_swz<64>(p1) << 1)) << 4), v1);
}

// 10 s2d row slots (9 in use at most: rows it, it+1 and it+2's four at an image boundary) keep the block at 79.5 KB
// of LDS, so two blocks share a CU and one block's dY transform (VALU) runs beside the other's MFMAs
constexpr int SWF_NS = 10;
__global__ void __launch_bounds__(256, 2) stem_wgrad_fused_kernel(SwfArgs f) {
  const SwArgs& a = f.s;
  __shared__ __attribute__((aligned(16))) char smem[SWF_NS * SW_SLOT + 2 * SW_DY + SW_JUNK];
  char* s2d = smem;
  char* dyi = smem + SWF_NS * SW_SLOT;
  char* junk = dyi + 2 * SW_DY;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;

  // zeros that no DMA / transform writes: pixels 128..135 of every s2d slot, pixels Q..127 of both dY images
  {
    const int s = t >> 4, c = t & 15;
    if (s < SWF_NS) *reinterpret_cast<uint4*>(s2d + s * SW_SLOT + 4096 + c * 16) = make_uint4(0, 0, 0, 0);
    for (int e = a.Q * 8 + t; e < 128 * 8; e += 256) {
      *reinterpret_cast<uint4*>(dyi + e * 16) = make_uint4(0, 0, 0, 0);
      *reinterpret_cast<uint4*>(dyi + SW_DY + e * 16) = make_uint4(0, 0, 0, 0);
    }
  }
  __syncthreads();

  const long r0 = (long)blockIdx.x * a.rpb;
  const long r1 = r0 + a.rpb < a.rows ? r0 + a.rpb : a.rows;
  const int n_mine = r0 < r1 ? (int)(r1 - r0) : 0;
  const int units = f.Q2 * 8;
  const int u0 = t, u1 = t + 256 < units ? t + 256 : t;  // (a second unit only where one exists)
  const bool has1 = t + 256 < units, has0 = t < units;
  const int ua = has0 ? u0 : 0, ub = u1 < units ? u1 : 0;
  float ka[8], kb[8], kc[8];
  {
    const int cc = t & 7;  // == (t + 256) & 7
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      ka[c] = f.coef[cc * 8 + c];
      kb[c] = f.coef[64 + cc * 8 + c];
      kc[c] = f.coef[128 + cc * 8 + c];
    }
  }
  const int sx = sw_px(t >> 1);
  const uint32_t soff = sx < a.Ws ? (uint32_t)(sx * 32 + (t & 1) * 16) : 0x80000000u;
  // s2d rows of output row `it` (4 pieces per thread always: unneeded / past-the-end ones go to the junk area)
  auto issue_s2d = [&](int it, int n, int h) {
    const int first = (it == 0 || h == 0) ? 0 : 3;
    const bool live = it < n_mine;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int L = n * a.Hs + h + j;
      const bool need = live && j >= first;
      const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(a.X + (long)(need ? L : 0) * a.Ws * 16), (short)0, a.Ws * 32, 0x00020000);
      char* dst = need ? s2d + (L % SWF_NS) * SW_SLOT : junk;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rx, (__attribute__((address_space(3))) void*)(dst + wave * 1024), 16, need ? soff : 0x80000000u, 0, 0, 0);
    }
  };
  int n = (int)(r0 / a.P), h = (int)(r0 % a.P);  // row it
  int ln = n, lh = h;                               // row it+1 (register loads)
  int in = n, ih = h;                               // row it+2 (s2d DMA)
  auto next = [&](int& nn, int& hh) {
    if (++hh == a.P) {
      hh = 0;
      ++nn;
    }
  };
  SwUnit ra, rb;
  // issue order (kept in every iteration, so the waits are constants): s2d(it), regs(it), s2d(it+1)
  issue_s2d(0, in, ih);
  next(in, ih);
  if (n_mine > 0) {
    swf_load(f, ln, lh, ua, ra);
    swf_load(f, ln, lh, ub, rb);
  }
  next(ln, lh);
  issue_s2d(1, in, ih);
  next(in, ih);

  v4f acc[4][4];
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[b][j] = (v4f){0.f, 0.f, 0.f, 0.f};

  for (int it = 0; it < n_mine; ++it) {
    // everything up to row it's registers landed (after them only row it+1's s2d pieces: 4)
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    char* img = dyi + (it & 1) * SW_DY;
    if (has0) swf_transform(f, h, u0, ra, ka, kb, kc, img);
    if (has1) swf_transform(f, h, u1, rb, ka, kb, kc, img);
    // row it+1's raw inputs (row it's again past the block's range: the count stays constant)
    {
      const bool more = it + 1 < n_mine;
      swf_load(f, more ? ln : n, more ? lh : h, ua, ra);
      swf_load(f, more ? ln : n, more ? lh : h, ub, rb);
    }
    next(ln, lh);
    // this row's dY image and s2d rows are complete for every wave; every wave is done with the image row it+1
    // overwrites and with the s2d slots row it+2 takes
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    issue_s2d(it + 2, in, ih);
    next(in, ih);
    const char* srow = s2d + ((n * a.Hs + h + wave) % SWF_NS) * SW_SLOT;
    // (two waves per SIMD here: the other block's wave covers this one's LDS latency, so one fragment set)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      v8bf fx[4], fy[4];
#pragma unroll
      for (int b = 0; b < 4; ++b) fx[b] = s2d_frag(srow, b, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fy[j] = dy_frag(img, 16 * j, ks, lane);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int b = 0; b < 4; ++b) asm volatile("" : "+v"(fx[b]));
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(fy[j]));
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[b][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fx[b], fy[j], acc[b][j], 0, 0, 0);
    }
    next(n, h);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

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
// producing dY [N][Hs-3][Ws-3][64]. ws: >= 512 * 16384 floats. Returns 0, or -1 (nothing launched) when the shape
// is not handled (Ws > 128) or an operand is misaligned.
DTF_API int dtf_stem_wgrad(const void* X, const void* dY, float* dW, int N, int Hs, int Ws, int accumulate,
                           float* ws, long ws_elems, void* stream) {
  using namespace dtf;
  if (((uintptr_t)X & 15) || ((uintptr_t)dY & 15) || !ws || N < 1 || Hs < 4 || Ws < 4 || Ws > 128) return -1;
  SwArgs a{};
  a.X = (const bf16_t*)X; a.dY = (const bf16_t*)dY; a.ws = ws;
  a.Hs = Hs; a.Ws = Ws; a.P = Hs - 3; a.Q = Ws - 3;
  a.rows = (long)N * a.P;
  int grid = 512;  // (the fused form's partition: both forms sum the same partials)
  while (grid > 8 && (long)grid * SW_OUT > ws_elems) grid /= 2;
  if ((long)grid * SW_OUT > ws_elems) return -1;
  a.rpb = (int)((a.rows + grid - 1) / grid);
  grid = (int)((a.rows + a.rpb - 1) / a.rpb);
  hipStream_t st = (hipStream_t)stream;
  static const int nb = getenv("DTF_STEM_NB") ? atoi(getenv("DTF_STEM_NB")) : 4;  // ring depth (A/B sweep)
  if (nb == 3) hipLaunchKernelGGL(stem_wgrad_kernel<3>, dim3(grid), dim3(256), 0, st, a);
  else if (nb == 5) hipLaunchKernelGGL(stem_wgrad_kernel<5>, dim3(grid), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(stem_wgrad_kernel<4>, dim3(grid), dim3(256), 0, st, a);
  if (hipGetLastError() != hipSuccess) return -1;
  dtf_sum_rows(ws, SW_OUT, grid, SW_OUT, dW, accumulate, st);
  return (int)hipGetLastError();
}

// Fused form: dW of the stem from its BatchNorm input yc [N][Hs-3][Ws-3][64], the pooled gradient dyp and argmax
// bytes arg [N][(Hs-3)/2][(Ws-3)/2][64] (3x3/2 pad-1 max pool) and the BN-backward coefficients coef [3][64]
// (dtf_maxpool_bn_bwd with dx = null leaves them in work[0, 192)): the stem's dY is formed per row in LDS, never
// stored. Returns -1 (nothing launched) when the shape is not handled.
DTF_API int dtf_stem_wgrad_fused(const void* X, const void* yc, const void* dyp, const void* arg, const float* coef,
                                 float* dW, int N, int Hs, int Ws, int accumulate, float* ws, long ws_elems,
                                 void* stream) {
  using namespace dtf;
  if (((uintptr_t)X & 15) || ((uintptr_t)yc & 15) || ((uintptr_t)dyp & 15) || ((uintptr_t)arg & 7) || !ws ||
      !coef || N < 1 || Hs < 5 || Ws < 5 || Ws > 128 || ((Hs - 3) & 1) || ((Ws - 3) & 1))
    return -1;
  SwfArgs f{};
  SwArgs& a = f.s;
  a.X = (const bf16_t*)X; a.ws = ws;
  a.Hs = Hs; a.Ws = Ws; a.P = Hs - 3; a.Q = Ws - 3;
  a.rows = (long)N * a.P;
  f.yc = (const bf16_t*)yc; f.dyp = (const bf16_t*)dyp; f.arg = (const uint8_t*)arg; f.coef = coef;
  f.P2 = a.P / 2; f.Q2 = a.Q / 2;
  if ((long)N * Hs >= (1l << 31)) return -1;
  int grid = 512;  // two blocks per CU
  while (grid > 8 && (long)grid * SW_OUT > ws_elems) grid /= 2;
  if ((long)grid * SW_OUT > ws_elems) return -1;
  a.rpb = (int)((a.rows + grid - 1) / grid);
  grid = (int)((a.rows + a.rpb - 1) / a.rpb);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(stem_wgrad_fused_kernel, dim3(grid), dim3(256), 0, st, f);
  if (hipGetLastError() != hipSuccess) return -1;
  dtf_sum_rows(ws, SW_OUT, grid, SW_OUT, dW, accumulate, st);
  return (int)hipGetLastError();
}

