// Persistent weight gradient of a 1x1 stride-1 convolution: dW[K][C] = sum over pixels p of dY[p][k] X[p][c].
//
// The reduction runs over millions of pixels into a small filter (ResNet-50 stage 1: 64 x 256, 256 x 64). The
// general tiles split the pixel range into f32 slabs of 128x64 / 64x256 output tiles and measured 1.1-1.8 TB/s on
// these layers (c1 1.9 ms, c3 1.1 ms at batch 1024, profiles/r6_resnet50_step_list.txt). Here:
//  * one block per CU, persistent over 64-pixel tiles (row slot s takes tiles s, s + splits, ...); the block's whole
//    output tile (KT x CT, <= 32 K floats) lives in the accumulators for the entire pixel range, so nothing but the
//    operands moves until one f32 partial per block is written at the end;
//  * both operands stream through a 3-deep LDS-DMA ring as K-outer images (the pixel is the reduction index, so
//    the MFMA fragments are read transposed with ds_read_b64_tr_b16, frag_kouter's addressing); the tile two ahead
//    stays in flight under the MFMAs of this one (explicit vmcnt waits; the transposed reads and the barrier are
//    inline asm so the compiler does not drain the DMA before them, as gemm_w4.hip does);
//  * blocks that share a pixel range (output tiles of a filter larger than one block tile) sit on one XCD, whose L2
//    then serves the operand they share.
// The partials ([splits][K][C] f32) are summed in a fixed order by dtf_sum_rows (deterministic, no atomics).
// Reference op: the Conv2D weight gradient of the model trainer/task.py:62-71 builds.
#include "gemm_core.h"

namespace dtf {
namespace {

struct WgArgs {
  const bf16_t* dY;  // [P][K]
  const bf16_t* X;   // [P][C]
  float* ws;         // [splits][K][C] partials
  int P, K, C;
  int tiles_p, tiles_c, n_out, splits;
};

// transposed fragment of a [64 pixel][R] K-outer image: columns cb..cb+15 (lane & 15), pixel substep kk
template <int R>
__device__ __forceinline__ v8bf wg_frag(const char* lds, int cb, int kk, int lane) {
  const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  v4s r[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = 32 * kk + 8 * G + 4 * h + q;
    const int g = ((cb >> 2) + p) ^ (kouter_swz<R>(k) << 2);
    const uint32_t addr = (uint32_t)(uintptr_t)LDS_PTR(char, lds + k * (R * 2) + g * 8);
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r[h]) : "v"(addr));
  }
  v8s both = __builtin_shufflevector(r[0], r[1], 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(v8bf, both);
}

// LDS-DMA of one operand's [64 pixel][R] slice (columns col0 .. col0+R of rows with stride ld elements) into the
// K-outer image: 256 threads x 16 B per wave-instruction set, each lane fetching the logical chunk that the XOR
// swizzle puts at its physical slot (GldsKOuter's mapping); pixels past P read zeros through the range check
template <int R>
struct WgOperand {
  static constexpr int L = R / 32;  // DMA instructions per thread per tile
  __amdgpu_buffer_rsrc_t rsrc;
  int kr[L], coff[L], rowb;

  __device__ __forceinline__ void init(const bf16_t* p, long rows, int ld, int col0) {
    const int t = threadIdx.x;
    rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)(rows * ld * 2), 0x00020000);
    rowb = ld * 2;
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int pb = i * 4096 + t * 16;
      kr[i] = pb / (R * 2);
      const int c = ((pb % (R * 2)) >> 4) ^ (kouter_swz<R>(kr[i]) << 1);
      coff[i] = (col0 + c * 8) * 2;
    }
  }

  __device__ __forceinline__ void issue(int p0, int P, char* lds) {
    const int wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int p = p0 + kr[i];
      const uint32_t off = p < P ? (uint32_t)(p * rowb + coff[i]) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsrc, (__attribute__((address_space(3))) void*)(lds + i * 4096 + wave * 1024), 16, off, 0, 0, 0);
    }
  }
};

// KT x CT output tile per block; WKR waves along k (the rest along c): wave tile (KT/WKR) x (CT*WKR/4)
template <int KT, int CT, int WKR>
__global__ void __launch_bounds__(256, 1) pw_wgrad_kernel(WgArgs a) {
  constexpr int WKC = 4 / WKR;
  constexpr int WK = KT / WKR, WC = CT / WKC;  // wave tile
  constexpr int FK = WK / 16, FC = WC / 16;    // fragments
  constexpr int IMG_Y = 64 * KT * 2, IMG_X = 64 * CT * 2, IMG = IMG_Y + IMG_X, NBUF = 3;
  constexpr int LD = KT / 32 + CT / 32;        // DMA instructions per thread per tile
  static_assert(FK >= 1 && FC >= 1 && FK * FC <= 32, "wave tile");
  __shared__ __attribute__((aligned(16))) char smem[NBUF * IMG];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wk = wave % WKR, wc = wave / WKR;

  // block -> (output tile, pixel slot): the blocks of one slot (every output tile) are on one XCD
  const int b = blockIdx.x, xcd = b & 7, j8 = b >> 3;
  const int o = j8 % a.n_out;
  const int slot = xcd + 8 * (j8 / a.n_out);
  const int k0 = (o / a.tiles_c) * KT, c0 = (o % a.tiles_c) * CT;

  WgOperand<KT> opy;
  WgOperand<CT> opx;
  opy.init(a.dY, a.P, a.K, k0);
  opx.init(a.X, a.P, a.C, c0);
  auto issue = [&](int tile, int buf) {
    char* img = smem + buf * IMG;
    opy.issue(tile * 64, a.P, img);
    opx.issue(tile * 64, a.P, img + IMG_Y);
  };

  const int step = a.splits;
  const int n_mine = slot < a.tiles_p ? (a.tiles_p - slot + step - 1) / step : 0;
  if (n_mine > 0) issue(slot, 0);
  if (n_mine > 1) issue(slot + step, 1);

  v4f acc[FC][FK];
#pragma unroll
  for (int i = 0; i < FC; ++i)
#pragma unroll
    for (int j = 0; j < FK; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};

  for (int it = 0; it < n_mine; ++it) {
    // tile `it` landed: the ops this thread issued after it are tile it+1's DMA (if any)
    if (it + 1 < n_mine) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LD) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // every wave's share landed; every wave is done with the buffer tile it+2 reuses (its reads were waited for
    // before the MFMAs that consumed them)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (it + 2 < n_mine) issue(slot + (it + 2) * step, (it + 2) % NBUF);
    const char* img = smem + (it % NBUF) * IMG;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      v8bf fx[FC], fy[FK];
#pragma unroll
      for (int i = 0; i < FC; ++i) fx[i] = wg_frag<CT>(img + IMG_Y, wc * WC + 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < FK; ++j) fy[j] = wg_frag<KT>(img, wk * WK + 16 * j, kk, lane);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      // (the asm reads' results exist only after that wait: tie every fragment to it)
#pragma unroll
      for (int i = 0; i < FC; ++i) asm volatile("" : "+v"(fx[i]));
#pragma unroll
      for (int j = 0; j < FK; ++j) asm volatile("" : "+v"(fy[j]));
      // D[c][k] (lane: 4 consecutive c of one k): src0 X^T rows = c, src1 dY columns = k
#pragma unroll
      for (int i = 0; i < FC; ++i)
#pragma unroll
        for (int j = 0; j < FK; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fx[i], fy[j], acc[i][j], 0, 0, 0);
    }
  }

  // one f32 partial of the output tile per block: lane holds c = cb + 4 (lane >> 4) + r of row k = kb + (lane & 15)
  float* slab = a.ws + (long)slot * a.K * a.C;
#pragma unroll
  for (int i = 0; i < FC; ++i)
#pragma unroll
    for (int j = 0; j < FK; ++j) {
      const int k = k0 + wk * WK + 16 * j + (lane & 15);
      const int c = c0 + wc * WC + 16 * i + 4 * (lane >> 4);
      *reinterpret_cast<float4*>(slab + (long)k * a.C + c) =
          make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
}

template <int KT, int CT, int WKR>
void launch_wg(const WgArgs& a, int grid, hipStream_t st) {
  hipLaunchKernelGGL((pw_wgrad_kernel<KT, CT, WKR>), dim3(grid), dim3(256), 0, st, a);
}

}  // namespace

// dW (f32 [K][C], accumulated when `accumulate`) of a 1x1 stride-1 conv over P pixels on the persistent kernel.
// Filters handled: K, C in {64, 128, 256} with K * C <= 32 K floats (one output tile per block); with split_out
// also 128 x 512 / 512 x 128 as two tiles (the operand a tile does not own is re-read once per tile: measured slower
// than the general 128x128 tiles on ResNet-50 stage 2, 6.3 vs 6.0 ms per step, so the router does not ask for it). ws: >= splits * K * C floats (splits <= 256). Returns 0,
// or -1 when the shape is not handled (nothing launched).
int pw_wgrad_try(const void* X, const void* dY, float* dW, long P, int C, int K, int accumulate, float* ws,
                 long ws_elems, hipStream_t st, bool split_out) {
  if (((uintptr_t)X & 15) || ((uintptr_t)dY & 15) || !ws) return -1;
  if (P * K * 2 >= (1l << 31) || P * C * 2 >= (1l << 31) || P < 64 * 8) return -1;
  int KT = 0, CT = 0;
  if ((long)K * C <= 32768 && (K == 64 || K == 128 || K == 256) && (C == 64 || C == 128 || C == 256)) {
    KT = K; CT = C;
  } else if (split_out && K == 128 && C == 512) {
    KT = 128; CT = 256;
  } else if (split_out && K == 512 && C == 128) {
    KT = 256; CT = 128;
  } else {
    return -1;
  }
  WgArgs a{};
  a.dY = (const bf16_t*)dY; a.X = (const bf16_t*)X; a.ws = ws;
  a.P = (int)P; a.K = K; a.C = C;
  a.tiles_p = (int)((P + 63) / 64);
  a.tiles_c = C / CT;
  a.n_out = (K / KT) * a.tiles_c;
  const long mn = (long)K * C;
  // one block per CU: 256 / n_out pixel slots (a multiple of 8), fewer when the workspace is short
  int splits = 256 / a.n_out;
  while (splits > 8 && (long)splits * mn > ws_elems) splits /= 2;
  if ((long)splits * mn > ws_elems || splits > a.tiles_p) return -1;
  a.splits = splits;
  const int grid = splits * a.n_out;
  const int key = KT * 1000 + CT;
  switch (key) {
    case 64064: launch_wg<64, 64, 2>(a, grid, st); break;
    case 64128: launch_wg<64, 128, 1>(a, grid, st); break;
    case 64256: launch_wg<64, 256, 1>(a, grid, st); break;
    case 128064: launch_wg<128, 64, 2>(a, grid, st); break;
    case 128128: launch_wg<128, 128, 2>(a, grid, st); break;
    case 128256: launch_wg<128, 256, 2>(a, grid, st); break;
    case 256064: launch_wg<256, 64, 4>(a, grid, st); break;
    case 256128: launch_wg<256, 128, 2>(a, grid, st); break;
    default: return -1;
  }
  if (hipGetLastError() != hipSuccess) return -1;
  dtf_sum_rows(ws, mn, splits, mn, dW, accumulate, st);
  return (int)hipGetLastError();
}

}  // namespace dtf
