// Shared pieces of the 4-wave 256-row GEMM kernels (gemm_w4.hip: bf16; gemm_w4_fp8.hip: fp8 on the block-scaled
// MFMA): the pinned barrier / LDS-wait helpers and the loop-invariant LDS-DMA operand loader.
#pragma once
#include <type_traits>

#include "gemm_core.h"

namespace dtf {
namespace {

constexpr int W4_THREADS = 256;
constexpr int W4_A = 256 * BK * 2;  // A image of one stage: 256 rows x 128 bytes (64 bf16 / 128 fp8 k) = 32 KiB

// raw s_barrier pinned in the schedule: register-only MFMAs may not move across it (an inline-asm wait alone does
// not order them: cdna_hip_programming.md §5.4 rule 18)
__device__ __forceinline__ void w4_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// pad for the first VALU read of an accumulator after the last inline-asm MFMA (hipcc inserts no hazard padding
// after inline asm)
__device__ __forceinline__ void w4_mfma_drain() {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
}

// wait for this wave's outstanding LDS reads (inline-asm reads hipcc does not track), pinned in the schedule
__device__ __forceinline__ void w4_lgkm0() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// Staged bf16 rows -> C for a full tile with nothing to combine (no beta, no activation backward): the LDS reads of
// 8 rows go out back to back, then their 16-B stores, so neither waits on the other row by row (the general loop's
// beta / dact branches made hipcc wait lgkmcnt(0) before every single store).
template <int BN, int ROWS>
__device__ __forceinline__ void w4_store_rows(const bf16_t* ct, bf16_t* c, long ldc, int r0, int c8) {
  constexpr int CS = BN + 8, RPP = W4_THREADS / (BN / 8), IT = ROWS / RPP, U = IT < 8 ? IT : 8;
#pragma unroll
  for (int i0 = 0; i0 < IT; i0 += U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const uint4*>(ct + (r0 + RPP * (i0 + u)) * CS + c8 * 8);
#pragma unroll
    for (int u = 0; u < U; ++u) *reinterpret_cast<uint4*>(c + (long)(r0 + RPP * (i0 + u)) * ldc) = v[u];
    __builtin_amdgcn_sched_group_barrier(0x100, U, 0);  // the U LDS reads first,
    __builtin_amdgcn_sched_group_barrier(0x040, U, 0);  // then the U global stores
  }
}

// LDS-DMA loader of one R-row (K-contiguous: [R rows][64 k]) or R-column (K-outer: [64 k][R cols]) operand image
// per K-tile, R/32 wave instructions per thread, in the lane-linear layouts frag_kcontig / frag_kouter<R> read (the
// XOR swizzle is applied on the source side, as gemm_core.h GldsLoader / GldsKOuter). Everything per-lane is
// loop-invariant: the k position of a tile goes into the instruction's SGPR offset and the LDS destination is a
// scalar (M0). Rows / columns past the operand get an out-of-range VGPR offset and read zeros. Every issued tile is
// a real one (the caller clamps the tile index), so in-range rows never read past their own row.
template <int R, int MODE>
struct W4Loader {
  static_assert(MODE == OP_KCONTIG || MODE == OP_KOUTER, "plain operands only");
  static constexpr int L = R / 32;
  __amdgpu_buffer_rsrc_t rsrc;
  int voff[L];
  int kstep;  // bytes per unit of k in the global operand: 2 (K-contiguous) or 2 * ld (K-outer)

  __device__ __forceinline__ void init(const GemmArgs& a, const bf16_t* p, long ld, int r0, int Rtot, int t) {
    const uint32_t bytes = MODE == OP_KCONTIG ? (uint32_t)((long)Rtot * ld * 2) : (uint32_t)((long)a.K * ld * 2);
    rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
    kstep = MODE == OP_KCONTIG ? 2 : (int)(ld * 2);
#pragma unroll
    for (int i = 0; i < L; ++i) {
      if constexpr (MODE == OP_KCONTIG) {
        const int row = 32 * i + (t >> 3);
        const int c = (t & 7) ^ ((row >> 1) & 7);
        voff[i] = r0 + row < Rtot ? (int)((long)(r0 + row) * ld * 2) + c * 16 : (int)0x80000000;
      } else {
        const int P = i * 4096 + t * 16;
        const int kr = P / (2 * R);
        const int c = ((P % (2 * R)) >> 4) ^ (kouter_swz<R>(kr) << 1);
        const int col = r0 + c * 8;
        voff[i] = col < Rtot ? (int)((long)kr * ld * 2) + col * 2 : (int)0x80000000;
      }
    }
  }
  // piece i of the K-tile starting at k0 into the stage image at LDS byte address lds (wave-uniform)
  __device__ __forceinline__ void issue1(int k0, uint32_t lds, int i) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)(uintptr_t)(lds + i * 4096),
                                             16, (uint32_t)voff[i], k0 * kstep, 0, 0);
  }
};

// Implicit-GEMM A operand for the 4-wave kernels. OP_IM2COL_T (convolution forward): row r = output pixel (n, p, q),
// k = (tap, input channel), C % 64 == 0. OP_DGRAD_T (stride-1 data gradient): row r = input pixel (n, h, w), k = (tap,
// output channel) gathered from dY, Kout % 64 == 0. Either way a 64-deep K-tile is ONE filter tap x 64 channels. Per
// lane and piece: the row's base offset and its in-image tap mask (loop-invariant); per K-tile: the tap's wave-uniform
// offset, and rows whose tap falls outside the image get an out-of-range offset (the buffer range check supplies
// zeros). Same LDS image and piece layout as W4Loader<R, OP_KCONTIG>.
template <int R, int MODE>
struct W4Gather {
  static_assert(MODE == OP_IM2COL_T || MODE == OP_DGRAD_T, "gathered operands only");
  static constexpr int L = R / 32;
  __amdgpu_buffer_rsrc_t rsrc;
  int roff[L];
  uint32_t tmask[L];
  FastDiv dCh, dS;  // (copies: the per-K-tile tap decode stays in scalar registers, no loads of the arguments)
  int tsh, tsw;     // byte offsets of one filter row / column step in the gathered tensor

  __device__ __forceinline__ void init(const GemmArgs& a, const bf16_t* p, long, int r0, int Rtot, int t) {
    const ConvGeom& g = a.g;
    dS = g.dS;
    if constexpr (MODE == OP_IM2COL_T) {
      dCh = g.dC;
      tsh = g.dh * g.W * g.C * 2;
      tsw = g.dw * g.C * 2;
      rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)((long)g.N * g.H * g.W * g.C * 2), 0x00020000);
    } else {
      dCh = g.dK;
      tsh = -(g.dh * g.Q * g.Kout * 2);
      tsw = -(g.dw * g.Kout * 2);
      rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)((long)g.N * g.P * g.Q * g.Kout * 2),
                                               0x00020000);
    }
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int row = 32 * i + (t >> 3);
      const int c = (t & 7) ^ ((row >> 1) & 7);
      const int r = r0 + row;
      uint32_t m = 0u;
      int off = 0;
      if (r < Rtot) {
        uint32_t n, rem, y, x;
        if constexpr (MODE == OP_IM2COL_T) {
          fdivmod((uint32_t)r, g.dPQ, n, rem);
          fdivmod(rem, g.dQ, y, x);
          const int hb = (int)y * g.sh - g.ph, wb = (int)x * g.sw - g.pw;
          off = (((int)n * g.H + hb) * g.W + wb) * g.C * 2;
          m = tap_mask(g.R, g.S, max(0, -hb), min(g.R - 1, g.H - 1 - hb), max(0, -wb), min(g.S - 1, g.W - 1 - wb),
                       a.g_rowrep);
        } else {
          fdivmod((uint32_t)r, g.dHW, n, rem);
          fdivmod(rem, g.dW, y, x);
          const int hb = (int)y + g.ph, wb = (int)x + g.pw;
          off = (((int)n * g.P + hb) * g.Q + wb) * g.Kout * 2;
          m = tap_mask(g.R, g.S, max(0, hb - g.P + 1), min(g.R - 1, hb), max(0, wb - g.Q + 1), min(g.S - 1, wb),
                       a.g_rowrep);
        }
      }
      roff[i] = off + c * 16;
      tmask[i] = m;
    }
  }
  __device__ __forceinline__ void issue1(int k0, uint32_t lds, int i) {
    uint32_t tap, c0, kh, kw;
    fdivmod((uint32_t)k0, dCh, tap, c0);
    fdivmod(tap, dS, kh, kw);
    const int toff = (int)kh * tsh + (int)kw * tsw + (int)c0 * 2;
    const uint32_t off = ((tmask[i] >> tap) & 1u) ? (uint32_t)(roff[i] + toff) : 0x80000000u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)(uintptr_t)(lds + i * 4096),
                                             16, off, 0, 0, 0);
  }
};

template <int R, int MODE>
using W4LoaderFor = typename std::conditional<MODE == OP_IM2COL_T || MODE == OP_DGRAD_T, W4Gather<R, MODE>,
                                              W4Loader<R, MODE>>::type;

}  // namespace
}  // namespace dtf
