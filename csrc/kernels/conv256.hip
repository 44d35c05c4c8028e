// 256-row, 8-wave, triple-buffered LDS-DMA implicit-GEMM kernel for the convolution (and plain GEMM) shapes of
// ResNet-50 on gfx950 — the conv counterpart of gemm256.hip's pipelined structure.
//
// Why a second conv kernel: the 128-row 4-wave kernels of gemm_core.h run one barrier per K-tile with at most
// one tile of LDS-DMA in flight (PIPE 4) or none (PIPE 3), which caps them near the ~0.9 PF ceiling of that
// structure (cdna_hip_programming.md §5, "The step-3 structure's ~900 TF ceiling"); the 3x3 convolutions ran at
// 650-860 TF and their weight gradients at 320-650 TF (profiles/r1_conv_roofline_all_tiles_v13.txt). Here:
//  * BM = 256 rows x BN = 64|128 columns per block, 8 waves as 4 (M) x 2 (N), each wave a 64 x BN/2 tile of
//    v_mfma_f32_16x16x32_bf16 fragments (issued (B, A)-swapped so a lane owns 4 consecutive output columns);
//  * both operands staged straight into LDS by buffer_load ... lds (16 B per lane, no VGPR round trip), THREE
//    stage buffers: tile t+2 is issued while tile t is computed, the only waits are counted s_waitcnt vmcnt(N)
//    (never 0 inside the loop) followed by a raw s_barrier, so two K-tiles of DMA stay in flight across every
//    barrier (the guide's "Pipelining across barriers" rule; __syncthreads() would drain them);
//  * the implicit-GEMM gathers are the tap-uniform forms of gemm_core.h (one filter tap x 64 channels per
//    K-tile: a wave-uniform tap offset plus a per-row base offset and in-image tap mask; masked rows get an
//    out-of-range buffer offset and the range check writes zeros) and the row-mapped K-outer forms of the
//    weight gradient (one pixel decode per lane per K-tile);
//  * the epilogue is gemm_core.h's gemm_epilogue (BN statistics, BN-backward statistics, beta / deferred ReLU
//    mask, row remap of strided dgrad phases, split-K slabs).
// The conv entry points of gemm.hip route eligible layers here (conv256_try); reference op family: the Conv2D /
// Conv2DBackpropInput / Conv2DBackpropFilter work TF's runtime does for the reference's model graph
// (SURVEY §2.4.b K4).
#include "gemm_core.h"

namespace dtf {
namespace {

constexpr int BMC = 256;
constexpr int NSTAGE = 3;

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

__device__ __forceinline__ void dma16(const __amdgpu_buffer_rsrc_t& rsrc, uint32_t off, char* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)lds, 16, off, 0, 0, 0);
}

// ---- K-contiguous operand image [R rows][64 k] (128-B rows, chunk swizzle c ^ ((row >> 1) & 7)) ------------------
// A wave instruction fills 1 KiB = 8 rows lane-linearly; instruction i of wave w covers rows 64 i + 8 w .. + 7;
// each lane fetches the LOGICAL chunk that the swizzle puts at its physical slot.
template <int R, int MODE, int NTH>
struct KcLoad {
  static_assert(MODE == OP_KCONTIG || MODE == OP_IM2COL_T || MODE == OP_DGRAD_T, "K-contiguous modes only");
  static constexpr int RPI = NTH / 8;  // rows per instruction round (8 lanes per 128-B row)
  static constexpr int L = R / RPI;    // instructions per thread per K-tile
  __amdgpu_buffer_rsrc_t rsrc;
  int roff[L];
  uint32_t tmask[L];
  int coff[L];

  __device__ __forceinline__ void init(const GemmArgs& a, const bf16_t* p, long ld, int r0, int Rtot) {
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const ConvGeom& g = a.g;
    uint32_t bytes;
    if constexpr (MODE == OP_KCONTIG) bytes = (uint32_t)((long)Rtot * ld * 2);
    else if constexpr (MODE == OP_IM2COL_T) bytes = (uint32_t)((long)g.N * g.H * g.W * g.C * 2);
    else bytes = (uint32_t)((long)g.N * g.P * g.Q * g.Kout * 2);
    rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int row = RPI * i + 8 * w + (lane >> 3);
      coff[i] = ((lane & 7) ^ ((row >> 1) & 7)) * 16;
      const int r = r0 + row;
      uint32_t m = 0;
      int off = 0;
      if (r < Rtot) {
        if constexpr (MODE == OP_KCONTIG) {
          m = ~0u;
          off = (int)((long)r * ld * 2);
        } else if constexpr (MODE == OP_IM2COL_T) {
          uint32_t n, rem, y, x;
          fdivmod((uint32_t)r, g.dPQ, n, rem);
          fdivmod(rem, g.dQ, y, x);
          const int hb = (int)y * g.sh - g.ph, wb = (int)x * g.sw - g.pw;
          off = (((int)n * g.H + hb) * g.W + wb) * g.C * 2;
          m = tap_mask(g.R, g.S, max(0, -hb), min(g.R - 1, g.H - 1 - hb), max(0, -wb), min(g.S - 1, g.W - 1 - wb),
                       a.g_rowrep);
        } else {
          uint32_t n, rem, y, x;
          fdivmod((uint32_t)r, g.dHW, n, rem);
          fdivmod(rem, g.dW, y, x);
          const int hb = (int)y + g.ph, wb = (int)x + g.pw;
          off = (((int)n * g.P + hb) * g.Q + wb) * g.Kout * 2;
          m = tap_mask(g.R, g.S, max(0, hb - g.P + 1), min(g.R - 1, hb), max(0, wb - g.Q + 1), min(g.S - 1, wb),
                       a.g_rowrep);
        }
      }
      roff[i] = off;
      tmask[i] = m;
    }
  }

  __device__ __forceinline__ void issue(const GemmArgs& a, int k0, int Kend, char* lds) {
    const int w = threadIdx.x >> 6;
    int toff;
    uint32_t tap = 0;
    if constexpr (MODE == OP_KCONTIG) {
      toff = k0 * 2;
    } else {
      const ConvGeom& g = a.g;
      uint32_t c0, kh, kw;
      fdivmod((uint32_t)k0, MODE == OP_IM2COL_T ? g.dC : g.dK, tap, c0);
      fdivmod(tap, g.dS, kh, kw);
      toff = MODE == OP_IM2COL_T ? (((int)kh * g.dh * g.W + (int)kw * g.dw) * g.C + (int)c0) * 2
                                 : ((int)c0 - ((int)kh * g.dh * g.Q + (int)kw * g.dw) * g.Kout) * 2;
    }
#pragma unroll
    for (int i = 0; i < L; ++i) {
      bool ok;
      if constexpr (MODE == OP_KCONTIG) ok = tmask[i] != 0u && k0 + (coff[i] >> 1) < Kend;
      else ok = (tmask[i] >> tap) & 1u;
      dma16(rsrc, ok ? (uint32_t)(roff[i] + toff + coff[i]) : 0x80000000u, lds + i * (NTH * 16) + w * 1024);
    }
  }
};

// ---- K-outer operand image [64 k][R cols] (R*2-B k-rows, read with ds_read_b64_tr_b16) ----------------------------
// OP_KOUTER: plain [K][cols] rows of stride ld; OP_KOUTER_R: dY rows of a weight gradient (k = output pixel,
// stride Kout); OP_WGRADX_R: X gathered at (output pixel k, filter tap of the column).
template <int R, int MODE, int NTH>
struct KoLoad {
  static_assert(MODE == OP_KOUTER || MODE == OP_KOUTER_R || MODE == OP_WGRADX_R, "K-outer modes only");
  static constexpr int ROWB = R * 2;
  static constexpr int L = (64 * ROWB) / (NTH * 16);  // instructions per thread per K-tile
  static_assert(L >= 1, "K-outer image smaller than one instruction round");
  __amdgpu_buffer_rsrc_t rsrc;
  int ldb;
  int kr[L], coff[L], hoff[L], woff[L];
  bool cv[L];

  __device__ __forceinline__ void init(const GemmArgs& a, const bf16_t* ptr, long ld, int r0, int Rtot) {
    const int t = threadIdx.x;
    const ConvGeom& g = a.g;
    const uint32_t bytes = MODE == OP_WGRADX_R ? (uint32_t)((long)g.N * g.H * g.W * g.C * 2)
                           : MODE == OP_KOUTER_R ? (uint32_t)((long)g.N * g.P * g.Q * g.Kout * 2)
                                                 : (uint32_t)((long)a.K * ld * 2);
    ldb = MODE == OP_KOUTER_R ? g.Kout * 2 : (int)(ld * 2);
    rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)ptr, (short)0, (int)bytes, 0x00020000);
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int P = i * (NTH * 16) + t * 16;
      kr[i] = P / ROWB;
      const int c = ((P % ROWB) >> 4) ^ (kouter_swz<R>(kr[i]) << 1);
      const int col = r0 + c * 8;
      cv[i] = col < Rtot;
      hoff[i] = woff[i] = 0;
      if constexpr (MODE == OP_WGRADX_R) {
        uint32_t rs, ci, kh, kw;
        fdivmod((uint32_t)(cv[i] ? col : 0), g.dC, rs, ci);
        fdivmod(rs, g.dS, kh, kw);
        hoff[i] = (int)kh * g.dh - g.ph;
        woff[i] = (int)kw * g.dw - g.pw;
        coff[i] = ((hoff[i] * g.W + woff[i]) * g.C + (int)ci) * 2;
      } else {
        coff[i] = col * 2;
      }
    }
  }

  __device__ __forceinline__ void issue(const GemmArgs& a, int k0, int Kend, char* lds) {
    const ConvGeom& g = a.g;
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int k = k0 + kr[i];
      bool ok = cv[i] && k < Kend;
      int off;
      if constexpr (MODE == OP_WGRADX_R) {
        if (g.R == 1 && g.S == 1 && g.sh == 1 && g.sw == 1 && g.ph == 0 && g.pw == 0) {
          off = k * g.C * 2 + coff[i];
        } else {
          uint32_t n, pq, pp, qq;
          fdivmod((uint32_t)(ok ? k : 0), g.dPQ, n, pq);
          fdivmod(pq, g.dQ, pp, qq);
          const int hb = (int)pp * g.sh, wb = (int)qq * g.sw;
          const int hi = hb + hoff[i], wi = wb + woff[i];
          ok = ok && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
          off = (((int)n * g.H + hb) * g.W + wb) * g.C * 2 + coff[i];
        }
      } else {
        off = k * ldb + coff[i];
      }
      dma16(rsrc, ok ? (uint32_t)off : 0x80000000u, lds + i * (NTH * 16) + w * 1024);
    }
  }
};

template <int R, int MODE, int NTH>
using LoadFor = typename std::conditional<kouter_mode(MODE), KoLoad<R, MODE, NTH>, KcLoad<R, MODE, NTH>>::type;

template <int R, int NTH>
constexpr int loads_per_tile() {
  return (64 * R * 2) / (NTH * 16);  // both image kinds: R x 64 bf16 per K-tile, 16 B per lane per instruction
}

// Wave layout: the largest wave tile (128 x 64) that the block shape allows, since LDS read bandwidth bounds a
// 64 x 64 wave tile (16 KB of fragments per 0.5 MFLOP: the LDS must deliver 128 B/clk/CU at the MFMA rate).
template <int BN, int NW>
struct WaveGeom {
  static constexpr int WN = BN == 64 ? 1 : (NW == 8 ? 4 : 2);
  static constexpr int WM = NW / WN;
};

template <int AM, int BMD, int BN, int NW, int NS>
__global__ void __launch_bounds__(NW * 64, 1) conv256_kernel(GemmArgs a) {
  constexpr int NTH = NW * 64;
  constexpr int WM = WaveGeom<BN, NW>::WM, WN = WaveGeom<BN, NW>::WN;
  constexpr int WTM = BMC / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int A_IMG = BMC * BK * 2, B_IMG = BN * BK * 2, STAGE_B = A_IMG + B_IMG;
  constexpr int G = loads_per_tile<BMC, NTH>() + loads_per_tile<BN, NTH>();  // LDS-DMA instructions per K-tile
  __shared__ __attribute__((aligned(16))) char smem[NS * STAGE_B];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / WN, wn = wave % WN;

  // ---- block -> tile: XCD-aware bijective remap, N-tiles of one M-tile adjacent (they share the A rows) ----
  const int nwg = a.tiles_m * a.tiles_n;
  int bid, z;
  xcd_block(nwg, bid, z);
  const int tile_m = bid / a.tiles_n, tile_n = bid % a.tiles_n;
  const int m0 = tile_m * BMC, n0 = tile_n * BN;
  const int bz = z / a.splitk, sk = z % a.splitk;
  const int kbeg = sk * a.kchunk;
  const int kend = min(a.K, kbeg + a.kchunk);

  LoadFor<BMC, AM, NTH> la;
  LoadFor<BN, BMD, NTH> lb;
  la.init(a, a.A + (long)bz * a.sA, a.lda, m0, a.M);
  lb.init(a, a.B + (long)bz * a.sB, a.ldb, n0, a.N);

  v4f acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};

  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  auto stage = [&](int s) { return smem + s * STAGE_B; };
  auto issue = [&](int t, int s) {
    la.issue(a, kbeg + t * BK, kend, stage(s));
    lb.issue(a, kbeg + t * BK, kend, stage(s) + A_IMG);
  };
  auto compute = [&](const char* cA, const char* cB) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      v8bf fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = frag<BMC, AM>(cA, wm * WTM + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = frag<BN, BMD>(cB, wn * WTN + j * 16, kk, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  };

  if constexpr (NS == 3) {
    // Tiles t+1 and t+2 in flight while t is computed. Before reading tile t every wave retires its own DMAs
    // of tile t (the G instructions of tile t+1 may stay outstanding), then the raw barrier makes everyone's
    // tile t visible AND proves every wave finished reading tile t-1, whose buffer (t+2) % 3 is then restaged.
    if (nk > 0) issue(0, 0);
    if (nk > 1) issue(1, 1);
    int s0 = 0;
    for (int t = 0; t < nk; ++t) {
      if (t + 1 < nk) wait_vm<G>();
      else wait_vm<0>();
      raw_barrier();
      const int s2 = s0 == 0 ? 2 : s0 - 1;  // (t + 2) % 3
      if (t + 2 < nk) issue(t + 2, s2);
      compute(stage(s0), stage(s0) + A_IMG);
      s0 = s0 == 2 ? 0 : s0 + 1;
    }
  } else {
    // Double buffer: tile t+1 is issued right after the barrier that retires tile t (and proves tile t-1's
    // buffer free), so its DMA runs under tile t's MFMAs.
    if (nk > 0) issue(0, 0);
    for (int t = 0; t < nk; ++t) {
      wait_vm<0>();
      raw_barrier();
      if (t + 1 < nk) issue(t + 1, (t + 1) & 1);
      compute(stage(t & 1), stage(t & 1) + A_IMG);
    }
  }
  __syncthreads();  // every wave is done with the stage buffers: the epilogue reuses the LDS
  gemm_epilogue<BMC, BN, WM, WN, NTH, NS * STAGE_B>(a, acc, smem, m0, n0, tile_m, z, bz);
}

// Variants (the tile codes 11-14 of gemm.hip): 0 = BN 128, 4 waves (128x64 wave tiles), 3 stages;
// 1 = BN 256, 8 waves (128x64), 2 stages; 2 = BN 64, 4 waves (64x64), 3 stages; 3 = BN 128, 8 waves (64x64), 3 stages.
template <int AM, int BMD>
void launch_cfg(GemmArgs& a, int cfg, hipStream_t st) {
  const int bn = cfg == 1 ? 256 : cfg == 2 ? 64 : 128;
  a.tiles_m = cdiv(a.M, BMC);
  a.tiles_n = cdiv(a.N, bn);
  dim3 grid(a.tiles_m * a.tiles_n, 1, a.batch * a.splitk);
  switch (cfg) {
    case 1: hipLaunchKernelGGL((conv256_kernel<AM, BMD, 256, 8, 2>), grid, dim3(512), 0, st, a); break;
    case 2: hipLaunchKernelGGL((conv256_kernel<AM, BMD, 64, 4, 3>), grid, dim3(256), 0, st, a); break;
    case 3: hipLaunchKernelGGL((conv256_kernel<AM, BMD, 128, 8, 3>), grid, dim3(512), 0, st, a); break;
    default: hipLaunchKernelGGL((conv256_kernel<AM, BMD, 128, 4, 3>), grid, dim3(256), 0, st, a); break;
  }
}

}  // namespace

bool conv256_on() { return true; }

// Launch C = A . B^T on the 256-row pipelined kernel when the operand modes are supported and the problem is
// large enough to fill the chip with 1-block/CU tiles (at least ~256 blocks). bn: 64 or 128 (0: by N).
// Returns 0 if launched, 1 if not eligible (the caller falls back to gemm_core's kernels).
int conv256_try(GemmArgs& a, int amode, int bmode, int cfg, hipStream_t st, bool force) {
  if ((!conv256_on() && !force) || a.atomic_out) return 1;
  // pointwise convolutions (K-contiguous x K-contiguous) stay on gemm_core.h's LDS-DMA tiles: measured slower here
  // on every ResNet-50 1x1 layer it was eligible for (fwd 49.5 vs 43 us stage-3 c1, 96-101 vs 71-73 us stage-4
  // c1/proj; dgrad 48 vs 41 us stage-3 c3: tools/conv_roofline.py --tiles, r3)
  if (!force && amode == OP_KCONTIG && bmode == OP_KCONTIG) return 1;
  if (cfg < 0) {
    // measured per ResNet-50 layer (profiles/r2_conv256_variants.txt): only the 256x256 8-wave form wins, and
    // only with a long K (>= 16 K-tiles: the 2-stage pipeline needs a main loop to amortise its 1-block/CU
    // prologue and epilogue) and N >= 256 (no half-empty column tiles); everything else stays on gemm_core.h
    if (!force && a.N >= 256 && a.K >= 1024) cfg = 1;
    else if (!force) return 1;
    else cfg = a.N <= 64 ? 2 : a.N >= 256 ? 1 : 0;
  }
  if (cfg < 0 || cfg > 3) return 1;
  const int bn = cfg == 1 ? 256 : cfg == 2 ? 64 : 128;
  const long blocks = (long)cdiv(a.M, BMC) * cdiv(a.N, bn) * a.batch * a.splitk;
  if (blocks < 192 && !force) return 1;
  if (a.kchunk % BK) return 1;
  // byte offsets of every staged operand fit the 31-bit buffer range (the range check supplies zeros)
  auto fits = [](long elems) { return elems * 2 < (1l << 31); };
  const ConvGeom& g = a.g;
  for (int s = 0; s < 2; ++s) {
    const int mode = s ? bmode : amode;
    const long rows = s ? a.N : a.M;
    const long ld = s ? a.ldb : a.lda;
    if (mode == OP_KCONTIG && (!fits(rows * ld) || (ld & 7))) return 1;
    if (mode == OP_KOUTER && (!fits((long)a.K * ld) || (ld & 7) || (rows & 7))) return 1;
    if (mode == OP_IM2COL_T && !fits((long)g.N * g.H * g.W * g.C)) return 1;
    if ((mode == OP_DGRAD_T || mode == OP_KOUTER_R) && !fits((long)g.N * g.P * g.Q * g.Kout)) return 1;
    if (mode == OP_WGRADX_R && !fits((long)g.N * g.H * g.W * g.C)) return 1;
  }
  if (((uintptr_t)a.A & 15) || ((uintptr_t)a.B & 15)) return 1;
#define C256_LAUNCH(AMODE, BMODE)           \
  if (amode == AMODE && bmode == BMODE) { \
    launch_cfg<AMODE, BMODE>(a, cfg, st); \
    return 0;                             \
  }
  C256_LAUNCH(OP_KCONTIG, OP_KCONTIG)
  C256_LAUNCH(OP_IM2COL_T, OP_KCONTIG)
  C256_LAUNCH(OP_DGRAD_T, OP_KCONTIG)
  C256_LAUNCH(OP_WGRADX_R, OP_KOUTER_R)
  C256_LAUNCH(OP_KOUTER, OP_KOUTER_R)
#undef C256_LAUNCH
  return 1;
}

}  // namespace dtf
