// Persistent 3x3 convolution forward for the 64-channel layers (ResNet-50 stage-1 c2: 64 -> 64, 3x3, stride 1), with
// the BatchNorm statistics of the output.
//
// With only 64 output channels the general 128x64 tile (gemm_core.h) cannot reach a wave tile that keeps the LDS
// below its 128 B/clk: every 16x16x32 MFMA needs fresh A and B fragments from LDS. Here each of the 4 waves keeps
// the WHOLE filter (64 columns x 576 = 9 taps x 64 channels, 288 VGPRs) in registers for the life of the block, so
// only the activation fragments are read from LDS (64 B/clk per CU at the MFMA rate), and the block is persistent
// over 256-row M-tiles (one block per CU):
//  * A = the implicit im2col tile, one tap per 64-deep K-tile (the tap-uniform gather of gemm_core.h: per-row base
//    offset + in-image tap mask, computed once per M-tile; taps outside the image read zeros via the buffer range
//    check), streamed by LDS-DMA through a 4-slot ring three K-tiles ahead — across M-tile boundaries;
//  * bf16 stores straight from the accumulators at the end of each M-tile, issued unconditionally (rows past M go
//    out of range) so the vmcnt waits are counted exactly; BN sum / sum of squares kept in registers across the
//    block's tiles: one partial row per block.
// Reference op: the ResNet Conv2D + FusedBatchNorm.
#include "gemm_core.h"

namespace dtf {
namespace {

typedef int v2i __attribute__((ext_vector_type(2)));

constexpr int C3_BM = 256;             // rows per M-tile (64 per wave)
constexpr int C3_NTH = 256;
constexpr int C3_L = C3_BM / 32;       // DMA instructions per thread per K-tile (32 rows per wave-instruction set)
constexpr int C3_SLOT = C3_BM * 128;   // one [256][64] K-tile image
constexpr int C3_NBUF = 4;
constexpr int C3_ST = 16;              // stores per thread per M-tile
constexpr int C3_NK = 9;               // K-tiles (taps) per M-tile

struct C3Args {
  const bf16_t* X;  // [N][H][W][64]
  const bf16_t* W;  // [64][3][3][64]
  bf16_t* Y;        // [M][64]
  float* stats;     // [nslots][128]
  ConvGeom g;
  uint64_t rowrep;
  int M, tiles_m, nslots;
};

template <int LD, int ST>
__device__ __forceinline__ void c3_wait(int nd, int ns) {
#define DTF_VMW(D, S)                                                      \
  if (nd == D && ns == S) {                                                \
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D * LD + S * ST) : "memory"); \
    return;                                                                \
  }
  DTF_VMW(0, 0) DTF_VMW(1, 0) DTF_VMW(2, 0) DTF_VMW(0, 1) DTF_VMW(1, 1) DTF_VMW(2, 1)
#undef DTF_VMW
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__global__ void __launch_bounds__(C3_NTH, 1) conv3_c64_kernel(C3Args a) {
  __shared__ __attribute__((aligned(16))) char smem[C3_NBUF * C3_SLOT];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const ConvGeom& g = a.g;

  // ---- the whole filter in registers: fb[j][s] = W row 16j+(lane&15), k = 32s + 8(lane>>4) (k = tap*64 + c)
  v8bf fb[4][2 * C3_NK];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int s = 0; s < 2 * C3_NK; ++s)
      fb[j][s] = *reinterpret_cast<const v8bf*>(a.W + (16 * j + (lane & 15)) * (64 * C3_NK) + 32 * s + 8 * (lane >> 4));

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.X, (short)0, (int)((long)g.N * g.H * g.W * 64 * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t yr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.Y, (short)0, (int)((long)a.M * 64 * 2), 0x00020000);

  const int first = blockIdx.x, mstep = a.nslots;
  const int n_mine = first < a.tiles_m ? (a.tiles_m - first + mstep - 1) / mstep : 0;
  const int total = n_mine * C3_NK;

  // DMA issue state: per-row base offsets and tap masks of the M-tile the issuing K-steps belong to
  const int coff = ((t & 7) ^ ((t >> 4) & 7)) * 16;  // (row >> 1) & 7 == (t >> 4) & 7 for rows 32 i + (t >> 3)
  int roff[C3_L];
  uint32_t tmask[C3_L];
  int dec_tile = -1;
  auto decode = [&](int tl) {
    const int mt = first + tl * mstep;
#pragma unroll
    for (int i = 0; i < C3_L; ++i) {
      const int r = mt * C3_BM + 32 * i + (t >> 3);
      uint32_t m = 0;
      int off = 0;
      if (r < a.M) {
        uint32_t n, rem, y, x;
        fdivmod((uint32_t)r, g.dPQ, n, rem);
        fdivmod(rem, g.dQ, y, x);
        const int hb = (int)y * g.sh - g.ph, wb = (int)x * g.sw - g.pw;
        off = (((int)n * g.H + hb) * g.W + wb) * 64 * 2;
        m = tap_mask(3, 3, max(0, -hb), min(2, g.H - 1 - hb), max(0, -wb), min(2, g.W - 1 - wb), a.rowrep);
      }
      roff[i] = off;
      tmask[i] = m;
    }
    dec_tile = tl;
  };
  auto issue = [&](int s) {
    const int tl = s / C3_NK, kt = s - tl * C3_NK;
    if (tl != dec_tile) decode(tl);
    const int kh = kt / 3, kw = kt - kh * 3;
    const int toff = (kh * g.W + kw) * 64 * 2;
    char* slot = smem + (s % C3_NBUF) * C3_SLOT;
#pragma unroll
    for (int i = 0; i < C3_L; ++i) {
      const uint32_t off = ((tmask[i] >> kt) & 1u) ? (uint32_t)(roff[i] + toff + coff) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          xr, (__attribute__((address_space(3))) void*)(slot + i * 4096 + wave * 1024), 16, off, 0, 0, 0);
    }
  };

  for (int s = 0; s < 3; ++s)
    if (s < total) issue(s);

  float cs[4][4], cq[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) cs[j][r] = cq[j][r] = 0.f;
  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};

  for (int tl = 0; tl < n_mine; ++tl) {
#pragma unroll
    for (int kt = 0; kt < C3_NK; ++kt) {
      const int s = tl * C3_NK + kt;
      {  // ops issued after D(s): [the previous tile's stores, if it ended at s-2 or s-1] D(s+1) ... D(s+2)
        const int nd = (s + 1 < total) + (s + 2 < total);
        const int ns = (kt <= 1 && tl > 0) ? 1 : 0;
        c3_wait<C3_L, C3_ST>(nd, ns);
      }
      __syncthreads();  // every wave's DMA share of K-step s landed; every wave is done with slot (s + 3) % 4
      const char* img = smem + (s % C3_NBUF) * C3_SLOT;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        v8bf fa[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = frag_kcontig(img, wave * 64 + 16 * i, kk, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][2 * kt + kk], fa[i], acc[i][j], 0, 0, 0);
      }
      if (kt == C3_NK - 1) {
        const int mt = first + tl * mstep;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = mt * C3_BM + wave * 64 + 16 * i + (lane & 15);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int n = 16 * j + 4 * (lane >> 4);
            uint2 o;
            o.x = pack2bf(acc[i][j][0], acc[i][j][1]);
            o.y = pack2bf(acc[i][j][2], acc[i][j][3]);
            const uint32_t off = m < a.M ? ((uint32_t)m * 64u + (uint32_t)n) * 2u : 0x80000000u;
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2i, o), yr, off, 0, 0);
            const float v0 = __uint_as_float(o.x << 16), v1 = __uint_as_float(o.x & 0xffff0000u);
            const float v2 = __uint_as_float(o.y << 16), v3 = __uint_as_float(o.y & 0xffff0000u);
            cs[j][0] += v0; cq[j][0] = fmaf(v0, v0, cq[j][0]);
            cs[j][1] += v1; cq[j][1] = fmaf(v1, v1, cq[j][1]);
            cs[j][2] += v2; cq[j][2] = fmaf(v2, v2, cq[j][2]);
            cs[j][3] += v3; cq[j][3] = fmaf(v3, v3, cq[j][3]);
            acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
          }
        }
      }
      if (s + 3 < total) issue(s + 3);
    }
  }

  // ---- one partial row per block (the 4 row waves through LDS, fixed order)
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);  // [4 waves][2][64]
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float sv = row16_sum(cs[j][r]), qv = row16_sum(cq[j][r]);
      if ((lane & 15) == 0) {
        const int c = 16 * j + 4 * (lane >> 4) + r;
        red[wave * 128 + c] = sv;
        red[wave * 128 + 64 + c] = qv;
      }
    }
  __syncthreads();
  if (t < 128) {
    const float v = red[t] + red[128 + t] + red[256 + t] + red[384 + t];
    a.stats[(long)blockIdx.x * 128 + t] = v;  // [0, 64): sum, [64, 128): sum of squares
  }
}

}  // namespace

bool conv3p_on() {
  static const bool on = [] {
    const char* e = getenv("DTF_CONV3P");
    return !(e && e[0] == '0');
  }();
  return on;
}

// 3x3 stride-1 dilation-1 forward conv 64 -> 64 channels with BN statistics (partial rows [rows][128]); returns the
// number of partial rows (> 0) or 0 when the shape is not handled.
int conv3p_try(const void* X, const void* W, void* Y, float* stats, int N, int H, int Wd, int C, int K, int R, int S,
               int P, int Q, int sh, int sw, int ph, int pw, int dh, int dw, hipStream_t st) {
  if (C != 64 || K != 64 || R != 3 || S != 3 || sh != 1 || sw != 1 || dh != 1 || dw != 1 || !stats) return 0;
  const long M = (long)N * P * Q;
  if ((long)N * H * Wd * 64 * 2 >= (1l << 31) || M * 64 * 2 >= (1l << 31)) return 0;
  if (((uintptr_t)X & 15) || ((uintptr_t)W & 15) || ((uintptr_t)Y & 15)) return 0;
  C3Args a{};
  a.X = (const bf16_t*)X; a.W = (const bf16_t*)W; a.Y = (bf16_t*)Y; a.stats = stats;
  ConvGeom& g = a.g;
  g.N = N; g.H = H; g.W = Wd; g.C = C; g.Kout = K; g.R = R; g.S = S; g.P = P; g.Q = Q;
  g.sh = sh; g.sw = sw; g.ph = ph; g.pw = pw; g.dh = dh; g.dw = dw;
  g.dPQ = make_fastdiv(P * Q); g.dQ = make_fastdiv(Q);
  uint64_t rr = 0;
  for (int kh = 0; kh < 3; ++kh) rr |= 1ull << (kh * 3);
  a.rowrep = rr;
  a.M = (int)M;
  a.tiles_m = (int)((M + C3_BM - 1) / C3_BM);
  if (a.tiles_m < 1) return 0;
  const int grid = std::min(256, a.tiles_m);
  a.nslots = grid;
  hipLaunchKernelGGL(conv3_c64_kernel, dim3(grid), dim3(C3_NTH), 0, st, a);
  return hipGetLastError() == hipSuccess ? grid : 0;
}

}  // namespace dtf

DTF_API int dtf_conv3p_fwd(const void* X, const void* W, void* Y, float* stats, int* rows, int N, int H, int Wd,
                           int P, int Q, int ph, int pw, void* stream) {
  const int r = dtf::conv3p_try(X, W, Y, stats, N, H, Wd, 64, 64, 3, 3, P, Q, 1, 1, ph, pw, 1, 1,
                                (hipStream_t)stream);
  if (rows) *rows = r;
  return r > 0 ? 0 : -1;
}
