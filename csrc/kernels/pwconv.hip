// Persistent pointwise-convolution forward for the channel-EXPANDING 1x1 layers (ResNet-50 bottleneck c3 and the
// stride-1 projection: C_in 64..256 -> K_out = 4 C_in), with the BatchNorm statistics of the output.
//
// Why a kernel of its own (tools/bw_probe.py, MI355X): these layers write 4x the bytes they read, and the general
// 128x64 LDS-DMA tile (gemm_core.h) re-runs its whole prologue / epilogue for every 128x64 output tile (25,088
// blocks for stage 1) and leaves one BN partial row per M-tile (6,272 rows for the stage-1 finalize to reduce): it
// streams at 2.4-3.2 TB/s against 6.3 TB/s of write-only bandwidth. Here:
//  * the grid is one 256-wide column tile per block, persistent over M-tiles (one block per CU, XCD-aware: the
//    blocks that share A rows for the N/256 column tiles sit on one XCD), so the block's whole weight slice
//    (64 columns x C_in per wave, <= 128 VGPRs) is loaded into REGISTERS once and never staged again;
//  * only A (the activation tile, BM x C_in) streams through LDS, by LDS-DMA into a 3-deep ring: the next two
//    tiles are in flight while this one is multiplied and stored, counted vmcnt waits (stores are issued
//    unconditionally — rows past M go to an out-of-range buffer offset — so the count is exact);
//  * the epilogue stores bf16 straight from the accumulators and keeps the BN sum / sum-of-squares of the
//    stored (bf16) values in registers across ALL of the block's tiles: one partial row per block (<= 256 rows).
// Reference op: the Conv2D + FusedBatchNorm pair of the model trainer/task.py:62-71 builds.
#include "gemm_core.h"

namespace dtf {
namespace {

typedef int v2i __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));

struct PwArgs {
  const bf16_t* X;  // [M][C] activations
  const bf16_t* W;  // [K][C] filters
  bf16_t* Y;        // [M][K]
  float* stats;     // [nslots][2K] partial rows (sum | sum of squares)
  int M, K;
  int tiles_m, tiles_n, nslots;
};

template <int C, int WMW, bool STG = false>
struct PwGeo {
  static constexpr int NTH = 256 * WMW;        // 4 column waves x WMW row waves
  static constexpr int BM = 64 * WMW;          // rows per tile (64 per row wave)
  static constexpr int NKT = C / 64;           // 64-deep K sub-images per tile
  static constexpr int RPI = NTH / 8;          // rows per DMA wave-instruction set (8 lanes x 16 B = one 128-B row)
  static constexpr int L = BM / RPI;           // DMA instructions per thread per sub-image
  static constexpr int LD = NKT * L;           // DMA instructions per thread per tile
  static constexpr int SUB = BM * 128;         // bytes of one [BM][64] sub-image
  static constexpr int IMG = NKT * SUB;        // bytes of one A tile
  static constexpr int NBUF = 3;
  // stores per thread per tile: 4 row frags x 4 column frags of 8 B, or (STG: the tile staged through LDS) 16-B
  // row-contiguous chunks, BM rows x 32 chunks over NTH threads
  static constexpr int ST = STG ? BM * 32 / NTH : 16;
  static constexpr int SROW = 256 + 8;         // staged row (bf16 elements): 16-B pad
  static constexpr int SMEM = NBUF * IMG + (STG ? BM * SROW * 2 : 0);
};

template <int C, int WMW, bool STG>
__global__ void __launch_bounds__(256 * WMW, 1) pw_conv_kernel(PwArgs a) {
  using G = PwGeo<C, WMW, STG>;
  __shared__ __attribute__((aligned(16))) char smem[G::SMEM];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wn = wave & 3, wm = wave >> 2;
  // block -> (column tile, row slot): the blocks of one row slot (all column tiles) are on one XCD
  const int b = blockIdx.x, xcd = b & 7, j8 = b >> 3;
  const int tile_n = j8 % a.tiles_n;
  const int slot = xcd + 8 * (j8 / a.tiles_n);
  const int n0 = tile_n * 256 + wn * 64;  // this wave's 64 columns

  // ---- the wave's filter slice in registers: fb[j][s] = W rows n0+16j+(lane&15), k = 32s + 8(lane>>4) .. +7
  v8bf fb[4][C / 32];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int s = 0; s < C / 32; ++s)
      fb[j][s] = *reinterpret_cast<const v8bf*>(a.W + (long)(n0 + 16 * j + (lane & 15)) * C + 32 * s +
                                                  8 * (lane >> 4));

  // ---- A tile DMA (lane-linear [BM][64] sub-images, source-side XOR swizzle undone by frag_kcontig)
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.X, (short)0, (int)((long)a.M * C * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t yr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.Y, (short)0, (int)((long)a.M * a.K * 2), 0x00020000);
  auto issue = [&](int mt, int buf) {
    char* img = smem + buf * G::IMG;
#pragma unroll
    for (int i = 0; i < G::L; ++i) {
      const int row = G::RPI * i + (t >> 3);
      const int r = mt * G::BM + row;
      const uint32_t base = r < a.M ? (uint32_t)r * (uint32_t)(C * 2) + (uint32_t)(((t & 7) ^ ((row >> 1) & 7)) * 16)
                                    : 0x80000000u;
#pragma unroll
      for (int kt = 0; kt < G::NKT; ++kt)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            xr, (__attribute__((address_space(3))) void*)(img + kt * G::SUB + i * (G::RPI * 128) + wave * 1024), 16,
            base + kt * 128, 0, 0, 0);
    }
  };

  const int first = slot, step = a.nslots;
  const int n_mine = first < a.tiles_m ? (a.tiles_m - first + step - 1) / step : 0;
  if (n_mine > 0) issue(first, 0);
  if (n_mine > 1) issue(first + step, 1);

  float cs[4][4], cq[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) cs[j][r] = cq[j][r] = 0.f;

  for (int it = 0; it < n_mine; ++it) {
    // tile `it` landed: the ops this thread issued after it are tile it+1's DMA (if any) and tile it-1's stores
    if (it + 1 < n_mine) {
      if (it == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::LD) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::LD + G::ST) : "memory");
    } else {
      if (it == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::ST) : "memory");
    }
    __syncthreads();  // every wave's DMA share landed; every wave is done with the buffer tile it+2 reuses
    if (it + 2 < n_mine) issue(first + (it + 2) * step, (it + 2) % G::NBUF);
    const char* img = smem + (it % G::NBUF) * G::IMG;

    v4f acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < G::NKT; ++kt)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        v8bf fa[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = frag_kcontig(img + kt * G::SUB, wm * 64 + 16 * i, kk, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][2 * kt + kk], fa[i], acc[i][j], 0, 0, 0);
      }

    // ---- epilogue: bf16 stores straight from the accumulators (lane: row (lane&15), 4 consecutive columns), or
    // (STG) through an LDS stage as 16-B row-contiguous chunks; rows past M store to an out-of-range offset (dropped
    // by the range check) so every thread issues ST stores
    const int mt = first + it * step;
    char* stg = smem + G::NBUF * G::IMG;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = mt * G::BM + wm * 64 + 16 * i + (lane & 15);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + 16 * j + 4 * (lane >> 4);
        uint2 o;
        o.x = pack2bf(acc[i][j][0], acc[i][j][1]);
        o.y = pack2bf(acc[i][j][2], acc[i][j][3]);
        if constexpr (STG) {
          const int ml = wm * 64 + 16 * i + (lane & 15), nl = wn * 64 + 16 * j + 4 * (lane >> 4);
          *reinterpret_cast<uint2*>(stg + (ml * G::SROW + nl) * 2) = o;
        } else {
          const uint32_t off = m < a.M ? ((uint32_t)m * (uint32_t)a.K + (uint32_t)n) * 2u : 0x80000000u;
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2i, o), yr, off, 0, 0);
        }
        // statistics of the stored values (rows past M hold exact zeros: they add nothing)
        const float v0 = __uint_as_float(o.x << 16), v1 = __uint_as_float(o.x & 0xffff0000u);
        const float v2 = __uint_as_float(o.y << 16), v3 = __uint_as_float(o.y & 0xffff0000u);
        cs[j][0] += v0; cq[j][0] = fmaf(v0, v0, cq[j][0]);
        cs[j][1] += v1; cq[j][1] = fmaf(v1, v1, cq[j][1]);
        cs[j][2] += v2; cq[j][2] = fmaf(v2, v2, cq[j][2]);
        cs[j][3] += v3; cq[j][3] = fmaf(v3, v3, cq[j][3]);
      }
    }
    if constexpr (STG) {
      __syncthreads();  // the tile is staged (the next tile's staging writes come after the next top barrier)
#pragma unroll
      for (int k = 0; k < G::ST; ++k) {
        const int c = t + k * G::NTH, row = c >> 5, ch = c & 31;
        const int m = mt * G::BM + row;
        const uint4 v = *reinterpret_cast<const uint4*>(stg + (row * G::SROW + ch * 8) * 2);
        const uint32_t off =
            m < a.M ? ((uint32_t)m * (uint32_t)a.K + (uint32_t)(tile_n * 256 + ch * 8)) * 2u : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), yr, off, 0, 0);
      }
    }
  }

  // ---- one partial row per block: the 16 row lanes by DPP, the WMW row waves through LDS (fixed order)
  __syncthreads();  // the ring is free (every wave's last tile is multiplied)
  float* red = reinterpret_cast<float*>(smem);  // [WMW][2][256]
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float s = row16_sum(cs[j][r]), q = row16_sum(cq[j][r]);
      if ((lane & 15) == 0) {
        const int c = wn * 64 + 16 * j + 4 * (lane >> 4) + r;
        red[(wm * 2) * 256 + c] = s;
        red[(wm * 2 + 1) * 256 + c] = q;
      }
    }
  __syncthreads();
  if (t < 256) {
    float s = 0.f, q = 0.f;
#pragma unroll
    for (int w = 0; w < WMW; ++w) { s += red[(w * 2) * 256 + t]; q += red[(w * 2 + 1) * 256 + t]; }
    float* prow = a.stats + (long)slot * 2 * a.K;
    prow[tile_n * 256 + t] = s;
    prow[a.K + tile_n * 256 + t] = q;
  }
}

template <int C, int WMW, bool STG = false>
void launch_pw(const PwArgs& a, int grid, hipStream_t st) {
  hipLaunchKernelGGL((pw_conv_kernel<C, WMW, STG>), dim3(grid), dim3(256 * WMW), 0, st, a);
}

}  // namespace

// Y[M][K] = X[M][C] . W[K][C]^T with the per-column BN statistics of Y as partial rows; C in {64, 128, 256},
// K a multiple of 256 with K/256 in {1, 2, 4, 8}. Returns the number of partial rows written (> 0) or 0 when the
// shape is not handled (the caller uses the general kernel).
int pwconv_try(const void* X, const void* W, void* Y, float* stats, long M, int C, int K, hipStream_t st) {
  if (!(C == 64 || C == 128 || C == 256) || (K % 256) || !stats) return 0;
  const int tiles_n = K / 256;
  if (tiles_n != 1 && tiles_n != 2 && tiles_n != 4 && tiles_n != 8) return 0;
  if (M * C * 2 >= (1l << 31) || M * K * 2 >= (1l << 31)) return 0;
  if (((uintptr_t)X & 15) || ((uintptr_t)W & 15) || ((uintptr_t)Y & 15)) return 0;
  // C 128 / 256: one row wave per block (the 128-VGPR filter slice; for C 128 the 3-deep ring plus the LDS store
  // stage of a 128-row tile would exceed the LDS); C 64: two row waves per block. Every tile is stored through an
  // LDS stage as row-contiguous 16-B chunks. (Measured alternatives, removed: several one-row-wave blocks per CU
  // for C 64, direct fragment stores: profiles/r4_pointwise_conv_bw_probe.txt, r4_negative_results.txt.)
  const int wmw = C == 64 ? 2 : 1;
  const int bm = 64 * wmw;
  PwArgs a{};
  a.X = (const bf16_t*)X; a.W = (const bf16_t*)W; a.Y = (bf16_t*)Y; a.stats = stats;
  a.M = (int)M; a.K = K;
  a.tiles_m = (int)((M + bm - 1) / bm);
  a.tiles_n = tiles_n;
  if (a.tiles_m < 8) return 0;
  // one block per CU (or bpc); fewer when there are fewer tiles (grid stays a multiple of 8 * tiles_n, and the
  // partial rows (one per row slot) never outnumber the M-tiles: the caller's scratch holds ceil(M/64) rows)
  int grid = 256;
  while (grid > 8 * tiles_n && grid / tiles_n > a.tiles_m) grid /= 2;
  a.nslots = grid / tiles_n;
  if (a.nslots > a.tiles_m && a.nslots > 8) return 0;
  if (C == 64) launch_pw<64, 2, true>(a, grid, st);
  else if (C == 128) launch_pw<128, 1, true>(a, grid, st);
  else launch_pw<256, 1, true>(a, grid, st);
  return hipGetLastError() == hipSuccess ? a.nslots : 0;
}


}  // namespace dtf

// Test / tuning entry: the pointwise forward on its own (stats: [nslots][2K] floats, nslots <= ceil(M/64)).
DTF_API int dtf_pwconv_fwd(const void* X, const void* W, void* Y, float* stats, int* rows, long M, int C, int K,
                           void* stream) {
  const int r = dtf::pwconv_try(X, W, Y, stats, M, C, K, (hipStream_t)stream);
  if (rows) *rows = r;
  return r > 0 ? 0 : -1;
}
