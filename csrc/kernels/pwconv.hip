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
// Two-pass ConvBN forward (MODE 1 then MODE 2, dtf_conv_bn_apply_fwd): the layer writes 4x the bytes it reads, so
// recomputing the product is cheaper than storing it and reading it back for the BatchNorm apply. MODE 1 keeps only
// the statistics (no stores); after the finalize, MODE 2 recomputes the same tiles (bitwise the same bf16 values:
// same MFMA sequence) and its epilogue applies the BatchNorm, adds the residual (optionally itself a deferred
// BatchNorm: res * rscale + rshift), applies the ReLU and stores the block output with its 1-bit ReLU mask (and the
// conv output yc only when the backward still needs it) — the standalone apply pass (read yc + res, write out) and
// the yc write/read disappear (ResNet-50 bottleneck c3: 17 -> 14 activation-widths of traffic, 10 without yc).
// Reference op: the Conv2D + FusedBatchNorm pair of the model trainer/task.py:62-71 builds.
#include "gemm_core.h"

namespace dtf {
namespace {

typedef int v2i __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));

struct PwArgs {
  const bf16_t* X;  // [M][C] activations
  const bf16_t* W;  // [K][C] filters
  bf16_t* Y;        // [M][K] (MODE 2: optional conv output)
  float* stats;     // [nslots][2K] partial rows (sum | sum of squares)
  int M, K;
  int tiles_m, tiles_n, nslots;
  // MODE 2 (BatchNorm apply epilogue): out = [relu](yc * scale + shift [+ res | + res * rscale + rshift])
  const float* scale;
  const float* shift;
  const bf16_t* res;
  const float* rscale;
  const float* rshift;
  bf16_t* out;
  uint8_t* mbits;  // 1-bit ReLU mask of out (relu only)
  int relu;
  // MODE 3 (the data gradient of a channel-REDUCING 1x1 conv, X = dY [M][C], W = its filter as [K][C], Y = dX):
  // Y = bf16(X W^T) (+ beta * cin, the old values zeroed where betamask's bit is clear: the residual gradient parked
  // for this conv, gemm_core.h's staged beta path operation for operation); with bnmean the BatchNorm-backward
  // partial rows of the stored values: [slot][0, K) sum dz, [K, 2K) sum dz * (bnx - bnmean), dz = value * bnmask bit
  const bf16_t* cin;
  const uint8_t* betamask;
  float beta;
  const bf16_t* bnx;
  const uint8_t* bnmask;
  const float* bnmean;
  // MODE 3 with bW > 0: cin is the compact [N][bH/2][bW/2][K] data gradient of a stride-2 1x1 projection of the same
  // input, added at the even pixels of the [N][bH][bW] grid only (beta 1, no mask)
  int bH, bW;
  // MODE 3, RX: the BN input bnx is not stored — it is the bf16 output of a 64-channel-input 1x1 conv, recomputed per
  // tile as bf16(rx rw^T) (rx [M][64], rw [K][64]) with that forward's MFMA sequence (bitwise its values)
  const bf16_t* rx;
  const bf16_t* rw;
};

template <int C, int WMW, bool STG = false, int MODE = 0>
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
  // vector-memory ops per thread per tile after the DMA: MODE 0 the stores, MODE 1 none, MODE 2 the out (+ yc)
  // stores and the mask bytes (counted for the vmcnt waits; the yc stores only when requested: see SW)
  static constexpr int STM = MODE == 1 ? 0 : ST;
};

// One 8-B fragment into the LDS store stage. Inline asm on purpose: the compiler cannot tell the stage from the DMA
// ring (LDS-DMA writes carry no alias information), so before a plain LDS store it waits for EVERY outstanding
// vector-memory op — draining the DMA of the tile two ahead before each epilogue and leaving one tile of prefetch.
// The stage never overlaps the ring; tile_barrier() waits for these writes before it publishes the tile.
__device__ __forceinline__ void stage_write(char* p, uint2 v) {
  const uint32_t addr = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)p;
  asm volatile("ds_write_b64 %0, %1" ::"v"(addr), "v"(v) : "memory");
}

// Workgroup barrier for the tile loop: this thread's LDS ops done, then s_barrier, as one asm statement (a compiler
// memory barrier too). __syncthreads()' fence makes the compiler drain every outstanding vector-memory op first (it
// counts the in-flight LDS-DMA of the next tiles as pending LDS writes); the loop orders its DMA with explicit vmcnt
// waits instead.
__device__ __forceinline__ void tile_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// N 16-B chunks of the LDS store stage (byte offsets off[i] from base), by inline asm for the same reason as
// stage_write: a plain LDS load here makes hipcc drain the DMA of the tile two ahead ("s_waitcnt vmcnt(0)") before the
// store pass of every tile. One wait for all N reads; each result is tied to it.
template <int N>
__device__ __forceinline__ void stage_read(uint4 (&v)[N], const char* base, const int (&off)[N]) {
  v4i r[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint32_t addr = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)(base + off[i]);
    asm volatile("ds_read_b128 %0, %1" : "=v"(r[i]) : "v"(addr));
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < N; ++i) {
    asm volatile("" : "+v"(r[i]));
    v[i] = __builtin_bit_cast(uint4, r[i]);
  }
}

template <int C, int WMW, bool STG, int MODE, bool RX = false>
__global__ void __launch_bounds__(256 * WMW, 1) pw_conv_kernel(PwArgs a) {
  static_assert(MODE < 2 || STG, "the apply / data-gradient epilogues work on the LDS-staged tile");
  static_assert(!RX || (MODE == 3 && WMW == 1), "bnx recompute: the data-gradient mode, one row wave");
  using G = PwGeo<C, WMW, STG, MODE>;
  constexpr int RIMG = G::BM * 128;                 // RX: one [BM][64] rx sub-image
  constexpr int LRX = RX ? G::BM / G::RPI : 0;      // RX: its DMA instructions per thread per tile
  constexpr int LDT = G::LD + LRX;                  // DMA instructions per thread per tile
  constexpr int YROW = 256 + 8;                     // RX: staged y row (bf16), 16-B pad
  __shared__ __attribute__((aligned(16))) char smem[G::SMEM + (RX ? 3 * RIMG + G::BM * YROW * 2 : 0)];
  char* rximg = smem + G::SMEM;
  char* ystg = rximg + 3 * RIMG;
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

  // RX: the recompute operands — the wave's rw slice in registers (rows n0 + 16 j + (lane & 15)), rx tiles by DMA
  v8bf fr[RX ? 4 : 1][2];
  const __amdgpu_buffer_rsrc_t rxr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.rx, (short)0, RX ? (int)((long)a.M * 128) : 0, 0x00020000);
  if constexpr (RX) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        fr[j][kk] = *reinterpret_cast<const v8bf*>(a.rw + (long)(n0 + 16 * j + (lane & 15)) * 64 + 32 * kk +
                                                   8 * (lane >> 4));
#pragma unroll
    for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(fr[j][0]), "v"(fr[j][1]));  // (waited for before any DMA)
  }
  auto issue_rx = [&](int mt, int buf) {
    if constexpr (RX) {
      char* img = rximg + buf * RIMG;
#pragma unroll
      for (int i = 0; i < LRX; ++i) {
        const int row = G::RPI * i + (t >> 3);
        const int r = mt * G::BM + row;
        const uint32_t base =
            r < a.M ? (uint32_t)r * 128u + (uint32_t)(((t & 7) ^ ((row >> 1) & 7)) * 16) : 0x80000000u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rxr, (__attribute__((address_space(3))) void*)(img + i * (G::RPI * 128) + wave * 1024), 16, base, 0, 0, 0);
      }
    }
  };

  const int first = slot, step = a.nslots;
  const int n_mine = first < a.tiles_m ? (a.tiles_m - first + step - 1) / step : 0;
  // every DMA is issued, past the block's last tile as a dummy one (every row out of range: zeros into a ring buffer no
  // tile uses), so each wait count below is the same on every iteration — and so are hipcc's own counts for the loads
  // issued before a DMA (with a conditional DMA it assumes the no-DMA path and drains it)
  auto tile_of = [&](int i) { return i < n_mine ? first + i * step : a.tiles_m; };

  float cs[4][4], cq[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) cs[j][r] = cq[j][r] = 0.f;

  // MODE 2: this thread's 8-channel chunk of the tile row is fixed (NTH % 32 == 0): its BN coefficients live in
  // registers for the whole kernel
  const int ch = t & 31;
  const int nch = tile_n * 256 + ch * 8;
  float bsc[8], bsh[8], rsc[8], rsh[8];
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.res, (short)0, (MODE == 2 && a.res) ? (int)((long)a.M * a.K * 2) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t orr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.out, (short)0, MODE == 2 ? (int)((long)a.M * a.K * 2) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t mr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.mbits, (short)0, (MODE == 2 && a.mbits) ? (int)((long)a.M * a.K / 8) : 0, 0x00020000);
  // MODE 3: the old values (beta source), the BN input and its mask, the batch mean of this thread's 8 channels, and the
  // thread's running sums of dz and dz * (x - mean) over all of its rows
  const __amdgpu_buffer_rsrc_t cr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.cin, (short)0, (MODE == 3 && a.cin) ? (int)((long)(a.bW ? a.M / 4 : a.M) * a.K * 2) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t xbr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.bnx, (short)0, (MODE == 3 && a.bnmean && !RX) ? (int)((long)a.M * a.K * 2) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t bmr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.betamask, (short)0, (MODE == 3 && a.betamask) ? (int)((long)a.M * a.K / 8) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t xmr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.bnmask, (short)0, (MODE == 3 && a.bnmask) ? (int)((long)a.M * a.K / 8) : 0, 0x00020000);
  const uint32_t bm_or = a.betamask ? 0u : 0xFFu, xm_or = a.bnmask ? 0u : 0xFFu;  // absent mask: every bit set
  float mu3[8], s3[8], q3[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s3[j] = q3[j] = 0.f;
    mu3[j] = (MODE == 3 && a.bnmean) ? a.bnmean[nch + j] : 0.f;
  }
  if constexpr (MODE == 2) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bsc[j] = a.scale[nch + j];
      bsh[j] = a.shift[nch + j];
      rsc[j] = a.rscale ? a.rscale[nch + j] : 1.f;
      rsh[j] = a.rscale ? a.rshift[nch + j] : 0.f;
    }
  }
  // consume every per-kernel register operand loaded above (filter slices, coefficients, means) BEFORE the first DMA:
  // hipcc otherwise places their vmcnt waits at their first use inside the tile loop, where on every later iteration
  // those waits hold up the in-flight DMA and stores instead
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int s = 0; s < C / 32; ++s) asm volatile("" ::"v"(fb[j][s]));
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if constexpr (MODE == 2) asm volatile("" ::"v"(bsc[j]), "v"(bsh[j]), "v"(rsc[j]), "v"(rsh[j]));
    if constexpr (MODE == 3) asm volatile("" ::"v"(mu3[j]));
  }
  issue(tile_of(0), 0);
  issue_rx(tile_of(0), 0);
  issue(tile_of(1), 1);
  issue_rx(tile_of(1), 1);

  for (int it = 0; it < n_mine; ++it) {
    // tile `it` landed. MODE 0: the ops this thread issued after it are tile it+1's DMA (a dummy past the last tile)
    // and tile it-1's stores. MODE 1: only tile it+1's DMA. MODE 2 / 3: tile `it` is older than tile it-1's loads,
    // which iteration it-1 waited for — only the first tile needs a wait here.
    if constexpr (MODE == 0) {
      if (it == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::LD) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::LD + G::ST) : "memory");
    } else if constexpr (MODE == 1) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::LD) : "memory");
    } else {  // MODE 2 / 3
      if (it == 0) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LDT) : "memory");
      }
    }
    tile_barrier();  // every wave's DMA share landed; every wave is done with the buffer tile it+2 reuses
    const int mt = first + it * step;
    // MODE 2: this tile's residual chunks, in flight under the MFMAs (issued before tile it+2's DMA, so waiting for
    // them leaves that DMA in flight)
    uint4 rv[G::ST];
    // MODE 3: this tile's old values (beta source), BN input chunks and mask bytes, likewise in flight under the
    // MFMAs (rows past M read as zeros through the range check: no beta term, dz = 0)
    uint4 xv[MODE == 3 ? G::ST : 1];
    uint32_t bmb[MODE == 3 ? G::ST : 1], xmb[MODE == 3 ? G::ST : 1];
    if constexpr (MODE == 3) {
      // addresses first (the compact source's pixel decomposition is all ALU), then the loads back to back
      uint32_t off[G::ST], boff[G::ST], coff[G::ST], cbits[G::ST];
#pragma unroll
      for (int k = 0; k < G::ST; ++k) {
        const int row = (t + k * G::NTH) >> 5;
        const int m = mt * G::BM + row;
        const uint32_t e = (uint32_t)m * (uint32_t)a.K + (uint32_t)nch;
        off[k] = m < a.M ? e * 2u : 0x80000000u;
        boff[k] = m < a.M ? e >> 3 : 0x80000000u;
        coff[k] = off[k];
        cbits[k] = 0xFFu;
        if (a.bW) {  // compact stride-2 source: even pixels only
          const uint32_t hw = (uint32_t)m % (uint32_t)(a.bH * a.bW), img = (uint32_t)m / (uint32_t)(a.bH * a.bW);
          const uint32_t h = hw / (uint32_t)a.bW, w = hw % (uint32_t)a.bW;
          const bool even = m < a.M && !((h | w) & 1u);
          coff[k] = even ? (((img * (uint32_t)(a.bH / 2) + (h >> 1)) * (uint32_t)(a.bW / 2) + (w >> 1)) *
                                (uint32_t)a.K + (uint32_t)nch) * 2u
                         : 0x80000000u;
          cbits[k] = even ? 0xFFu : 0u;
        }
      }
      // (unconditional: a null operand has a zero-size range, its loads return zeros without touching memory)
#pragma unroll
      for (int k = 0; k < G::ST; ++k) {
        rv[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(cr, coff[k], 0, 0));
        if constexpr (!RX) xv[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xbr, off[k], 0, 0));
        bmb[k] = ((uint32_t)__builtin_amdgcn_raw_buffer_load_b8(bmr, boff[k], 0, 0) | bm_or) & cbits[k];
        xmb[k] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(xmr, boff[k], 0, 0) | xm_or;
      }
    }
    if constexpr (MODE == 2) {  // (unconditional: without a residual the range is empty and the loads return zeros;
                                 // a branch here makes hipcc wait for them at the join)
#pragma unroll
      for (int k = 0; k < G::ST; ++k) {
        const int row = (t + k * G::NTH) >> 5;
        const int m = mt * G::BM + row;
        const uint32_t off = m < a.M ? ((uint32_t)m * (uint32_t)a.K + (uint32_t)nch) * 2u : 0x80000000u;
        rv[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0));
      }
    }
    issue(tile_of(it + 2), (it + 2) % G::NBUF);
    issue_rx(tile_of(it + 2), (it + 2) % G::NBUF);
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
          if constexpr (MODE != 1) {
            const int ml = wm * 64 + 16 * i + (lane & 15), nl = wn * 64 + 16 * j + 4 * (lane >> 4);
            stage_write(stg + (ml * G::SROW + nl) * 2, o);
          }
        } else if constexpr (MODE != 1) {
          const uint32_t off = m < a.M ? ((uint32_t)m * (uint32_t)a.K + (uint32_t)n) * 2u : 0x80000000u;
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2i, o), yr, off, 0, 0);
        }
        if constexpr (MODE < 2) {
          // statistics of the stored values (rows past M hold exact zeros: they add nothing)
          const float v0 = __uint_as_float(o.x << 16), v1 = __uint_as_float(o.x & 0xffff0000u);
          const float v2 = __uint_as_float(o.y << 16), v3 = __uint_as_float(o.y & 0xffff0000u);
          cs[j][0] += v0; cq[j][0] = fmaf(v0, v0, cq[j][0]);
          cs[j][1] += v1; cq[j][1] = fmaf(v1, v1, cq[j][1]);
          cs[j][2] += v2; cq[j][2] = fmaf(v2, v2, cq[j][2]);
          cs[j][3] += v3; cq[j][3] = fmaf(v3, v3, cq[j][3]);
        }
      }
    }
    if constexpr (STG && MODE == 0) {
      tile_barrier();  // the tile is staged (the next tile's staging writes come after the next top barrier)
      uint4 sv[G::ST];
      int so[G::ST];
#pragma unroll
      for (int k = 0; k < G::ST; ++k) so[k] = (((t + k * G::NTH) >> 5) * G::SROW + ((t + k * G::NTH) & 31) * 8) * 2;
      stage_read(sv, stg, so);
#pragma unroll
      for (int k = 0; k < G::ST; ++k) {
        const int c = t + k * G::NTH, row = c >> 5, ch = c & 31;
        const int m = mt * G::BM + row;
        const uint4 v = sv[k];
        const uint32_t off =
            m < a.M ? ((uint32_t)m * (uint32_t)a.K + (uint32_t)(tile_n * 256 + ch * 8)) * 2u : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), yr, off, 0, 0);
      }
    }
    if constexpr (MODE == 2) {
      tile_barrier();  // the tile is staged
      // the residual chunks are in: everything but tile it+2's DMA (issued after them) has completed
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::LD) : "memory");
      uint4 sv[G::ST];
      int so[G::ST];
#pragma unroll
      for (int k = 0; k < G::ST; ++k) so[k] = (((t + k * G::NTH) >> 5) * G::SROW + ch * 8) * 2;
      stage_read(sv, stg, so);
#pragma unroll
      for (int k = 0; k < G::ST; ++k) {
        const int row = (t + k * G::NTH) >> 5;
        const int m = mt * G::BM + row;
        const uint4 yv = sv[k];
        const uint32_t e = (uint32_t)m * (uint32_t)a.K + (uint32_t)nch;  // element index (valid rows)
        const uint32_t off = m < a.M ? e * 2u : 0x80000000u;
        if (a.Y) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, yv), yr, off, 0, 0);
        // bn_apply_row's arithmetic, operation for operation (bitwise the same block output)
        const uint32_t yw[4] = {yv.x, yv.y, yv.z, yv.w};
        const uint32_t rw[4] = {rv[k].x, rv[k].y, rv[k].z, rv[k].w};
        float o[8];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int j = 2 * q + h;
            const float f = __uint_as_float(h ? (yw[q] & 0xffff0000u) : (yw[q] << 16));
            float v = fmaf(f, bsc[j], bsh[j]);
            if (a.res) {
              const float r = __uint_as_float(h ? (rw[q] & 0xffff0000u) : (rw[q] << 16));
              v += a.rscale ? fmaf(r, rsc[j], rsh[j]) : r;
            }
            if (a.relu) v = fmaxf(v, 0.f);
            o[j] = v;
          }
        const uint4 ov = make_uint4(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]), pack2bf(o[4], o[5]),
                                    pack2bf(o[6], o[7]));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, ov), orr, off, 0, 0);
        if (a.mbits) {
          uint32_t bits = 0;
#pragma unroll
          for (int j = 0; j < 8; ++j) bits |= (uint32_t)(f2bf(o[j]) != 0 && o[j] > 0.f) << j;
          __builtin_amdgcn_raw_buffer_store_b8((uint8_t)bits, mr, m < a.M ? e >> 3 : 0x80000000u, 0, 0);
        }
      }
    }
    if constexpr (MODE == 3) {
      if constexpr (RX) {
        // the BN input of this tile: y = bf16(rx rw^T) for the wave's 64 columns, the producing pwconv forward's MFMA
        // sequence (fragments in the same k order, kk 0 then 1), staged for the store pass
        const char* rimg = rximg + (it % G::NBUF) * RIMG;
        v4f ay[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) ay[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          v8bf fa[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) fa[i] = frag_kcontig(rimg, 16 * i, kk, lane);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) ay[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[j][kk], fa[i], ay[i][j], 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            uint2 o;
            o.x = pack2bf(ay[i][j][0], ay[i][j][1]);
            o.y = pack2bf(ay[i][j][2], ay[i][j][3]);
            stage_write(ystg + ((16 * i + (lane & 15)) * YROW + wn * 64 + 16 * j + 4 * (lane >> 4)) * 2, o);
          }
      }
      tile_barrier();  // the tile is staged (RX: and its BN input)
      // the tile's loads are in: everything but tile it+2's DMA (issued after them) has completed
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LDT) : "memory");
      uint4 sv[G::ST];
      int so[G::ST];
#pragma unroll
      for (int k = 0; k < G::ST; ++k) so[k] = (((t + k * G::NTH) >> 5) * G::SROW + ch * 8) * 2;
      stage_read(sv, stg, so);
      if constexpr (RX) {
#pragma unroll
        for (int k = 0; k < G::ST; ++k) so[k] = (((t + k * G::NTH) >> 5) * YROW + ch * 8) * 2;
        stage_read(xv, ystg, so);
      }
#pragma unroll
      for (int k = 0; k < G::ST; ++k) {
        const int row = (t + k * G::NTH) >> 5;
        const int m = mt * G::BM + row;
        uint4 val = sv[k];
        if (a.cin) {  // gemm_epilogue's staged beta path, operation for operation
          const uint32_t vw[4] = {val.x, val.y, val.z, val.w}, ow[4] = {rv[k].x, rv[k].y, rv[k].z, rv[k].w};
          float f[8], g[8];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            f[2 * q] = __uint_as_float(vw[q] << 16); f[2 * q + 1] = __uint_as_float(vw[q] & 0xffff0000u);
            g[2 * q] = __uint_as_float(ow[q] << 16); g[2 * q + 1] = __uint_as_float(ow[q] & 0xffff0000u);
          }
#pragma unroll
          for (int r = 0; r < 8; ++r) f[r] = ((bmb[k] >> r) & 1u) ? fmaf(a.beta, g[r], f[r]) : f[r];
          val = make_uint4(pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]), pack2bf(f[6], f[7]));
        }
        const uint32_t off = m < a.M ? ((uint32_t)m * (uint32_t)a.K + (uint32_t)nch) * 2u : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, val), yr, off, 0, 0);
        {  // (unconditional: with no bnmean the sums are of zeros and never written; a branch here leaves the xv
           // loads unconsumed on one path, and the compiler then drains every load before the next tile's)
          const uint32_t vw[4] = {val.x, val.y, val.z, val.w}, xw[4] = {xv[k].x, xv[k].y, xv[k].z, xv[k].w};
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int r = 2 * q + h;
              const float dv = __uint_as_float(h ? (vw[q] & 0xffff0000u) : (vw[q] << 16));
              const float xx = __uint_as_float(h ? (xw[q] & 0xffff0000u) : (xw[q] << 16));
              const float dz = ((xmb[k] >> r) & 1u) ? dv : 0.f;
              s3[r] += dz;
              q3[r] = fmaf(dz, xx - mu3[r], q3[r]);
            }
        }
      }
    }
  }
  // the dummy DMA past the last tile (and, for blocks without tiles, both prologue ones) lands in the ring before it
  // is reused below
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (MODE == 2) return;  // (no statistics)
  if constexpr (MODE == 3) {
    if (!a.bnmean) return;
    // one partial row per block: the NTH / 32 threads of each 8-channel chunk folded through LDS in a fixed order
    __syncthreads();  // the ring is free
    float* red = reinterpret_cast<float*>(smem);  // [thread][sum 8 | sq 8]
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[t * 16 + j] = s3[j];
      red[t * 16 + 8 + j] = q3[j];
    }
    __syncthreads();
    if (t < 256) {  // column t of this block's 256: chunk t >> 3, channel t & 7
      const int c8 = t >> 3, j = t & 7;
      float sv = 0.f, qv = 0.f;
      for (int u = c8; u < G::NTH; u += 32) {
        sv += red[u * 16 + j];
        qv += red[u * 16 + 8 + j];
      }
      float* prow = a.stats + (long)slot * 2 * a.K;
      prow[tile_n * 256 + t] = sv;
      prow[a.K + tile_n * 256 + t] = qv;
    }
    return;
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

template <int C, int WMW, bool STG, int MODE, bool RX = false>
void launch_pw(const PwArgs& a, int grid, hipStream_t st) {
  hipLaunchKernelGGL((pw_conv_kernel<C, WMW, STG, MODE, RX>), dim3(grid), dim3(256 * WMW), 0, st, a);
}

template <int MODE>
void launch_pw_c(const PwArgs& a, int C, int grid, hipStream_t st) {
  // (MODE 3 keeps one row wave for C 64 too: its epilogue holds four operands per chunk in flight, which needs the
  // one-wave-per-SIMD register budget — two row waves spill)
  if constexpr (MODE == 3) {  // (RX: the stage-1 BN inputs, consumed by the C 64 / 128 data gradients only)
    if (a.rx && C == 64) return launch_pw<64, 1, true, MODE, true>(a, grid, st);
    if (a.rx && C == 128) return launch_pw<128, 1, true, MODE, true>(a, grid, st);
  }
  if (C == 64) {
    if constexpr (MODE == 3) launch_pw<64, 1, true, MODE>(a, grid, st);
    else launch_pw<64, 2, true, MODE>(a, grid, st);
  } else if (C == 128) launch_pw<128, 1, true, MODE>(a, grid, st);
  else launch_pw<256, 1, true, MODE>(a, grid, st);
}

// grid / row-slot plan shared by every mode (the same tile -> block assignment in both passes of the two-pass form)
bool pw_plan(PwArgs& a, long M, int C, int K, int& grid, bool one_row_wave = false) {
  if (!(C == 64 || C == 128 || C == 256) || (K % 256)) return false;
  const int tiles_n = K / 256;
  if (tiles_n != 1 && tiles_n != 2 && tiles_n != 4 && tiles_n != 8) return false;
  if (M * C * 2 >= (1l << 31) || M * K * 2 >= (1l << 31)) return false;
  // C 128 / 256: one row wave per block (the 128-VGPR filter slice; for C 128 the 3-deep ring plus the LDS store
  // stage of a 128-row tile would exceed the LDS); C 64: two row waves per block. Every tile is stored through an
  // LDS stage as row-contiguous 16-B chunks. (Measured alternatives, removed: several one-row-wave blocks per CU
  // for C 64, direct fragment stores: profiles/r4_pointwise_conv_bw_probe.txt, r4_negative_results.txt.)
  const int wmw = (C == 64 && !one_row_wave) ? 2 : 1;
  const int bm = 64 * wmw;
  a.M = (int)M; a.K = K;
  a.tiles_m = (int)((M + bm - 1) / bm);
  a.tiles_n = tiles_n;
  if (a.tiles_m < 8) return false;
  // one block per CU (or bpc); fewer when there are fewer tiles (grid stays a multiple of 8 * tiles_n, and the
  // partial rows (one per row slot) never outnumber the M-tiles: the caller's scratch holds ceil(M/64) rows)
  grid = 256;
  while (grid > 8 * tiles_n && grid / tiles_n > a.tiles_m) grid /= 2;
  a.nslots = grid / tiles_n;
  if (a.nslots > a.tiles_m && a.nslots > 8) return false;
  return true;
}

}  // namespace

// Y[M][K] = X[M][C] . W[K][C]^T with the per-column BN statistics of Y as partial rows; C in {64, 128, 256},
// K a multiple of 256 with K/256 in {1, 2, 4, 8}. Returns the number of partial rows written (> 0) or 0 when the
// shape is not handled (the caller uses the general kernel).
int pwconv_try(const void* X, const void* W, void* Y, float* stats, long M, int C, int K, hipStream_t st) {
  if (!stats) return 0;
  if (((uintptr_t)X & 15) || ((uintptr_t)W & 15) || ((uintptr_t)Y & 15)) return 0;
  PwArgs a{};
  int grid = 0;
  if (!pw_plan(a, M, C, K, grid)) return 0;
  a.X = (const bf16_t*)X; a.W = (const bf16_t*)W; a.Y = (bf16_t*)Y; a.stats = stats;
  launch_pw_c<0>(a, C, grid, st);
  return hipGetLastError() == hipSuccess ? a.nslots : 0;
}

// MODE 3: dX[M][N] = dY[M][Kc] . Wck^T (Wck: the conv filter as [N][Kc], i.e. [C][1][1][K]) for a channel-reducing
// 1x1 conv's data gradient (Kc in {64, 128, 256}, N a multiple of 256 with N/256 in {1, 2, 4, 8}), optionally
// accumulating beta * dX in place (betamask: the deferred ReLU bits of the old values) and with bnmean the
// BatchNorm-backward partial rows of dX into part. Returns the number of partial rows (> 0), or 0 when not handled.
// bsrc2 (with H, W even): instead of beta * dX, add the compact stride-2 shortcut gradient at the even pixels.
int pwconv_dgrad_try(const void* dY, const void* Wck, void* dX, float beta, const void* betamask, const void* bnx,
                     const void* bnmask, const float* bnmean, float* part, long M, int Kc, int N, const void* bsrc2,
                     int H, int W, hipStream_t st, const void* bnrx, const void* bnrw) {
  if (((uintptr_t)dY & 15) || ((uintptr_t)Wck & 15) || ((uintptr_t)dX & 15) || ((uintptr_t)bnx & 15) ||
      ((uintptr_t)bsrc2 & 15))
    return 0;
  if ((bnmean != nullptr) != (part != nullptr) || (bnmean && !bnx && !bnrx) || (betamask && beta == 0.f)) return 0;
  if (bnrx && (bnx || !bnmean || !bnrw || N != 256 || (Kc != 64 && Kc != 128) || ((uintptr_t)bnrx & 15) ||
               ((uintptr_t)bnrw & 15) || M * 128 >= (1l << 31)))
    return 0;
  if (bsrc2 && (betamask || (H & 1) || (W & 1) || (long)H * W <= 0 || M % ((long)H * W))) return 0;
  PwArgs a{};
  int grid = 0;
  if (!pw_plan(a, M, Kc, N, grid, true)) return 0;
  a.X = (const bf16_t*)dY; a.W = (const bf16_t*)Wck; a.Y = (bf16_t*)dX; a.stats = part;
  if (bsrc2) {
    a.cin = (const bf16_t*)bsrc2;
    a.bH = H; a.bW = W;
    beta = 1.f;
  } else {
    a.cin = beta != 0.f ? (const bf16_t*)dX : nullptr;
  }
  a.beta = beta;
  a.betamask = (const uint8_t*)betamask;
  a.bnx = (const bf16_t*)bnx; a.bnmask = (const uint8_t*)bnmask; a.bnmean = bnmean;
  a.rx = (const bf16_t*)bnrx; a.rw = (const bf16_t*)bnrw;
  launch_pw_c<3>(a, Kc, grid, st);
  return hipGetLastError() == hipSuccess ? a.nslots : 0;
}

}  // namespace dtf

DTF_API int dtf_bn_finalize(float* part, int T, const float* gamma, const float* beta, float* running_mean,
                            float* running_var, long M, int C, float momentum, float eps, float* scale,
                            float* shift, float* mean_out, float* invstd_out, void* stream);  // norm.hip

// Two-pass training ConvBN forward of a channel-expanding 1x1 conv (see the MODE notes at the top):
//   pass 1: statistics of yc = X W^T (nothing stored) -> part;  finalize -> scale/shift/mean/invstd + running stats;
//   pass 2: out = [relu](yc * scale + shift [+ res | + res * rscale + rshift]) with its ReLU mask mbits (relu only),
//           and yc itself only when Y != nullptr.
// part: >= ceil(M/64) * 2K floats of scratch. Returns 0, or -1 when the shape is not handled (nothing launched).
DTF_API int dtf_conv_bn_apply_fwd(const void* X, const void* W, void* Y, void* out, void* mbits, const void* res,
                                  const float* rscale, const float* rshift, long M, int C, int K, int relu,
                                  float* part, const float* gamma, const float* beta, float* rmean, float* rvar,
                                  float momentum, float eps, float* scale, float* shift, float* mean, float* invstd,
                                  void* stream) {
  using namespace dtf;
  hipStream_t st = (hipStream_t)stream;
  if (((uintptr_t)X & 15) || ((uintptr_t)W & 15) || ((uintptr_t)Y & 15) || ((uintptr_t)out & 15) ||
      ((uintptr_t)res & 15) || !out || !part || ((rscale == nullptr) != (rshift == nullptr)))
    return -1;
  PwArgs a{};
  int grid = 0;
  if (!pw_plan(a, M, C, K, grid)) return -1;
  a.X = (const bf16_t*)X; a.W = (const bf16_t*)W; a.stats = part;
  launch_pw_c<1>(a, C, grid, st);
  int rc = dtf_bn_finalize(part, a.nslots, gamma, beta, rmean, rvar, M, K, momentum, eps, scale, shift, mean, invstd,
                           stream);
  if (rc) return rc;
  a.Y = (bf16_t*)Y;
  a.scale = scale; a.shift = shift;
  a.res = (const bf16_t*)res;
  a.rscale = res ? rscale : nullptr;
  a.rshift = res ? rshift : nullptr;
  a.out = (bf16_t*)out;
  a.mbits = relu ? (uint8_t*)mbits : nullptr;
  a.relu = relu;
  launch_pw_c<2>(a, C, grid, st);
  return (int)hipGetLastError();
}

// Test / tuning entry: the pointwise forward on its own (stats: [nslots][2K] floats, nslots <= ceil(M/64)).
DTF_API int dtf_pwconv_fwd(const void* X, const void* W, void* Y, float* stats, int* rows, long M, int C, int K,
                           void* stream) {
  const int r = dtf::pwconv_try(X, W, Y, stats, M, C, K, (hipStream_t)stream);
  if (rows) *rows = r;
  return r > 0 ? 0 : -1;
}
