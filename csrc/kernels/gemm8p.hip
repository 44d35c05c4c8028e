// 256x256x64 bf16 GEMM / implicit-GEMM convolution with the 8-phase counted-vmcnt schedule, gfx950.
//
// C = A . B^T for K-contiguous B (weights [N][K]) and K-contiguous A that is either a plain [M][K] matrix or an
// implicit-GEMM gather (the tap-uniform conv forward / stride-1 data-gradient forms of gemm_core.h: a 64-wide K-tile
// is one filter tap x 64 channels, so a tile is a wave-uniform tap offset added to per-row pixel offsets, with a
// per-row in-image tap mask; masked rows read zeros through the buffer range check).
//
// Why (profiles/r3_conv_roofline.txt): the 128-row conv tiles of gemm_core.h run one
// barrier per K-tile with at most one tile of LDS-DMA in flight and sit at 650-870 TF on the ResNet-50 3x3
// convolutions; gemm256.hip's 4-phase schedule reaches ~1.2 PF on 8192^3. This kernel is the structure of
// cdna_hip_programming.md §5 "The 256^2 8-phase template": 8 waves (2 M x 4 N, 128x64 output per wave), both
// operands staged straight into LDS by LDS-DMA (buffer_load ... lds, 16 B per lane), 2 stage buffers x 4 half-tiles
// (A0 A1 B0 B1, 16 KiB each), and each K-tile split into 4 phases, one output quadrant each
// (A0xB0, A0xB1, A1xB1, A1xB0: 16 MFMA 16x16x32 per wave):
//     ds_read the phase's fragments -> issue ONE half-tile of the prefetch stream -> [vmcnt] -> s_barrier ->
//     lgkmcnt(0) -> setprio(1) 16 x MFMA setprio(0) -> s_barrier
// Prefetch order (tile T in stage T&1, phases q0..q3): q0 A1(T+1), q1 B0(T+2), q2 A0(T+2), q3 B1(T+2). A half is
// restaged one phase after the phase that last read it (its reads were retired by that phase's lgkmcnt(0) before
// its closing barrier), and read one phase after the counted wait that retires it: vmcnt(6) at q3 leaves exactly
// the three half-tiles of T+2 in flight and retires A1(T+1), the last half of the next tile. Never vmcnt(0) in the
// steady state; raw s_barrier only (__syncthreads() would drain the in-flight LDS-DMA).
// The LDS image of a half is lane-linear (a wave instruction fills 8 rows x 128 B); the bank-conflict swizzle
// (chunk ^ ((row >> 1) & 7)) is applied on the per-lane SOURCE address and undone by frag_kcontig's read.
// Epilogue: gemm_core.h gemm_epilogue (bias / activation / BatchNorm statistics / BN finalize / split-K slabs).
// Reference op family: MatMul / Conv2D of the TF runtime the reference drives.
#include "gemm_core.h"

namespace dtf {
namespace {

constexpr int T8 = 512;          // threads: 8 waves
constexpr int HA_BYTES = 128 * 128;  // bytes of one A half-tile image: 128 rows x 64 bf16

// Tile geometry by output width BN: 256 -> 8 waves as 2 (M) x 4 (N), 128x64 per wave, 16 MFMA per phase;
// 128 -> 4 (M) x 2 (N), 64x64 per wave, 8 MFMA per phase (the ResNet-50 stage-2..4 widths: twice the tiles).
template <int BN>
struct Geo8 {
  static constexpr int WM = BN == 256 ? 2 : 4, WN = 8 / WM;
  static constexpr int WTM = 256 / WM, WTN = BN / WN;
  static constexpr int HA = WTM / 2, HBC = WTN / 2;   // rows (A) / columns (B) of one wave in one half image
  static constexpr int FA = HA / 16, FB = HBC / 16;   // fragments per wave per half
  static constexpr int HB_BYTES = BN * 64;            // one B half image: BN/2 rows x 64 bf16
  static constexpr int STAGE = 2 * HA_BYTES + 2 * HB_BYTES;  // A0 | A1 | B0 | B1
  static constexpr int UA = 2, UB = HB_BYTES / 8192;  // LDS-DMA instructions per thread per half
  static constexpr int VM_Q3 = 2 * UB + UA;           // halves of tile t+2 in flight at the q3 wait (B0 A0 B1)
};

__device__ __forceinline__ void barrier8() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// image row r of half h -> row of the block operand: a wave's S rows (A) / columns (B) of one half are contiguous in
// the image, the two halves of a wave's 2S interleave in the block
template <int S>
__device__ __forceinline__ int blk_row(int r, int h) { return (r / S) * (2 * S) + h * S + (r % S); }

// One operand's two half images. Thread t fills, per half and instruction u (0, 1), image row 64u + 8 wave +
// (lane >> 3), physical 16-B slot lane & 7, i.e. logical chunk (lane & 7) ^ ((row >> 1) & 7) (the same for every u
// and half: bits 1..3 of the row come from wave and lane only).
template <int MODE, int S, int U>  // S: rows of a wave per half (blk_row); U: instructions per half (image rows 64U)
struct HalfLoad {
  static_assert(MODE == OP_KCONTIG || MODE == OP_IM2COL_T || MODE == OP_DGRAD_T, "K-contiguous modes only");
  __amdgpu_buffer_rsrc_t rsrc;
  int roff[2][U];
  uint32_t tmask[2][U];
  int coff;

  __device__ __forceinline__ void init(const GemmArgs& a, const bf16_t* p, long ld, int r0, int Rtot) {
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const ConvGeom& g = a.g;
    uint32_t bytes;
    if constexpr (MODE == OP_KCONTIG) bytes = (uint32_t)((long)Rtot * ld * 2);  // host: < 2 GiB
    else if constexpr (MODE == OP_IM2COL_T) bytes = (uint32_t)((long)g.N * g.H * g.W * g.C * 2);
    else bytes = (uint32_t)((long)g.N * g.P * g.Q * g.Kout * 2);
    rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
    const int rr = 8 * w + (lane >> 3);
    coff = ((lane & 7) ^ ((rr >> 1) & 7)) * 16;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int ir = 64 * u + rr;
        const int r = r0 + blk_row<S>(ir, h);
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
        roff[h][u] = off;
        tmask[h][u] = m;
      }
  }

  // issue half h of the K-tile starting at k0 into its image at `img` (U LDS-DMA instructions per thread)
  __device__ __forceinline__ void issue(const GemmArgs& a, int k0, int h, char* img) {
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
    for (int u = 0; u < U; ++u) {
      const bool ok = (tmask[h][u] >> tap) & 1u;
      const uint32_t off = ok ? (uint32_t)(roff[h][u] + toff + coff) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsrc, (__attribute__((address_space(3))) void*)(img + u * 8192 + w * 1024), 16, off, 0, 0, 0);
    }
  }
};

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int AM, int BN>
__global__ void __launch_bounds__(T8, 1) gemm8p_kernel(GemmArgs a) {
  using G = Geo8<BN>;
  constexpr int STAGE = G::STAGE, FA = G::FA, FB = G::FB;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / G::WN, wc = wave % G::WN;

  // block -> tile: XCD-aware bijective remap, then groups of 4 M-tiles x all N-tiles (shared A rows / B columns)
  const int nwg = a.tiles_m * a.tiles_n;
  int bid, z;
  xcd_block(nwg, bid, z);
  constexpr int GROUP = 4;
  const int per_group = GROUP * a.tiles_n;
  const int grp = bid / per_group;
  const int first_m = grp * GROUP;
  const int gsize = min(a.tiles_m - first_m, GROUP);
  const int in_g = bid - grp * per_group;
  const int tile_m = first_m + in_g % gsize;
  const int tile_n = in_g / gsize;
  const int m0 = tile_m * 256, n0 = tile_n * BN;
  if (a.zero_slot && blockIdx.x == 0 && blockIdx.z == 0 && threadIdx.x == 0) *a.zero_slot = 0.f;
  const int bz = z / a.splitk, sk = z % a.splitk;
  const int kbeg = sk * a.kchunk;
  const int kend = min(a.K, kbeg + a.kchunk);
  const int nk = kend > kbeg ? (kend - kbeg) / BK : 0;

  HalfLoad<AM, G::HA, G::UA> la;
  HalfLoad<OP_KCONTIG, G::HBC, G::UB> lb;
  la.init(a, a.A + (long)bz * a.sA, a.lda, m0, a.M);
  lb.init(a, a.B + (long)bz * a.sB, a.ldb, n0, a.N);

  v4f acc[2 * FA][2 * FB];
#pragma unroll
  for (int i = 0; i < 2 * FA; ++i)
#pragma unroll
    for (int j = 0; j < 2 * FB; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
  v8bf fa[FA][2], fb0[FB][2], fb1[FB][2];

  // half: 0 A0, 1 A1, 2 B0, 3 B1
  auto img = [&](int t, int half) {
    return smem + (t & 1) * STAGE + (half < 2 ? half * HA_BYTES : 2 * HA_BYTES + (half - 2) * G::HB_BYTES);
  };
  auto issue = [&](int t, int half) {
    if (half < 2) la.issue(a, kbeg + t * BK, half, img(t, half));
    else lb.issue(a, kbeg + t * BK, half - 2, img(t, half));
  };
  auto read_a = [&](int t, int h) {
    const char* base = img(t, h);
#pragma unroll
    for (int i = 0; i < FA; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fa[i][kk] = frag_kcontig(base, wr * G::HA + i * 16, kk, lane);
  };
  auto read_b = [&](v8bf (&fb)[FB][2], int t, int h) {
    const char* base = img(t, 2 + h);
#pragma unroll
    for (int j = 0; j < FB; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fb[j][kk] = frag_kcontig(base, wc * G::HBC + j * 16, kk, lane);
  };
  auto mma = [&](const v8bf (&fb)[FB][2], int ha, int hb) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < FA; ++i)
#pragma unroll
        for (int j = 0; j < FB; ++j)
          acc[ha * FA + i][hb * FB + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][kk], fa[i][kk], acc[ha * FA + i][hb * FB + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue: tile 0 whole, then B0 A0 B1 of tile 1 (tile -1's q1..q3 issues); wait for tile 0
  if (nk > 0) {
    issue(0, 0); issue(0, 2); issue(0, 3); issue(0, 1);
  }
  if (nk > 1) {
    issue(1, 2); issue(1, 0); issue(1, 3);
    vm_wait<G::VM_Q3>();
  } else {
    vm_wait<0>();
  }
  barrier8();

  for (int t = 0; t < nk; ++t) {
    const bool n1 = t + 1 < nk, n2 = t + 2 < nk;
    // q0: A0 x B0 (issue A1 of tile t+1)
    read_b(fb0, t, 0);
    read_a(t, 0);
    if (n1) issue(t + 1, 1);
    barrier8();
    mma(fb0, 0, 0);
    barrier8();
    // q1: A0 x B1 (issue B0 of tile t+2: B0 of this stage was last read in q0)
    read_b(fb1, t, 1);
    if (n2) issue(t + 2, 2);
    barrier8();
    mma(fb1, 0, 1);
    barrier8();
    // q2: A1 x B1 (issue A0 of tile t+2)
    read_a(t, 1);
    if (n2) issue(t + 2, 0);
    barrier8();
    mma(fb1, 1, 1);
    barrier8();
    // q3: A1 x B0 from registers (issue B1 of tile t+2); retire every half of tile t+1 before the barrier
    if (n2) issue(t + 2, 3);
    if (n2) vm_wait<G::VM_Q3>();
    else vm_wait<0>();
    barrier8();
    mma(fb0, 1, 0);
    barrier8();
  }
  __syncthreads();  // (no LDS-DMA in flight: the last tiles drained with vmcnt(0)) the epilogue reuses the LDS
  gemm_epilogue<256, BN, G::WM, G::WN, T8, 2 * STAGE>(a, acc, smem, m0, n0, tile_m, z, bz);
}

}  // namespace

template <int BN>
void launch8p(GemmArgs& a, int amode, hipStream_t st) {
  a.tiles_m = cdiv(a.M, 256);
  a.tiles_n = cdiv(a.N, BN);
  prep_fin(a);
  dim3 grid(a.tiles_m * a.tiles_n, 1, a.batch * a.splitk);
  if (amode == OP_KCONTIG) hipLaunchKernelGGL((gemm8p_kernel<OP_KCONTIG, BN>), grid, dim3(T8), 0, st, a);
  else if (amode == OP_IM2COL_T) hipLaunchKernelGGL((gemm8p_kernel<OP_IM2COL_T, BN>), grid, dim3(T8), 0, st, a);
  else hipLaunchKernelGGL((gemm8p_kernel<OP_DGRAD_T, BN>), grid, dim3(T8), 0, st, a);
}

// Launch C = A . B^T on the 8-phase kernel with tile width bn (256 or 128) when eligible (K-contiguous B,
// K % 64 == 0 per split, 16-B aligned rows, operands < 2 GiB). Returns 0 if launched, 1 if not eligible.
int gemm8p_try(GemmArgs& a, int amode, int bmode, hipStream_t st, int bn) {
  if (bmode != OP_KCONTIG || a.atomic_out) return 1;
  if (amode != OP_KCONTIG && amode != OP_IM2COL_T && amode != OP_DGRAD_T) return 1;
  if (a.kchunk % BK || (a.K % BK) || (a.lda & 7) || (a.ldb & 7)) return 1;
  if (((uintptr_t)a.A & 15) || ((uintptr_t)a.B & 15)) return 1;
  auto fits = [](long elems) { return elems * 2 < (1l << 31); };
  const ConvGeom& g = a.g;
  if (amode == OP_KCONTIG && !fits((long)a.M * a.lda)) return 1;
  if (amode == OP_IM2COL_T && !fits((long)g.N * g.H * g.W * g.C)) return 1;
  if (amode == OP_DGRAD_T && !fits((long)g.N * g.P * g.Q * g.Kout)) return 1;
  if (!fits((long)a.N * a.ldb)) return 1;
  if (bn == 256) launch8p<256>(a, amode, st);
  else if (bn == 128) launch8p<128>(a, amode, st);
  else return 1;
  return 0;
}

}  // namespace dtf

// Direct entry for benchmarks/tests: C[M][N] (bf16 or f32) = A[M][K] . B[N][K]^T on the 8-phase kernel.
DTF_API int dtf_gemm8p(const void* A, const void* B, void* C, int M, int N, int K, long lda, long ldb, long ldc,
                       int out_f32, int bn, void* stream) {
  dtf::GemmArgs a{};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.batch = 1; a.splitk = 1; a.kchunk = K; a.alpha = 1.f; a.beta = 0.f; a.out_f32 = out_f32;
  if ((N & 3) || (K % dtf::BK)) return -1;
  if (dtf::gemm8p_try(a, dtf::OP_KCONTIG, dtf::OP_KCONTIG, (hipStream_t)stream, bn)) return -2;
  return (int)hipGetLastError();
}
