// 256x256 GEMM with FOUR waves (one per SIMD), each owning a 128x128 output tile, for gfx950 — bf16 (16x16x32 MFMA)
// and fp8 (block-scaled 16x16x128 MFMA, per-tensor scales in the epilogue).
//
// Why: gemm256.hip's 8-wave form gives each wave a 128x64 tile, so per K-tile every CU reads 8 x (128 + 64) x 64 x 2 B
// = 192 KiB of operand fragments out of LDS for 2 MFLOP x 8 of MFMA work — at 128 B/clk that is ~1.5k LDS cycles
// against ~1k MFMA cycles per SIMD: the loop is LDS-read bound (the fp8 form, with the same
// LDS bytes per K-tile and twice the FLOPs, doubly so). A 128x128 wave tile halves the fragment bytes per FLOP
// ((128 + 128) vs 2 x (128 + 64) per 2x the work): 4 waves x 256 x 64 x 2 B = 128 KiB per K-tile against ~2k MFMA
// cycles per SIMD — MFMA bound. The price is 256 f32 accumulators per lane (8 x 8 fragments of 16x16), which the
// 1-wave-per-SIMD occupancy (__launch_bounds__(256, 1): 512 registers per lane) pays for.
//
// Staging: both operands go straight into LDS by LDS-DMA (buffer/global_load_lds, 16 B per lane), two stages of four
// 16-KiB half images (A rows 0-127 | A rows 128-255 | B cols 0-127 | B cols 128-255): wave (wm, wn) reads A half wm
// and B half wn. K-contiguous halves are [128 rows][64 k] with the chunk XOR swizzle of gemm_core.h (frag_kcontig);
// K-outer halves are [64 k][128 cols] read with ds_read_b64_tr_b16 (gemm256.hip's half image: frag_ko). One raw
// barrier per K-tile: tile t+1's DMA is issued right after the barrier that publishes tile t, and runs under tile
// t's 128 (bf16) / 64 (fp8) MFMAs per wave.
// Epilogue: gemm256.hip's (alpha/beta, bias, ReLU/GELU, pre-activation side output, fused activation derivative,
// f32 output, split-K slabs), bf16 outputs staged through LDS one 128-row half at a time for whole 16-B row stores.
// Requirements (host-checked, as gemm256_try): K % 64 == 0 per split (bf16 elements; fp8 bytes / 2), 16-B aligned
// rows, K-outer operands with a row count % 8 == 0. M, N arbitrary (edge rows clamped on load, masked on store).
// Reference op family: the MatMul / Dense gradients of SURVEY §2.4.b K3/K3f (reference call site of the optimizer's
// gradient computation: trainer/task.py:138).
#include "gemm_core.h"

namespace dtf {
namespace {

constexpr int NT4 = 256;
constexpr int HALF4 = 128 * 128;   // bytes of one half image (128 rows x 64 bf16, or 64 k x 128 cols)
constexpr int STAGE4 = 4 * HALF4;  // A0 | A1 | B0 | B1

// K-outer half image [64 k][128 cols] (gemm256.hip): physical 16-B chunk of logical chunk c in k-row k = c ^ swz(k)
__device__ __forceinline__ int ko4_swz(int k) { return (k & 3) << 1; }
__device__ __forceinline__ v8bf frag_ko4(const char* lds, int rb, int kk, int lane) {
  const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  v4s r[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = 32 * kk + 8 * G + 4 * h + q, g = (rb >> 2) + p;
    r[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        LDS_PTR(v4s, lds + k * 256 + (((g >> 1) ^ ko4_swz(k)) << 4) + (g & 1) * 8));
  }
  v8s both = __builtin_shufflevector(r[0], r[1], 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(v8bf, both);
}

__device__ __forceinline__ void glds16(const bf16_t* g, char* lds) {
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

__device__ __forceinline__ void raw_barrier4() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int AM, int BMD, int FP8>
__global__ void __launch_bounds__(NT4, 1) gemm4w_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;

  // ---- block -> tile (XCD-aware bijective remap, grouped order: 4 M-tiles share their B columns) ----
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
  const int m0 = tile_m * 256, n0 = tile_n * 256;
  if (a.zero_slot && blockIdx.x == 0 && blockIdx.z == 0 && threadIdx.x == 0) *a.zero_slot = 0.f;
  const int bz = z / a.splitk, sk = z % a.splitk;
  const int kbeg = sk * a.kchunk;
  const int kend = min(a.K, kbeg + a.kchunk);
  const bf16_t* Ap = a.A + (long)bz * a.sA;
  const bf16_t* Bp = a.B + (long)bz * a.sB;

  // ---- per-thread LDS-DMA sources: half h (0,1 = A rows/cols h*128..; 2,3 = B), instruction u (4 per half) ----
  const bf16_t* src[4][4];
  long kstep[4];
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const bool isA = h < 2;
    const bool ko = isA ? (AM == OP_KOUTER) : (BMD == OP_KOUTER);
    const bf16_t* P = isA ? Ap : Bp;
    const long ld = isA ? a.lda : a.ldb;
    const int lim = isA ? a.M : a.N;
    const int o0 = (isA ? m0 : n0) + (h & 1) * 128;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (!ko) {  // [128 rows][64 k], 8 lanes per 128-B row: instruction u of wave w fills rows 32u + 8w .. + 7
        const int r = 32 * u + 8 * w + (lane >> 3);
        const int lc = (lane & 7) ^ ((r >> 1) & 7);
        const int g = min(o0 + r, lim - 1);
        src[h][u] = P + (long)g * ld + kbeg + lc * 8;
      } else {    // [64 k][128 cols], 16 lanes per 256-B k-row: instruction u of wave w fills k-rows 16u + 4w .. + 3
        const int k = 16 * u + 4 * w + (lane >> 4);
        const int lc = (lane & 15) ^ ko4_swz(k);
        const int g = min(o0 + lc * 8, lim - 8);
        src[h][u] = P + (long)(kbeg + k) * ld + g;
      }
    }
    kstep[h] = ko ? (long)BK * ld : (long)BK;
  }
  auto issue = [&](int t, int buf) {
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const long off = (long)t * kstep[h];
      char* d = smem + buf * STAGE4 + h * HALF4 + w * 1024;
#pragma unroll
      for (int u = 0; u < 4; ++u) glds16(src[h][u] + off, d + u * 4096);
    }
  };

  v4f acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const char* ha = smem + buf * STAGE4 + wm * HALF4;
    const char* hb = smem + buf * STAGE4 + (2 + wn) * HALF4;
    if constexpr (FP8) {
      // 128 fp8 of K per tile: one block-scaled 16x16x128 MFMA per fragment pair
      v8i fa[8], fb[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[i] = frag_fp8x128(ha, i * 16, lane);
#pragma unroll
      for (int j = 0; j < 8; ++j) fb[j] = frag_fp8x128(hb, j * 16, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = mfma_fp8_ab<FP8>(fb[j], fa[i], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    } else {
      // fragments of k-substep 1 are read while the 64 MFMAs of k-substep 0 issue (one wave per SIMD: nothing
      // else hides the LDS latency)
      v8bf fa[2][8], fb[2][8];
      auto rd = [&](int kk) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if constexpr (AM == OP_KOUTER) fa[kk][i] = frag_ko4(ha, i * 16, kk, lane);
          else fa[kk][i] = frag_kcontig(ha, i * 16, kk, lane);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if constexpr (BMD == OP_KOUTER) fb[kk][j] = frag_ko4(hb, j * 16, kk, lane);
          else fb[kk][j] = frag_kcontig(hb, j * 16, kk, lane);
        }
      };
      rd(0);
      rd(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[kk][j], fa[kk][i], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    }
  };

  // ---- main loop: one raw barrier per K-tile; tile t+1's DMA runs under tile t's MFMAs ----
  const int nk = kend > kbeg ? (kend - kbeg) / BK : 0;
  if (nk > 0) issue(0, 0);
  for (int t = 0; t < nk; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMAs of tile t (the only ones in flight) landed
    raw_barrier4();  // everyone's tile t is visible, and everyone is done reading tile t-1's buffer
    if (t + 1 < nk) issue(t + 1, (t + 1) & 1);
    compute(t & 1);
  }
  __syncthreads();  // every wave is done with the stage buffers: the epilogue reuses the LDS

  // ---- epilogue (gemm256.hip's, 128-column wave tiles) ----
  const float alpha = a.scales ? a.alpha * a.scales[0] * a.scales[1] : a.alpha;
  const long cbase = a.slab > 0 ? (long)z * a.slab : (long)bz * a.sC;
  const bool staged = !a.out_f32 && (a.beta == 0.f || (!a.aux && !a.act)) && a.slab == 0 && !(a.N & 7) &&
                      !(a.ldc & 7) && !(reinterpret_cast<uintptr_t>(a.C) & 15) &&
                      !(reinterpret_cast<uintptr_t>(a.aux) & 15);
  if (staged) {
    constexpr int CS = 256 + 8;  // LDS row stride (elements): conflict-free 8-B fragment writes
    bf16_t* ct = reinterpret_cast<bf16_t*>(smem);
    for (int o = 0; o < (a.aux ? 2 : 1); ++o) {
      bf16_t* dst = (o ? a.aux : reinterpret_cast<bf16_t*>(a.C)) + cbase;
      for (int h = 0; h < 2; ++h) {
        if (wm == h) {
#pragma unroll
          for (int i = 0; i < 8; ++i) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const int nl = wn * 128 + j * 16 + (lane >> 4) * 4;
              float v[4];
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] = alpha * acc[i][j][r];
              if (a.bias && n0 + nl < a.N) {
                const float4 b = *reinterpret_cast<const float4*>(a.bias + n0 + nl);
                v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
              }
              if (o == 0 && a.act == 1) {
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
              } else if (o == 0 && a.act == 2) {
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = gelu_tanh(v[r]);
              }
              uint2 pk;
              pk.x = pack2bf(v[0], v[1]);
              pk.y = pack2bf(v[2], v[3]);
              *reinterpret_cast<uint2*>(ct + (i * 16 + (lane & 15)) * CS + nl) = pk;
            }
          }
        }
        __syncthreads();
#pragma unroll 4
        for (int c = threadIdx.x; c < 128 * 32; c += NT4) {
          const int row = c >> 5, c8 = c & 31;
          const int m = m0 + h * 128 + row, n = n0 + c8 * 8;
          if (m < a.M && n < a.N) {
            uint4 val = *reinterpret_cast<const uint4*>(ct + row * CS + c8 * 8);
            if (o == 0 && a.beta != 0.f) {
              const uint4 old = *reinterpret_cast<const uint4*>(dst + (long)m * a.ldc + n);
              const uint32_t vw[4] = {val.x, val.y, val.z, val.w}, ow[4] = {old.x, old.y, old.z, old.w};
              float f[8];
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                f[2 * q] = fmaf(a.beta, __uint_as_float(ow[q] << 16), __uint_as_float(vw[q] << 16));
                f[2 * q + 1] = fmaf(a.beta, __uint_as_float(ow[q] & 0xffff0000u), __uint_as_float(vw[q] & 0xffff0000u));
              }
              val.x = pack2bf(f[0], f[1]); val.y = pack2bf(f[2], f[3]);
              val.z = pack2bf(f[4], f[5]); val.w = pack2bf(f[6], f[7]);
            }
            if (o == 0 && a.dact)
              val = dact8(val, *reinterpret_cast<const uint4*>(a.dact_src + (long)m * a.ldc + n), a.dact);
            *reinterpret_cast<uint4*>(dst + (long)m * a.ldc + n) = val;
          }
        }
        __syncthreads();
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wm * 128 + i * 16 + (lane & 15);
    if (m >= a.M) continue;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = n0 + wn * 128 + j * 16 + (lane >> 4) * 4;
      if (n >= a.N) continue;  // N % 4 == 0 (host)
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = alpha * acc[i][j][r];
      const long off = cbase + (long)m * a.ldc + n;
      if (a.beta != 0.f) {
        if (a.out_f32) {
          const float4 o = *reinterpret_cast<const float4*>(reinterpret_cast<float*>(a.C) + off);
          v[0] += a.beta * o.x; v[1] += a.beta * o.y; v[2] += a.beta * o.z; v[3] += a.beta * o.w;
        } else {
          const uint2 o = *reinterpret_cast<const uint2*>(reinterpret_cast<bf16_t*>(a.C) + off);
          v[0] += a.beta * __uint_as_float(o.x << 16); v[1] += a.beta * __uint_as_float(o.x & 0xffff0000u);
          v[2] += a.beta * __uint_as_float(o.y << 16); v[3] += a.beta * __uint_as_float(o.y & 0xffff0000u);
        }
      }
      if (a.bias) {
        const float4 b = *reinterpret_cast<const float4*>(a.bias + n);
        v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
      }
      if (a.aux) {
        uint2 o;
        o.x = pack2bf(v[0], v[1]);
        o.y = pack2bf(v[2], v[3]);
        *reinterpret_cast<uint2*>(a.aux + off) = o;
      }
      if (a.act == 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
      } else if (a.act == 2) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = gelu_tanh(v[r]);
      }
      if (a.out_f32) {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(a.C) + off) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        uint2 o;
        o.x = pack2bf(v[0], v[1]);
        o.y = pack2bf(v[2], v[3]);
        if (a.dact) {
          const uint2 pr = *reinterpret_cast<const uint2*>(a.dact_src + (long)m * a.ldc + n);
          const uint4 d = dact8(make_uint4(o.x, o.y, 0, 0), make_uint4(pr.x, pr.y, 0, 0), a.dact);
          o.x = d.x; o.y = d.y;
        }
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(a.C) + off) = o;
      }
    }
  }
}

}  // namespace

bool gemm4w_on() {
  static const bool on = [] {
    const char* e = getenv("DTF_GEMM4W");
    return e && e[0] == '1';
  }();
  return on;
}

// Launch on the 4-wave 256x256 kernel if eligible (same requirements as gemm256_try); 0 if launched.
int gemm4w_try(GemmArgs& a, int amode, int bmode, hipStream_t st, int fp8) {
  if (a.kchunk % BK || a.kchunk < 2 * BK || (a.lda & 7) || (a.ldb & 7) || a.stats || a.atomic_out || a.crm ||
      a.betamask || a.bsrc)
    return 1;
  if ((a.splitk > 1 && a.K % a.kchunk && (a.K % a.kchunk) % BK) || a.K % BK) return 1;
  if (((uintptr_t)a.A & 15) || ((uintptr_t)a.B & 15)) return 1;
  if ((amode == OP_KOUTER && (a.M & 7)) || (bmode == OP_KOUTER && (a.N & 7))) return 1;
  if ((amode != OP_KCONTIG && amode != OP_KOUTER) || (bmode != OP_KCONTIG && bmode != OP_KOUTER)) return 1;
  if (fp8 && (amode != OP_KCONTIG || bmode != OP_KCONTIG)) return 1;
  a.tiles_m = cdiv(a.M, 256);
  a.tiles_n = cdiv(a.N, 256);
  dim3 grid(a.tiles_m * a.tiles_n, 1, a.batch * a.splitk);
  if (fp8 == 2) hipLaunchKernelGGL((gemm4w_kernel<OP_KCONTIG, OP_KCONTIG, 2>), grid, dim3(NT4), 0, st, a);
  else if (fp8) hipLaunchKernelGGL((gemm4w_kernel<OP_KCONTIG, OP_KCONTIG, 1>), grid, dim3(NT4), 0, st, a);
  else if (amode == OP_KCONTIG && bmode == OP_KCONTIG)
    hipLaunchKernelGGL((gemm4w_kernel<OP_KCONTIG, OP_KCONTIG, 0>), grid, dim3(NT4), 0, st, a);
  else if (amode == OP_KCONTIG)
    hipLaunchKernelGGL((gemm4w_kernel<OP_KCONTIG, OP_KOUTER, 0>), grid, dim3(NT4), 0, st, a);
  else if (bmode == OP_KCONTIG)
    hipLaunchKernelGGL((gemm4w_kernel<OP_KOUTER, OP_KCONTIG, 0>), grid, dim3(NT4), 0, st, a);
  else hipLaunchKernelGGL((gemm4w_kernel<OP_KOUTER, OP_KOUTER, 0>), grid, dim3(NT4), 0, st, a);
  return 0;
}

}  // namespace dtf

// Direct entry for tests / benchmarks: C[M][N] = A(m,k) . B(n,k) on the 4-wave kernel (A [M][K] or [K][M] when
// a_kouter; B [N][K] or [K][N] when b_kouter), bf16 in, bf16 or f32 out. fp8 (1: e4m3 x e4m3, 2: e5m2 x e4m3): A and
// B are [rows][K] fp8 (K, lda, ldb in BYTES), scales: device [s_a, s_b] folded into the epilogue.
DTF_API int dtf_gemm4w(const void* A, const void* B, void* C, int M, int N, int K, long lda, long ldb, long ldc,
                       int a_kouter, int b_kouter, int out_f32, int fp8, const float* scales, void* stream) {
  dtf::GemmArgs a{};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C;
  a.M = M; a.N = N; a.ldc = ldc;
  a.batch = 1; a.splitk = 1; a.alpha = 1.f; a.beta = 0.f; a.out_f32 = out_f32;
  if (N & 3) return -1;
  if (fp8) {  // the loaders move 16-B chunks: fp8 rows viewed as bf16_t pairs
    if ((K & 127) || (lda & 15) || (ldb & 15)) return -1;
    a.K = K / 2; a.lda = lda / 2; a.ldb = ldb / 2; a.scales = scales;
  } else {
    a.K = K; a.lda = lda; a.ldb = ldb;
  }
  a.kchunk = (a.K + dtf::BK - 1) / dtf::BK * dtf::BK;
  if (dtf::gemm4w_try(a, a_kouter ? dtf::OP_KOUTER : dtf::OP_KCONTIG, b_kouter ? dtf::OP_KOUTER : dtf::OP_KCONTIG,
                      (hipStream_t)stream, fp8))
    return -2;
  return (int)hipGetLastError();
}
