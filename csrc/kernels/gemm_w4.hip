// 256 x BN x 64 bf16 GEMM (BN 256 or 128), one wave per SIMD, 128 x BN/2 output per wave, gfx950.
//
// C = alpha * A . B^T (+ bias, activation, pre-activation side output, beta, activation backward, split-K slabs)
// for K-contiguous or K-outer operands: the dense forward (NT), data-gradient (NN) and weight-gradient (TN) forms.
//
// Why this shape (profiles/r5_gemm_vs_hipblaslt.txt): the 8-wave kernels (gemm256.hip, gemm8p.hip) give each wave a
// 128x64 output, so every 16x16x32 MFMA costs 24 KB of LDS fragment reads per wave per K-tile and the SIMD's two
// waves must hide each other's read bursts and barrier waits. Four waves with a 128x128 output each halve the LDS
// bytes per FLOP (32 KB per 128 MFMAs) and keep all 256 accumulators of a wave in the AGPR half of the unified
// register file (launch bounds: 1 wave per SIMD -> 512 registers), which leaves VGPRs for TWO fragment sets.
// With one wave per SIMD nothing else hides a stall, so the loop is software-pipelined by hand:
//   * K-tile t = two k-substeps (kk 0, 1). Each substep is cut into steps of 4 MFMAs, every step pinned by a
//     sched_barrier: during substep (t, 0) the steps also read the fragments of (t, 1); during substep (t, 1) they
//     read the fragments of (t+1, 0) and issue the LDS-DMA pieces of tile t+2. The DMA issue cost and the LDS reads
//     therefore sit between MFMAs instead of in bursts the MFMA pipe waits behind (ablation at 8192^3: no DMA
//     +17%, no reads +5%: tools/bench_gemm_w4.py --var).
//   * Both operands go straight into LDS (buffer_load ... lds, 16 B per lane), two stages. The loads of tile t+2
//     use the stage tile t vacates; ONE barrier per K-tile, between the two substeps: before it every wave has
//     retired its reads of stage t (lgkmcnt(0)) and waited for tile t+1 (vmcnt(0)), so it both publishes t+1 and
//     frees t. A tile's loads have a whole K-tile of MFMAs (~2k cycles) to land.
//   * Per-lane DMA state is loop-invariant (the tile's k goes into the SGPR offset, the LDS destination is M0), so a
//     piece is s_add + s_mov m0 + buffer_load.
//   * MFMAs are inline asm with a tied AGPR accumulator (w4_mfma), K-outer fragments inline-asm transposed reads
//     (w4_frag_kouter): see those for why.
// Epilogue: w4_epilogue (LDS-staged 16-B row stores for bf16 outputs).
// Reference op family: MatMul and its gradients in the TF graph the reference builds (SURVEY §2.4.b K3;
// /root/reference/trainer/task.py:137-139).
#include <cstdlib>

#include "gemm_w4.h"

namespace dtf {
namespace {


template <int BN>
struct W4Geo {
  static constexpr int JN = BN / 32;                    // B fragments per wave per substep (wave tile 128 x BN/2)
  static constexpr int B_BYTES = BN * BK * 2;           // B image of one stage
  static constexpr int STAGE = W4_A + B_BYTES;
  static constexpr int EPI = 256 * (BN + 8) * 2;        // the epilogue's staged bf16 C tile
  static constexpr int SMEM = EPI > 2 * STAGE ? EPI : 2 * STAGE;
  static constexpr int SMEM_ST = EPI + 16384 > 2 * STAGE ? EPI + 16384 : 2 * STAGE;  // + BN statistics partials
  static constexpr int NSTEP = 2 * JN;                  // 4-MFMA steps per substep (8 x JN MFMAs)
  static constexpr int NREAD = 8 + JN;                  // fragments per substep
  static constexpr int NG = 8 + BN / 32;                // LDS-DMA pieces per K-tile (A 8, B BN/32)
};

// acc += B . A on the MFMA, accumulating IN PLACE. Written as inline asm with a tied AGPR operand because the builtin
// lets the register allocator give the result a new register tuple: with all 256 AGPRs holding accumulators there is
// no free tuple, and hipcc then rotated accumulators through VGPRs (50-470 v_accvgpr moves per K-tile depending on
// unrelated code). hipcc pads no hazard inside asm (cdna_hip_programming.md §5.7): in this kernel no MFMA reads a
// result of the MFMA before it (consecutive MFMAs update different accumulators; an accumulator's next update is
// >= 31 MFMAs later), the A/B fragments come from LDS reads that are waited for (hipcc's own lgkmcnt, which does see
// the asm operands, or w4_lgkm0), and the first VALU read of an accumulator after the loop is padded by
// w4_mfma_drain().
__device__ __forceinline__ void w4_mfma(v4f& c, const v8bf& b, const v8bf& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(b), "v"(a));
}
// Transposed fragment of a K-outer [64 k][R cols] image (frag_kouter<R>'s addressing) read by inline-asm
// ds_read_b64_tr_b16: the builtin makes hipcc wait vmcnt for the in-flight LDS-DMA of the OTHER stage before every
// such read (it cannot tell the two apart), which drained the prefetch every K-tile (NN / TN 0.4-0.5x of NT). hipcc
// neither sees nor waits for these asm reads: the main loop waits lgkmcnt(0) before the MFMAs that consume them.
template <int R>
__device__ __forceinline__ v8bf w4_frag_kouter(const char* lds, int cb, int kk, int lane) {
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
template <int R, int MODE>
__device__ __forceinline__ v8bf w4_frag(const char* lds, int rb, int kk, int lane) {
  if constexpr (MODE == OP_KOUTER) return w4_frag_kouter<R>(lds, rb, kk, lane);
  else return frag_kcontig(lds, rb, kk, lane);
}
// Epilogue. gemm_core.h's generic gemm_epilogue serves every fused feature through runtime branches; instantiated
// over 64 fragments per lane it compiled to ~57k instructions with ~7.7k SGPR-spill lane moves and cost ~20 us per
// 256x256 tile (3x the tile's MFMA time at K = 768: tools/bench_gemm_w4.py --sweepk). This one covers what the dense
// layers need, nothing else (gemm_w4_try routes every other feature elsewhere):
//   bf16 C: alpha, bias, activation with its pre-activation side output (aux), beta (C += old C), activation
//           backward (dact: C *= act'(pre)); staged through LDS so every global access is a whole 16-B row chunk;
//   f32 C:  alpha, beta, split-K slabs; 16-B row pieces straight from the fragments.
// Lane l of wave (wm, wn) holds acc[i][j][r] = C[m0 + 128 wm + 16 i + (l & 15)][n0 + BN/2 wn + 16 j + 4 (l >> 4) + r].
// ST: also the training BatchNorm statistics of the stored bf16 values (a convolution forward's epilogue): one partial
// row per 256-row tile, stats[tile][0, N) = column sums, [N, 2N) = sums of squares, reduced over the tile's 16-lane
// row groups (DPP) and its two wave rows (LDS) in a fixed order.
template <int BN, bool ST = false>
__device__ __forceinline__ void w4_epilogue(const GemmArgs& a, v4f (&acc)[8][BN / 32], char* smem, int m0, int n0,
                                            int z, int bz) {
  constexpr int JN = BN / 32, WTN = BN / 2;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const long cbase = a.slab > 0 ? (long)z * a.slab : (long)bz * a.sC;
  const float alpha = a.alpha;
  if (a.out_f32) {
    float* C = reinterpret_cast<float*>(a.C) + cbase;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + wm * 128 + i * 16 + (lane & 15);
      if (m >= a.M) continue;
      float* crow = C + (long)m * a.ldc;
#pragma unroll
      for (int j = 0; j < JN; ++j) {
        const int n = n0 + wn * WTN + j * 16 + (lane >> 4) * 4;
        if (n >= a.N) continue;
        float4 v = make_float4(alpha * acc[i][j][0], alpha * acc[i][j][1], alpha * acc[i][j][2], alpha * acc[i][j][3]);
        if (a.beta != 0.f) {
          const float4 o = *reinterpret_cast<const float4*>(crow + n);
          v.x += a.beta * o.x; v.y += a.beta * o.y; v.z += a.beta * o.z; v.w += a.beta * o.w;
        }
        *reinterpret_cast<float4*>(crow + n) = v;
      }
    }
    return;
  }
  // bf16: fragments -> LDS tile [256][BN + 8] (16-B row pad) with bias / aux / activation applied
  constexpr int CS = BN + 8;
  bf16_t* ct = reinterpret_cast<bf16_t*>(smem);
  float csum[ST ? JN : 1][4], csq[ST ? JN : 1][4];
  if constexpr (ST) {
#pragma unroll
    for (int j = 0; j < JN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) csum[j][r] = csq[j][r] = 0.f;
  }
  float4 bias[JN];
#pragma unroll
  for (int j = 0; j < JN; ++j) {
    const int n = n0 + wn * WTN + j * 16 + (lane >> 4) * 4;
    bias[j] = (a.bias && n < a.N) ? *reinterpret_cast<const float4*>(a.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int ml = wm * 128 + i * 16 + (lane & 15);
    const int m = m0 + ml;
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      const int nl = wn * WTN + j * 16 + (lane >> 4) * 4;
      const int n = n0 + nl;
      float v[4] = {alpha * acc[i][j][0] + bias[j].x, alpha * acc[i][j][1] + bias[j].y,
                    alpha * acc[i][j][2] + bias[j].z, alpha * acc[i][j][3] + bias[j].w};
      if (a.aux && m < a.M && n < a.N) {
        uint2 o;
        o.x = pack2bf(v[0], v[1]);
        o.y = pack2bf(v[2], v[3]);
        *reinterpret_cast<uint2*>(a.aux + cbase + (long)m * a.ldc + n) = o;
      }
      if (a.act == 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
      } else if (a.act == 2) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = gelu_tanh(v[r]);
      }
      uint2 o;
      o.x = pack2bf(v[0], v[1]);
      o.y = pack2bf(v[2], v[3]);
      *reinterpret_cast<uint2*>(ct + ml * CS + nl) = o;
      if constexpr (ST) {
        if (m < a.M && !a.bnx) {
          const float f[4] = {__uint_as_float(o.x << 16), __uint_as_float(o.x & 0xffff0000u),
                              __uint_as_float(o.y << 16), __uint_as_float(o.y & 0xffff0000u)};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            csum[j][r] += f[r];
            csq[j][r] = fmaf(f[r], f[r], csq[j][r]);
          }
        }
      }
    }
  }
  float* red = reinterpret_cast<float*>(smem + 256 * CS * 2);  // [sum | sq][wm][BN]
  if constexpr (ST) {
#pragma unroll
    for (int j = 0; j < JN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float sv = row16_sum(csum[j][r]), qv = row16_sum(csq[j][r]);
        const int nl = wn * WTN + j * 16 + (lane >> 4) * 4 + r;
        if ((lane & 15) == 0 && !a.bnx) {
          red[wm * BN + nl] = sv;
          red[2 * BN + wm * BN + nl] = qv;
        }
      }
  }
  __syncthreads();
  // LDS -> C in whole 16-B chunks: a row is BN/8 consecutive threads
  constexpr int TPR = BN / 8, RPP = W4_THREADS / TPR;
  const int c8 = threadIdx.x % TPR, r0 = threadIdx.x / TPR;
  const int n = n0 + c8 * 8;
  if constexpr (ST) {
    float* prow = a.stats + (long)(m0 / 256) * 2 * a.N;
    if (!a.bnx) {
      for (int nl = threadIdx.x; nl < BN; nl += W4_THREADS) {
        const int nn = n0 + nl;
        if (nn < a.N) {
          prow[nn] = red[nl] + red[BN + nl];
          prow[a.N + nn] = red[2 * BN + nl] + red[3 * BN + nl];
        }
      }
    } else {
      // data gradient of a BatchNorm(+ReLU) output (bnx: the BN input, bnmask: its ReLU bits, bnmean): the BN
      // backward reduction of the stored values, sum dz and sum dz * (x - mean) with dz = the masked gradient, taken
      // from whole 16-B chunks in the store pass; the RPP threads of a chunk column are folded in a fixed order
      float bs[8], bq[8], mu[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) bs[r] = bq[r] = mu[r] = 0.f;
      bf16_t* C = reinterpret_cast<bf16_t*>(a.C) + cbase;
      if (n < a.N) {
        const float4 m0v = *reinterpret_cast<const float4*>(a.bnmean + n);
        const float4 m1v = *reinterpret_cast<const float4*>(a.bnmean + n + 4);
        mu[0] = m0v.x; mu[1] = m0v.y; mu[2] = m0v.z; mu[3] = m0v.w;
        mu[4] = m1v.x; mu[5] = m1v.y; mu[6] = m1v.z; mu[7] = m1v.w;
#pragma unroll 4
        for (int it = 0; it < 256 / RPP; ++it) {
          const int ml = r0 + RPP * it;
          const int m = m0 + ml;
          if (m >= a.M) break;
          const uint4 val = *reinterpret_cast<const uint4*>(ct + ml * CS + c8 * 8);
          const long e = (long)m * a.ldc + n;
          *reinterpret_cast<uint4*>(C + e) = val;
          const uint4 xr = *reinterpret_cast<const uint4*>(a.bnx + e);
          const uint32_t bits = a.bnmask ? (uint32_t)a.bnmask[e >> 3] : 0xFFu;  // e % 8 == 0
          const uint32_t vw[4] = {val.x, val.y, val.z, val.w}, xw[4] = {xr.x, xr.y, xr.z, xr.w};
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int r = 2 * q + h;
              const float dv = __uint_as_float(h ? (vw[q] & 0xffff0000u) : (vw[q] << 16));
              const float xv = __uint_as_float(h ? (xw[q] & 0xffff0000u) : (xw[q] << 16));
              const float dz = ((bits >> r) & 1u) ? dv : 0.f;
              bs[r] += dz;
              bq[r] = fmaf(dz, xv - mu[r], bq[r]);
            }
        }
      }
      float* red2 = reinterpret_cast<float*>(smem + 256 * CS * 2);  // [thread][sum 8 | sq 8]
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        red2[threadIdx.x * 16 + r] = bs[r];
        red2[threadIdx.x * 16 + 8 + r] = bq[r];
      }
      __syncthreads();
      for (int nl = threadIdx.x; nl < BN; nl += W4_THREADS) {
        const int nn = n0 + nl;
        if (nn >= a.N) continue;
        float sv = 0.f, qv = 0.f;
#pragma unroll
        for (int k = 0; k < RPP; ++k) {
          const int t = (nl >> 3) + k * TPR;
          sv += red2[t * 16 + (nl & 7)];
          qv += red2[t * 16 + 8 + (nl & 7)];
        }
        prow[nn] = sv;
        prow[a.N + nn] = qv;
      }
      return;
    }
  }
  if (n >= a.N) return;
  bf16_t* C = reinterpret_cast<bf16_t*>(a.C) + cbase;
  if (a.beta == 0.f && !a.dact && m0 + 256 <= a.M) {
    w4_store_rows<BN, 256>(ct, C + (long)m0 * a.ldc + n, a.ldc, r0, c8);
    return;
  }
#pragma unroll 4
  for (int it = 0; it < 256 / RPP; ++it) {
    const int ml = r0 + RPP * it;
    const int m = m0 + ml;
    if (m >= a.M) break;
    uint4 val = *reinterpret_cast<const uint4*>(ct + ml * CS + c8 * 8);
    const long e = (long)m * a.ldc + n;
    if (a.beta != 0.f) {
      const uint4 old = *reinterpret_cast<const uint4*>(C + e);
      const uint32_t vw[4] = {val.x, val.y, val.z, val.w}, ow[4] = {old.x, old.y, old.z, old.w};
      uint32_t rw[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float f0 = __uint_as_float(vw[q] << 16) + a.beta * __uint_as_float(ow[q] << 16);
        const float f1 = __uint_as_float(vw[q] & 0xffff0000u) + a.beta * __uint_as_float(ow[q] & 0xffff0000u);
        rw[q] = pack2bf(f0, f1);
      }
      val = make_uint4(rw[0], rw[1], rw[2], rw[3]);
    }
    if (a.dact) val = dact8(val, *reinterpret_cast<const uint4*>(a.dact_src + e), a.dact);
    *reinterpret_cast<uint4*>(C + e) = val;
  }
}

// VAR (ablation builds for tools/bench_gemm_w4.py --var; 0 = the kernel): 1 no LDS-DMA in the loop, 2 no fragment
// reads in the loop (MFMAs on stale fragments), 3 both, 4 no epilogue — timing only, results are wrong for VAR != 0.
template <int AM, int BMODE, int BN, int VAR = 0>
__global__ void __launch_bounds__(W4_THREADS, 1) gemm_w4_kernel(GemmArgs a) {
  using G = W4Geo<BN>;
  constexpr int JN = G::JN, WTN = BN / 2, NSTEP = G::NSTEP, NREAD = G::NREAD, NG = G::NG;
  constexpr int SPR = JN / 4;  // steps per accumulator row
  constexpr bool ST = (VAR & 16) != 0;  // BN statistics epilogue (convolution forward)
  __shared__ __attribute__((aligned(16))) char smem[ST ? G::SMEM_ST : G::SMEM];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

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
  const int bz = z / a.splitk, sk = z % a.splitk;
  const int kbeg = sk * a.kchunk;
  const int kend = min(a.K, kbeg + a.kchunk);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  W4LoaderFor<256, AM> la;
  W4Loader<BN, BMODE> lb;
  la.init(a, a.A + (long)bz * a.sA, a.lda, m0, a.M, threadIdx.x);
  lb.init(a, a.B + (long)bz * a.sB, a.ldb, n0, a.N, threadIdx.x);
  // LDS byte address of this wave's 1 KiB slot of piece 0 in stage 0 (wave-uniform: a scalar)
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem +
                        (uint32_t)__builtin_amdgcn_readfirstlane(wave) * 1024u;

  v4f acc[8][JN];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
  v8bf fa0[8], fb0[JN], fa1[8], fb1[JN];
  // VAR bit 8: row sums of A (the fused bias gradient of a weight gradient, GemmArgs::rowsum): each A fragment
  // (16 rows x 32 k, 8 k per lane) is summed once per substep with 4 v_dot2c_f32_bf16 against 1.0 — VALU work that
  // issues beside the MFMAs, no extra LDS traffic
  constexpr bool RS = (VAR & 8) != 0;
  float rs[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) rs[i] = 0.f;

  // piece s (0..NG-1) of tile t's LDS-DMA: A instruction s, then B instruction s - 8. Tiles past the last one load
  // the last tile again (into the stage t would use, which nothing reads any more): no branch in the loop body.
  auto issue1 = [&](int t, int s) {
    const uint32_t st = lds0 + (uint32_t)((t & 1) * G::STAGE);
    const int k0 = kbeg + min(t, nk - 1) * BK;
    if (s < 8) la.issue1(k0, st, s);
    else lb.issue1(k0, st + W4_A, s - 8);
  };
  auto issue = [&](int t) {
#pragma unroll
    for (int s = 0; s < NG; ++s) issue1(t, s);
  };
  // fragment s (0..NREAD-1) of a k-substep: the B fragments, then the A fragments (the order the next substep's
  // MFMAs need them: its first SPR steps use every B fragment, steps SPR i .. the A fragment i)
  auto read1 = [&](v8bf (&fa)[8], v8bf (&fb)[JN], int t, int kk, int s) {
    const char* st = smem + (t & 1) * G::STAGE;
    if (s < JN) fb[s] = w4_frag<BN, BMODE>(st + W4_A, wn * WTN + s * 16, kk, lane);
    else fa[s - JN] = w4_frag<256, AM>(st, wm * 128 + (s - JN) * 16, kk, lane);
  };
  auto read = [&](v8bf (&fa)[8], v8bf (&fb)[JN], int t, int kk) {
#pragma unroll
    for (int s = 0; s < NREAD; ++s) read1(fa, fb, t, kk, s);
  };
  // MFMAs 4s .. 4s+3 of a k-substep (row i = s / SPR, columns 4 (s % SPR) ..)
  auto mma4 = [&](const v8bf (&fa)[8], const v8bf (&fb)[JN], int s) {
    const int i = s / SPR, j0 = (s % SPR) * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) w4_mfma(acc[i][j0 + j], fb[j0 + j], fa[i]);
    if constexpr (RS) {
      if (s % SPR == 0) {
        typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
        const bf2_t one = {(__bf16)1.0f, (__bf16)1.0f};
        const v8bf f = fa[i];
        float r = rs[i];
        r = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(f, f, 0, 1), one, r, false);
        r = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(f, f, 2, 3), one, r, false);
        r = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(f, f, 4, 5), one, r, false);
        r = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(f, f, 6, 7), one, r, false);
        rs[i] = r;
      }
    }
  };
  // the fragment reads of a substep go out in the first half of the next one's steps (NREAD over NSTEP/2 steps),
  // so the explicit lgkmcnt(0) ahead of the substep that consumes them finds them done
  auto reads_at = [&](v8bf (&fa)[8], v8bf (&fb)[JN], int t, int kk, int s) {
    constexpr int H = NSTEP / 2;
    if (s < H) {
#pragma unroll
      for (int r = s * NREAD / H; r < (s + 1) * NREAD / H; ++r) read1(fa, fb, t, kk, r);
    }
  };

  // prologue: tiles 0 and 1 in flight, wait for tile 0 (NG LDS-DMA instructions per thread per tile)
  if (nk > 0) issue(0);
  if (nk > 1) {
    issue(1);
    if constexpr (NG == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  w4_barrier();
  if (nk > 0) {
    read(fa0, fb0, 0, 0);
    if constexpr ((VAR & 2) != 0) read(fa1, fb1, 0, 1);
  }

  // Steady state (no branch inside the body: tiles past the end are still "issued", see issue1)
  for (int t = 0; t + 1 < nk; ++t) {
    w4_lgkm0();
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) {
      if constexpr (!(VAR & 2)) reads_at(fa1, fb1, t, 1, s);
      mma4(fa0, fb0, s);
      __builtin_amdgcn_sched_barrier(0);
    }
    // every wave: its reads of stage t retired (lgkmcnt), tile t+1 landed (vmcnt) -> stage t is free, t+1 visible
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    w4_barrier();
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) {
      if constexpr (!(VAR & 1)) {
#pragma unroll
        for (int g = s * NG / NSTEP; g < (s + 1) * NG / NSTEP; ++g) issue1(t + 2, g);
      }
      if constexpr (!(VAR & 2)) reads_at(fa0, fb0, t + 1, 0, s);
      mma4(fa1, fb1, s);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (nk > 0) {
    w4_lgkm0();
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) {
      reads_at(fa1, fb1, nk - 1, 1, s);
      mma4(fa0, fb0, s);
      __builtin_amdgcn_sched_barrier(0);
    }
    w4_lgkm0();
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) mma4(fa1, fb1, s);
  }
  w4_mfma_drain();
  if constexpr (RS) {  // lanes l, l^16, l^32, l^48 hold the same row's k-groups: fold them, lanes 0..15 write
    if (tile_n == 0 && wn == 0 && a.rowsum) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float v = rs[i];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        const int m = m0 + wm * 128 + i * 16 + lane;
        if (lane < 16 && m < a.M) a.rowsum[(long)z * a.M + m] = v;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // the epilogue reuses the LDS
  if constexpr ((VAR & 4) != 0) {  // ablation: no epilogue (one store of a value that depends on every accumulator)
    float x = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < JN; ++j) x += acc[i][j][0] + acc[i][j][3];
    if (x == 12345.f) reinterpret_cast<float*>(a.C)[threadIdx.x] = x;
    return;
  }
  w4_epilogue<BN, ST>(a, acc, smem, m0, n0, z, bz);
}

template <int AM, int BMODE, int BN, int VAR>
void w4_go(GemmArgs& a, hipStream_t st) {
  dim3 grid(a.tiles_m * a.tiles_n, 1, a.batch * a.splitk);
  hipLaunchKernelGGL((gemm_w4_kernel<AM, BMODE, BN, VAR>), grid, dim3(W4_THREADS), 0, st, a);
}

template <int BN, int VAR = 0>
void w4_launch(GemmArgs& a, int amode, int bmode, hipStream_t st) {
  a.tiles_m = cdiv(a.M, 256);
  a.tiles_n = cdiv(a.N, BN);
  if constexpr (VAR != 0) {  // ablation builds: NT only
    w4_go<OP_KCONTIG, OP_KCONTIG, BN, VAR>(a, st);
    return;
  }
  if (a.rowsum) {  // (gemm_w4_ok: K-outer operands, f32 out)
    w4_go<OP_KOUTER, OP_KOUTER, BN, 8>(a, st);
    return;
  }
  if (amode == OP_IM2COL_T) {  // (gemm_w4_ok: convolution forward, with or without BN statistics)
    if (a.stats) w4_go<OP_IM2COL_T, OP_KCONTIG, BN, 16>(a, st);
    else w4_go<OP_IM2COL_T, OP_KCONTIG, BN, 0>(a, st);
    return;
  }
  if (amode == OP_DGRAD_T) {  // stride-1 data gradient, with or without the BN-backward statistics
    if (a.stats) w4_go<OP_DGRAD_T, OP_KCONTIG, BN, 16>(a, st);
    else w4_go<OP_DGRAD_T, OP_KCONTIG, BN, 0>(a, st);
    return;
  }

  if (amode == OP_KCONTIG && bmode == OP_KCONTIG) w4_go<OP_KCONTIG, OP_KCONTIG, BN, VAR>(a, st);
  else if (amode == OP_KCONTIG) w4_go<OP_KCONTIG, OP_KOUTER, BN, VAR>(a, st);
  else if (bmode == OP_KCONTIG) w4_go<OP_KOUTER, OP_KCONTIG, BN, VAR>(a, st);
  else w4_go<OP_KOUTER, OP_KOUTER, BN, VAR>(a, st);
}

}  // namespace

// True if the 4-wave kernel can run C = A . B^T with these arguments: K % 64 == 0 per split, 16-B aligned operand
// rows, K-outer operands with row counts % 8 == 0, operands < 2 GiB, and only the epilogue features w4_epilogue has.
bool gemm_w4_ok(const GemmArgs& a, int amode, int bmode) {
  if (a.atomic_out || a.crm || a.bsrc || a.betamask || a.scales || a.q8 || a.q8T || a.q8col || a.zero_slot)
    return false;
  // BN statistics: convolution forward (IM2COL_T) or the BN-backward reduction of a data gradient (DGRAD_T + bnx);
  // bf16 out, nothing else in the epilogue, one tile row per stats row
  if (a.stats && ((amode != OP_IM2COL_T && amode != OP_DGRAD_T) || (amode == OP_DGRAD_T) != (a.bnx != nullptr) ||
                  a.out_f32 || a.beta != 0.f || a.bias || a.act || a.aux || a.dact || a.batch > 1 || a.splitk > 1 ||
                  (a.bnx && (a.N & 7))))
    return false;
  if (a.bnx && !a.stats) return false;
  if (amode == OP_IM2COL_T || amode == OP_DGRAD_T) {  // tap-uniform K-tiles, gathered tensor < 2 GiB, K-contiguous B
    const ConvGeom& g = a.g;
    const bool fwd = amode == OP_IM2COL_T;
    if (bmode != OP_KCONTIG || ((fwd ? g.C : g.Kout) & 63) || g.R * g.S > 32 ||
        (fwd ? (long)g.N * g.H * g.W * g.C : (long)g.N * g.P * g.Q * g.Kout) * 2 >= (1l << 31) ||
        (!fwd && (g.sh != 1 || g.sw != 1)) ||
        a.batch > 1 || a.splitk > 1 || a.out_f32 || (a.N & 7) || (a.ldc & 7) || ((uintptr_t)a.C & 15) ||
        (a.K % BK) || (a.ldb & 7) || ((uintptr_t)a.A & 15) || ((uintptr_t)a.B & 15) ||
        (long)a.N * a.ldb * 2 >= (1l << 31))
      return false;
    return true;
  }
  if (a.out_f32 ? (a.bias || a.act || a.aux || a.dact || (a.ldc & 3) || ((uintptr_t)a.C & 15))
                : ((a.N & 7) || (a.ldc & 7) || ((uintptr_t)a.C & 15)))
    return false;
  if ((amode != OP_KCONTIG && amode != OP_KOUTER) || (bmode != OP_KCONTIG && bmode != OP_KOUTER)) return false;
  if (a.rowsum && (!a.out_f32 || amode != OP_KOUTER || bmode != OP_KOUTER || a.batch > 1)) return false;
  if (a.kchunk % BK || a.K % BK || (a.lda & 7) || (a.ldb & 7)) return false;
  if (((uintptr_t)a.A & 15) || ((uintptr_t)a.B & 15)) return false;
  auto fits = [](long elems) { return elems * 2 < (1l << 31); };
  if (amode == OP_KCONTIG ? !fits((long)a.M * a.lda) : (!fits((long)a.K * a.lda) || (a.M & 7))) return false;
  if (bmode == OP_KCONTIG ? !fits((long)a.N * a.ldb) : (!fits((long)a.K * a.ldb) || (a.N & 7))) return false;
  return true;
}

// Launch on the 4-wave kernel with tile width bn (256 or 128). Returns 0 if launched, 1 if not eligible.
int gemm_w4_try(GemmArgs& a, int amode, int bmode, hipStream_t st, int bn) {
  if (!gemm_w4_ok(a, amode, bmode)) return 1;
  count_launch(bn == 128 ? LC_W4_128 : LC_W4_256);
  if (bn == 128) w4_launch<128>(a, amode, bmode, st);
  else w4_launch<256>(a, amode, bmode, st);
  return 0;
}

}  // namespace dtf

// Ablation builds (timing only): var 1..4, see gemm_w4_kernel; NT layout, bf16 out, tile width bn.
DTF_API int dtf_gemm_w4_var(const void* A, const void* B, void* C, int M, int N, int K, int var, int bn,
                            void* stream) {
  using namespace dtf;
  GemmArgs a{};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C;
  a.M = M; a.N = N; a.K = K; a.lda = K; a.ldb = K; a.ldc = N;
  a.batch = 1; a.splitk = 1; a.kchunk = K; a.alpha = 1.f;
  if ((N & 7) || (K % BK) || (bn != 128 && bn != 256)) return -1;
  hipStream_t st = (hipStream_t)stream;
  const int m = OP_KCONTIG;
  if (bn == 128) {
    if (var == 1) w4_launch<128, 1>(a, m, m, st);
    else if (var == 2) w4_launch<128, 2>(a, m, m, st);
    else if (var == 3) w4_launch<128, 3>(a, m, m, st);
    else if (var == 4) w4_launch<128, 4>(a, m, m, st);
    else w4_launch<128, 0>(a, m, m, st);
  } else {
    if (var == 1) w4_launch<256, 1>(a, m, m, st);
    else if (var == 2) w4_launch<256, 2>(a, m, m, st);
    else if (var == 3) w4_launch<256, 3>(a, m, m, st);
    else if (var == 4) w4_launch<256, 4>(a, m, m, st);
    else w4_launch<256, 0>(a, m, m, st);
  }
  return (int)hipGetLastError();
}

// Direct entry for benchmarks/tests: C[M][N] (bf16, or f32 with out_f32) = A . B^T on the 4-wave kernel with tile
// width bn (256 or 128), A [M][K] (or [K][M] with a_kouter), B [N][K] (or [K][N] with b_kouter).
DTF_API int dtf_gemm_w4(const void* A, const void* B, void* C, int M, int N, int K, long lda, long ldb, long ldc,
                        int a_kouter, int b_kouter, int out_f32, int bn, void* stream) {
  dtf::GemmArgs a{};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.batch = 1; a.splitk = 1; a.kchunk = K; a.alpha = 1.f; a.beta = 0.f; a.out_f32 = out_f32;
  if ((N & 3) || (K % dtf::BK)) return -1;
  if (dtf::gemm_w4_try(a, a_kouter ? dtf::OP_KOUTER : dtf::OP_KCONTIG, b_kouter ? dtf::OP_KOUTER : dtf::OP_KCONTIG,
                       (hipStream_t)stream, bn))
    return -2;
  return (int)hipGetLastError();
}
