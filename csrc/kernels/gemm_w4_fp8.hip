// 256 x BN x 128 fp8 GEMM (BN 256 or 128) on the block-scaled 32x32x64 MFMA, one wave per SIMD, gfx950.
//
// C = (s0 s1 alpha) * A_q . B_q^T (+ bias, activation with its pre-activation side output; f32 out with beta 0/1 and
// split-K slabs), A OCP e4m3 (activations / weights) or e5m2 (gradients), B e4m3, both K-contiguous: the fp8
// projections of ops/fp8.py (forward, data gradient, weight gradient through the transposing quantizer's copies).
//
// The 4-wave structure of gemm_w4.hip (read that header first) with fp8 operands: a K-tile is 128 bytes per row
// (128 fp8 k), the same LDS image and LDS-DMA loader as the bf16 kernel's 64-k tile, so the staged bytes per K-tile
// are unchanged while the MFMA work per K-tile doubles in k. The MFMA is v_mfma_scale_f32_32x32x64_f8f6f4 with unit
// block scales (E8M0 127): twice the cycles of the bf16 32x32x16 at 4x the k, i.e. 2x the bf16 FLOP rate
// (MI355X_MICROARCH.md, Matrix cores). 32x32 (not 16x16x128) because a 16x16x128 fragment is 32 B per lane per
// 16 rows: two fragment sets for a 128 x 128 wave tile would need 256 VGPRs next to the 256 accumulator AGPRs; a
// 32x32x64 fragment covers 32 rows with the same 32 B, so a k-substep (64 k) of the wave tile is 4 A + BN/64 B
// fragments = 64 VGPRs per set, exactly the bf16 kernel's budget (acc[4][BN/64] x 16 AGPRs = 256).
//   * K-tile t = two 64-k substeps; substep (t, 0) reads the fragments of (t, 1), substep (t, 1) those of (t+1, 0)
//     and issues the LDS-DMA pieces of tile t+2; steps of 2 MFMAs pinned by sched_barrier; one barrier per K-tile.
//   * Any assignment of the 64 k of a substep to the (2 lane groups x 32 bytes) of a fragment is a valid operand as
//     long as A and B use the same: lane (G = l >> 5, r = l & 31) takes bytes 64 kk + 32 G .. + 31 of its row, two
//     swizzled 16-B chunks (ds_read_b128 each).
// Output: lane l of wave (wm, wn) holds acc[i][j][4q + p] = C[m0 + 128 wm + 32 i + (l & 31)]
//                                                              [n0 + BN/2 wn + 32 j + 8 q + 4 (l >> 5) + p].
// Reference op family: the GPT-2-medium fp8 projections of BASELINE.json ("CDNA4 fp8 MFMA"); SURVEY §2.4.b K3f.
#include "gemm_w4.h"

namespace dtf {
namespace {

template <int BN>
struct W8Geo {
  static constexpr int JN = BN / 64;                    // B fragments (32 columns each) per wave per substep
  static constexpr int STAGE = W4_A + BN * 128;
  static constexpr int EPI = 256 * (BN + 8) * 2 + 16 * BN * 4;  // staged bf16 C tile + q8 column-sum partials
  static constexpr int SMEM = EPI > 2 * STAGE ? EPI : 2 * STAGE;
  static constexpr int NSTEP = 2 * JN;                  // 2-MFMA steps per substep (4 x JN MFMAs)
  static constexpr int NREAD = 4 + JN;                  // fragments per substep
  static constexpr int NG = 8 + BN / 32;                // LDS-DMA pieces per K-tile (A 8, B BN/32)
};

// 32 rows x 64 k fp8 fragment of substep kk of a [R][128 B] K-contiguous stage image (see the header comment).
// Inline-asm ds_read_b128: with two LDS-DMA pieces per step in flight hipcc cannot tell them from these reads and
// put vmcnt(0) ahead of every read (the prefetch drained 4x per K-tile); the main loop waits lgkmcnt(0) itself
// before the MFMAs that consume a fragment set.
typedef int v4i_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v8i w8_frag(const char* lds, int rb, int kk, int lane) {
  const int row = rb + (lane & 31), G = lane >> 5, sw = (row >> 1) & 7;
  const int c0 = 4 * kk + 2 * G;
  const uint32_t base = (uint32_t)(uintptr_t)LDS_PTR(char, lds + row * 128);
  v4i_t lo, hi;
  asm volatile("ds_read_b128 %0, %1" : "=v"(lo) : "v"(base + ((c0 ^ sw) << 4)));
  asm volatile("ds_read_b128 %0, %1" : "=v"(hi) : "v"(base + (((c0 + 1) ^ sw) << 4)));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// acc += B . A over 64 k, in place (inline asm with a tied AGPR tuple, as w4_mfma). Operand formats: B (first) e4m3,
// A (second, blgp) e4m3 (FA 0) or e5m2 (FA 1); both block scales are the register sc = 0x7f7f7f7f (2^0).
template <int FA>
__device__ __forceinline__ void w8_mfma(v16f& c, const v8i& b, const v8i& a, int sc) {
  if constexpr (FA == 0)
    asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0]"
                 : "+a"(c) : "v"(b), "v"(a), "v"(sc));
  else
    asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0] blgp:1"
                 : "+a"(c) : "v"(b), "v"(a), "v"(sc));
}
// a 32x32 MFMA runs 16 passes: pad the first VALU read of the last accumulators written
__device__ __forceinline__ void w8_mfma_drain() {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\t"
               "s_nop 7" ::: "memory");
}

template <int BN>
__device__ __forceinline__ void w8_epilogue(const GemmArgs& a, v16f (&acc)[4][BN / 64], char* smem, int m0, int n0,
                                            int z) {
  constexpr int JN = BN / 64, WTN = BN / 2;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const long cbase = a.slab > 0 ? (long)z * a.slab : 0;
  const float alpha = a.scales ? a.alpha * a.scales[0] * a.scales[1] : a.alpha;
  const int mr = lane & 31, nq = 4 * (lane >> 5);
  if (a.out_f32) {
    float* C = reinterpret_cast<float*>(a.C) + cbase;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm * 128 + i * 32 + mr;
      if (m >= a.M) continue;
      float* crow = C + (long)m * a.ldc;
#pragma unroll
      for (int j = 0; j < JN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int n = n0 + wn * WTN + j * 32 + 8 * q + nq;
          if (n >= a.N) continue;
          float4 v = make_float4(alpha * acc[i][j][4 * q], alpha * acc[i][j][4 * q + 1], alpha * acc[i][j][4 * q + 2],
                                 alpha * acc[i][j][4 * q + 3]);
          if (a.beta != 0.f) {
            const float4 o = *reinterpret_cast<const float4*>(crow + n);
            v.x += a.beta * o.x; v.y += a.beta * o.y; v.z += a.beta * o.z; v.w += a.beta * o.w;
          }
          *reinterpret_cast<float4*>(crow + n) = v;
        }
    }
    return;
  }
  // bf16: fragments -> LDS tile [256][BN + 8] with bias / aux / activation applied, then whole 16-B row chunks
  constexpr int CS = BN + 8;
  bf16_t* ct = reinterpret_cast<bf16_t*>(smem);
#pragma unroll
  for (int j = 0; j < JN; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int nl = wn * WTN + j * 32 + 8 * q + nq;
      const int n = n0 + nl;
      const float4 bias = (a.bias && n < a.N) ? *reinterpret_cast<const float4*>(a.bias + n)
                                              : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ml = wm * 128 + i * 32 + mr;
        const int m = m0 + ml;
        float v[4] = {alpha * acc[i][j][4 * q] + bias.x, alpha * acc[i][j][4 * q + 1] + bias.y,
                      alpha * acc[i][j][4 * q + 2] + bias.z, alpha * acc[i][j][4 * q + 3] + bias.w};
        if (a.aux && m < a.M && n < a.N) {
          uint2 o;
          o.x = pack2bf(v[0], v[1]);
          o.y = pack2bf(v[2], v[3]);
          *reinterpret_cast<uint2*>(a.aux + (long)m * a.ldc + n) = o;
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
      }
    }
  __syncthreads();
  // fp8 copies of the final bf16 values for the next fp8 layer (GemmArgs::q8*, as gemm256.hip's staged epilogue):
  // the delayed scale (block 0 publishes the one used), row-major copy, transposed copy and per-128-row column sums
  // from a column pass over the LDS tile, and the block's max |value| into the amax slot
  const bool q8on = a.q8 || a.q8T || a.q8col;
  const bool q8tp = a.q8T || a.q8col;
  const float q8fmax = a.q8fmt ? 57344.f : 448.f;
  float q8inv = 0.f, q8max = 0.f;
  if (q8on) {
    const float ap = a.q8amax_prev ? a.q8amax_prev[0] : 0.f;
    const float s8 = ap > 0.f ? ap / q8fmax : fmaxf(a.q8scale[0], 1e-30f);
    q8inv = 1.f / s8;
    if (a.q8used && blockIdx.x == 0 && blockIdx.z == 0 && threadIdx.x == 0) {
      a.q8used[0] = s8;
      if (a.q8used2) a.q8used2[0] = s8;
    }
  }
  auto q8v = [&](float f) { return fminf(fmaxf(f * q8inv, -q8fmax), q8fmax); };
  constexpr int TPR = BN / 8, RPP = W4_THREADS / TPR;
  const int c8 = threadIdx.x % TPR, r0 = threadIdx.x / TPR;
  const int n = n0 + c8 * 8;
  bf16_t* C = reinterpret_cast<bf16_t*>(a.C);
  if (n < a.N && !q8on && !a.dact && !a.no_c && m0 + 256 <= a.M) {
    w4_store_rows<BN, 256>(ct, C + (long)m0 * a.ldc + n, a.ldc, r0, c8);
  } else if (n < a.N) {
#pragma unroll 4
    for (int it = 0; it < 256 / RPP; ++it) {
      const int ml = r0 + RPP * it;
      const int m = m0 + ml;
      if (m >= a.M) break;
      const long e = (long)m * a.ldc + n;
      uint4 val = *reinterpret_cast<const uint4*>(ct + ml * CS + c8 * 8);
      if (a.dact) val = dact8(val, *reinterpret_cast<const uint4*>(a.dact_src + e), a.dact);
      if (!a.no_c) *reinterpret_cast<uint4*>(C + e) = val;
      if (q8on) {
        const uint32_t vw[4] = {val.x, val.y, val.z, val.w};
        float f[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          f[2 * q] = __uint_as_float(vw[q] << 16);
          f[2 * q + 1] = __uint_as_float(vw[q] & 0xffff0000u);
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) q8max = fmaxf(q8max, fabsf(f[r]));
        if (a.q8)
          *reinterpret_cast<uint2*>(a.q8 + (long)m * a.N + n) =
              make_uint2(q8pack4(a.q8fmt, q8v(f[0]), q8v(f[1]), q8v(f[2]), q8v(f[3])),
                         q8pack4(a.q8fmt, q8v(f[4]), q8v(f[5]), q8v(f[6]), q8v(f[7])));
        if (q8tp && a.dact) *reinterpret_cast<uint4*>(ct + ml * CS + c8 * 8) = val;  // the column pass's values
      }
    }
  }
  if (q8tp) {
    __syncthreads();
    // transposed copy + column sums from 16-row x 8-column blocks: a thread reads its block's 16 rows as 16-B LDS
    // chunks (consecutive threads: consecutive chunks of a row), writes the 8 transposed 16-B pieces and its 8
    // partial column sums (row order within the block) to LDS; the sums of each 128-row half are then folded over
    // the 8 blocks in block order (deterministic)
    constexpr int NC8 = BN / 8;
    float* part = reinterpret_cast<float*>(smem + 256 * CS * 2);  // [16 row blocks][BN]
    for (int task = threadIdx.x; task < 16 * NC8; task += W4_THREADS) {
      const int cc = task % NC8, rg = task / NC8;
      uint4 v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = *reinterpret_cast<const uint4*>(ct + (rg * 16 + i) * CS + cc * 8);
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        float f[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const uint32_t w = c < 2 ? v[i].x : c < 4 ? v[i].y : c < 6 ? v[i].z : v[i].w;
          f[i] = __uint_as_float((c & 1) ? (w & 0xffff0000u) : (w << 16));
        }
        float cs = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) cs += f[i];
        part[rg * BN + cc * 8 + c] = cs;
        const int nn = n0 + cc * 8 + c;
        if (a.q8T && nn < a.N) {
          uint4 qv;
          qv.x = q8pack4(a.q8fmt, q8v(f[0]), q8v(f[1]), q8v(f[2]), q8v(f[3]));
          qv.y = q8pack4(a.q8fmt, q8v(f[4]), q8v(f[5]), q8v(f[6]), q8v(f[7]));
          qv.z = q8pack4(a.q8fmt, q8v(f[8]), q8v(f[9]), q8v(f[10]), q8v(f[11]));
          qv.w = q8pack4(a.q8fmt, q8v(f[12]), q8v(f[13]), q8v(f[14]), q8v(f[15]));
          *reinterpret_cast<uint4*>(a.q8T + (long)nn * a.M + m0 + rg * 16) = qv;
        }
      }
    }
    if (a.q8col) {
      __syncthreads();
      for (int t = threadIdx.x; t < 2 * BN; t += W4_THREADS) {
        const int nl = t % BN, h = t / BN;
        if (n0 + nl >= a.N) continue;
        float cs = 0.f;
#pragma unroll
        for (int rg = 0; rg < 8; ++rg) cs += part[(h * 8 + rg) * BN + nl];
        a.q8col[(long)((m0 + h * 128) >> 7) * a.N + n0 + nl] = cs;
      }
    }
  }
  if (q8on && a.q8amax) {  // block max |value| -> the amax slot (relaxed check first: most blocks lose)
    float mx = q8max;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);
    if (lane == 0) red[wave] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
      for (int i = 1; i < W4_THREADS / 64; ++i) mx = fmaxf(mx, red[i]);
      unsigned int* am = reinterpret_cast<unsigned int*>(a.q8amax);
      const unsigned int cur = __hip_atomic_load(am, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__float_as_uint(mx) > cur) atomicMax(am, __float_as_uint(mx));
    }
  }
}

// FA: A operand format (0 e4m3, 1 e5m2). GemmArgs in the fp8 entry points' convention: K, kchunk, lda, ldb in 2-byte
// units (a 64-unit K-tile = 128 fp8).
template <int BN, int FA>
__global__ void __launch_bounds__(W4_THREADS, 1) gemm_w4_fp8_kernel(GemmArgs a) {
  using G = W8Geo<BN>;
  constexpr int JN = G::JN, WTN = BN / 2, NSTEP = G::NSTEP, NREAD = G::NREAD, NG = G::NG;
  constexpr int SPR = JN / 2 > 0 ? JN / 2 : 1;  // steps per accumulator row (2 MFMAs per step)
  __shared__ __attribute__((aligned(16))) char smem[G::SMEM];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  if (a.zero_slot && blockIdx.x == 0 && blockIdx.z == 0 && threadIdx.x == 0) *a.zero_slot = 0.f;

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
  const int sk = z % a.splitk;
  const int kbeg = sk * a.kchunk;
  const int kend = min(a.K, kbeg + a.kchunk);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  W4Loader<256, OP_KCONTIG> la;
  W4Loader<BN, OP_KCONTIG> lb;
  la.init(a, a.A, a.lda, m0, a.M, threadIdx.x);
  lb.init(a, a.B, a.ldb, n0, a.N, threadIdx.x);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem +
                        (uint32_t)__builtin_amdgcn_readfirstlane(wave) * 1024u;
  const int sc = 0x7f7f7f7f;

  v16f acc[4][JN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  v8i fa0[4], fb0[JN], fa1[4], fb1[JN];

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
  auto read1 = [&](v8i (&fa)[4], v8i (&fb)[JN], int t, int kk, int s) {
    const char* st = smem + (t & 1) * G::STAGE;
    if (s < JN) fb[s] = w8_frag(st + W4_A, wn * WTN + s * 32, kk, lane);
    else fa[s - JN] = w8_frag(st, wm * 128 + (s - JN) * 32, kk, lane);
  };
  auto read = [&](v8i (&fa)[4], v8i (&fb)[JN], int t, int kk) {
#pragma unroll
    for (int s = 0; s < NREAD; ++s) read1(fa, fb, t, kk, s);
  };
  // MFMAs 2s, 2s+1 of a substep (row i = s / SPR, columns 2 (s % SPR) ..)
  auto mma2 = [&](const v8i (&fa)[4], const v8i (&fb)[JN], int s) {
    const int i = s / SPR, j0 = (s % SPR) * 2;
#pragma unroll
    for (int j = 0; j < 2; ++j) w8_mfma<FA>(acc[i][j0 + j], fb[j0 + j], fa[i], sc);
  };
  auto reads_at = [&](v8i (&fa)[4], v8i (&fb)[JN], int t, int kk, int s) {
    constexpr int H = NSTEP / 2;
    if (s < H) {
#pragma unroll
      for (int r = s * NREAD / H; r < (s + 1) * NREAD / H; ++r) read1(fa, fb, t, kk, r);
    }
  };

  if (nk > 0) issue(0);
  if (nk > 1) {
    issue(1);
    if constexpr (NG == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  w4_barrier();
  if (nk > 0) read(fa0, fb0, 0, 0);

  for (int t = 0; t + 1 < nk; ++t) {
    w4_lgkm0();
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) {
      reads_at(fa1, fb1, t, 1, s);
      mma2(fa0, fb0, s);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    w4_barrier();
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) {
#pragma unroll
      for (int g = s * NG / NSTEP; g < (s + 1) * NG / NSTEP; ++g) issue1(t + 2, g);
      reads_at(fa0, fb0, t + 1, 0, s);
      mma2(fa1, fb1, s);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (nk > 0) {
    w4_lgkm0();
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) {
      reads_at(fa1, fb1, nk - 1, 1, s);
      mma2(fa0, fb0, s);
      __builtin_amdgcn_sched_barrier(0);
    }
    w4_lgkm0();
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) mma2(fa1, fb1, s);
  }
  w8_mfma_drain();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  w8_epilogue<BN>(a, acc, smem, m0, n0, z);
}

}  // namespace

// True if the fp8 4-wave kernel can run these arguments (fp8 entry-point convention: 2-byte units).
bool gemm_w4_fp8_ok(const GemmArgs& a) {
  if (a.atomic_out || a.stats || a.bnx || a.crm || a.bsrc || a.betamask || a.batch > 1) return false;
  const bool q8 = a.q8 || a.q8T || a.q8col;
  if (a.out_f32 ? (a.bias || a.act || a.aux || a.dact || q8 || (a.ldc & 3) || ((uintptr_t)a.C & 15))
                : (a.beta != 0.f || (a.N & 7) || (a.ldc & 7) || ((uintptr_t)a.C & 15) || ((uintptr_t)a.dact_src & 15)))
    return false;
  if (q8 && ((a.M & 255) || !a.q8scale || a.slab > 0 || (a.q8 && ((uintptr_t)a.q8 & 7)) ||
             (a.q8T && ((uintptr_t)a.q8T & 15)) || (a.dact && a.ldc != a.N)))
    return false;
  if (a.kchunk % BK || a.K % BK || (a.lda & 7) || (a.ldb & 7)) return false;
  if (((uintptr_t)a.A & 15) || ((uintptr_t)a.B & 15)) return false;
  auto fits = [](long units) { return units * 2 < (1l << 31); };
  return fits((long)a.M * a.lda) && fits((long)a.N * a.ldb);
}

// Launch with tile width bn (256 / 128); fp8: 1 = A e4m3, 2 = A e5m2. Returns 0 if launched, 1 if not eligible.
int gemm_w4_fp8_try(GemmArgs& a, int fp8, hipStream_t st, int bn) {
  if (!gemm_w4_fp8_ok(a) || (bn != 128 && bn != 256)) return 1;
  count_launch(bn == 128 ? LC_W4F8_128 : LC_W4F8_256);
  a.tiles_m = cdiv(a.M, 256);
  a.tiles_n = cdiv(a.N, bn);
  dim3 grid(a.tiles_m * a.tiles_n, 1, a.splitk);
  if (bn == 256) {
    if (fp8 == 2) hipLaunchKernelGGL((gemm_w4_fp8_kernel<256, 1>), grid, dim3(W4_THREADS), 0, st, a);
    else hipLaunchKernelGGL((gemm_w4_fp8_kernel<256, 0>), grid, dim3(W4_THREADS), 0, st, a);
  } else {
    if (fp8 == 2) hipLaunchKernelGGL((gemm_w4_fp8_kernel<128, 1>), grid, dim3(W4_THREADS), 0, st, a);
    else hipLaunchKernelGGL((gemm_w4_fp8_kernel<128, 0>), grid, dim3(W4_THREADS), 0, st, a);
  }
  return 0;
}

}  // namespace dtf

// Direct entry for benchmarks/tests: C[M][N] (bf16, or f32 with out_f32) = A_q[M][K] . B_q[N][K]^T (fp8 bytes, lda /
// ldb in bytes), unit scales, A e4m3 (fmt_a 0) or e5m2 (1), tile width bn.
DTF_API int dtf_gemm_w4_fp8(const void* A, const void* B, void* C, int M, int N, int K, long lda, long ldb, long ldc,
                            int fmt_a, int out_f32, int bn, void* stream) {
  if ((K & 127) || (lda & 15) || (ldb & 15) || (N & 7)) return -1;
  dtf::GemmArgs a{};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C;
  a.M = M; a.N = N; a.K = K / 2; a.lda = lda / 2; a.ldb = ldb / 2; a.ldc = ldc;
  a.batch = 1; a.splitk = 1; a.kchunk = a.K; a.alpha = 1.f; a.beta = 0.f; a.out_f32 = out_f32;
  if (dtf::gemm_w4_fp8_try(a, fmt_a == 1 ? 2 : 1, (hipStream_t)stream, bn)) return -2;
  return (int)hipGetLastError();
}
