// 256x256x64 bf16 GEMM for large K-contiguous problems (C = alpha * A B^T (+ beta C, bias, act)), gfx950.
//
// The register-staged 128x128 kernel (gemm_core.h) tops out near the ~0.9 PF ceiling of a one-barrier-per-
// K-step structure; this kernel is the 1-block/CU pipelined form:
//  * 8 waves (2 M x 4 N), each owning a 128x64 output tile = 8x4 MFMA 16x16 fragments (128 accumulators);
//  * A and B tiles staged straight into LDS by global_load_lds (16 B/lane, no VGPR round trip), double-
//    buffered, each K-tile split into four half-tiles A0 A1 B0 B1 (128 rows x 64 k, 16 KiB); the LDS image is
//    lane-linear, so the bank-conflict XOR swizzle is applied to the per-lane SOURCE address and undone on
//    the ds_read side (same involution);
//  * every K-tile runs as 4 phases, one per output quadrant (A0B0, A0B1, A1B1, A1B0); each half is read
//    from LDS once per tile. Each phase issues one half-tile of the prefetch stream, so 2-3 half-tiles stay
//    in flight across the raw s_barriers; the only waits are counted `s_waitcnt vmcnt(N)` (never 0 inside
//    the loop), and the two 4-wave groups run one phase apart so MFMA work of one group covers the LDS
//    reads / barrier waits of the other on every SIMD (schedule and hazard distances: see the K-loop).
// K-outer operands (stored [K][rows], e.g. dY^T and X^T of a weight gradient, or W of a data gradient) use
// a [64 k][128 rows] half image (256-B k-rows, 16-B chunks XOR-swizzled by (k & 3) << 1) filled by the same
// lane-linear glds and read with ds_read_b64_tr_b16. Split-K writes f32 slabs (blockIdx.z = batch*splitk +
// split) reduced by dtf_sum_rows.
// Requirements (host-checked): K % 64 == 0 per split, 16-B aligned rows (lda, ldb % 8 == 0), K-outer
// operands need their row count % 8 == 0. M, N arbitrary (edge rows clamped on load, masked on store).
#include "gemm_core.h"

namespace dtf {
namespace {

constexpr int NT2 = 512;
constexpr int HALF = 128 * 128;  // bytes of one A half-tile image (128 rows x 64 bf16)
// B half-tile image: BN/2 rows x 64 bf16; buffer = A0 | A1 | B0 | B1
template <int BN> constexpr int half_b() { return BN * 64; }
template <int BN> constexpr int buf_bytes() { return 2 * HALF + 2 * half_b<BN>(); }
template <int BN> constexpr int half_off(int h) { return h < 2 ? h * HALF : 2 * HALF + (h - 2) * half_b<BN>(); }

// LDS image row -> block-tile row (A: two 64-row slices per M-wave; B: two BN/8-col slices per N-wave)
__device__ __forceinline__ int a_row(int r, int h) { return (r >> 6) * 128 + h * 64 + (r & 63); }
template <int BN>
__device__ __forceinline__ int b_row(int r, int h) {
  constexpr int S = BN / 8;  // columns of one N-wave in one half
  return (r / S) * (2 * S) + h * S + (r % S);
}

// K-outer half image [64 k][128 cols]: physical 16-B chunk of logical chunk c in k-row k. A transposed fragment read
// (frag_ko) has its 4 lane groups G on k-rows 8 apart; every 256-B k-row starts on bank 0, so bit 3 of k moves the
// odd groups' rows to the other 32 banks (without it, groups 0 and 1 hit the same banks: 50% of the LDS cycles of a
// K-outer x K-outer GEMM were bank-conflict cycles, SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, profiles/)
__device__ __forceinline__ int ko_swz(int k) { return ((k & 3) << 1) | (((k >> 3) & 1) << 3); }
// transposed fragment of a K-outer half: lane (G, i) gets col rb + i, k = 32 kk + 8 G + 0..7
__device__ __forceinline__ v8bf frag_ko(const char* lds, int rb, int kk, int lane) {
  const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  v4s r[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = 32 * kk + 8 * G + 4 * h + q, g = (rb >> 2) + p;
    r[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        LDS_PTR(v4s, lds + k * 256 + (((g >> 1) ^ ko_swz(k)) << 4) + (g & 1) * 8));
  }
  v8s both = __builtin_shufflevector(r[0], r[1], 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(v8bf, both);
}

__device__ __forceinline__ void glds16(const bf16_t* g, char* lds) {
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

__device__ __forceinline__ void barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// BN = 256 (each wave 128x64: 8x4 fragments) or 128 (each wave 128x32: 8x2 fragments; 256x128 tiles fill the
// chip where 256x256 would leave half of it idle, e.g. M = 8192 x N = 1024)
template <int AM, int BMD, int FP8 = 0, int BN = 256, bool AUXD = (FP8 == 0)>
__global__ void __launch_bounds__(NT2, 1) gemm256_kernel(GemmArgs a) {
  constexpr int BUF = buf_bytes<BN>();
  constexpr int JN = BN / 128;           // B fragments per wave per half (and glds instructions per B half)
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 2, wc = w & 3;

  // ---- block -> tile (XCD-aware bijective remap, grouped order) ----
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
  const bf16_t* Ap = a.A + (long)bz * a.sA;
  const bf16_t* Bp = a.B + (long)bz * a.sB;

  // ---- per-thread glds sources: half h (0,1 = A0,A1; 2,3 = B0,B1), instruction u; advance per K-tile ----
  const bf16_t* src[4][2];
  long kstep[4];
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const bool isA = h < 2;
    const bool ko = isA ? (AM == OP_KOUTER) : (BMD == OP_KOUTER);
    const bf16_t* P = isA ? Ap : Bp;
    const long ld = isA ? a.lda : a.ldb;
    const int lim = isA ? a.M : a.N;
    const int o0 = isA ? m0 : n0;
    const bool narrow = !isA && BN == 128;  // 64-row B half
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (!ko) {  // [rows][64 k] image, 8 lanes per 128-B row
        const int r = 8 * (u * 8 + w) + (lane >> 3);
        const int lc = (lane & 7) ^ ((r >> 1) & 7);
        const int g = min(o0 + (isA ? a_row(r, h) : b_row<BN>(r, h - 2)), lim - 1);
        src[h][u] = P + (long)g * ld + kbeg + lc * 8;
      } else if (!narrow) {  // [64 k][128 cols] image, 16 lanes per 256-B k-row
        const int k = 4 * (u * 8 + w) + (lane >> 4);
        const int lc = (lane & 15) ^ ko_swz(k);
        const int col = lc * 8;
        const int g = min(o0 + (isA ? a_row(col, h) : b_row<BN>(col, h - 2)), lim - 8);
        src[h][u] = P + (long)(kbeg + k) * ld + g;
      } else {  // [64 k][64 cols] image, 8 lanes per 128-B k-row (gemm_core.h K-outer swizzle, R = 64)
        const int k = 8 * (u * 8 + w) + (lane >> 3);
        const int lc = (lane & 7) ^ (kouter_swz<64>(k & 63) << 1);
        const int g = min(o0 + b_row<BN>(lc * 8, h - 2), lim - 8);
        src[h][u] = P + (long)(kbeg + (k & 63)) * ld + g;
      }
    }
    kstep[h] = ko ? (long)BK * ld : (long)BK;
  }
  auto issue = [&](int h, int t, int buf) {
    const long ko = (long)t * kstep[h];
    char* d = smem + buf * BUF + half_off<BN>(h) + w * 1024;
    glds16(src[h][0] + ko, d);
    if (h < 2 || JN == 2) glds16(src[h][1] + ko, d + 8 * 1024);
  };

  v4f acc[8][2 * JN];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 2 * JN; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
  // bf16: 2 k-substeps of 32 per 64-wide K-tile (16-B fragments); fp8 (OCP e4m3, K-tile = 128 bytes, same LDS image)
  // fp8: ONE block-scaled 16x16x128 MFMA per fragment pair and K-tile (32-B fragments, 2x the bf16 FLOP rate)
  using FragT = typename std::conditional<FP8 != 0, v8i, v8bf>::type;
  constexpr int KS = FP8 ? 1 : 2;
  FragT fa[4][KS], fb0[JN][KS], fb1[JN][KS];

  auto read_a = [&](int buf, int h) {
    const char* base = smem + buf * BUF + half_off<BN>(h);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        if constexpr (FP8) fa[i][kk] = frag_fp8x128(base, wr * 64 + i * 16, lane);
        else if constexpr (AM == OP_KOUTER) fa[i][kk] = frag_ko(base, wr * 64 + i * 16, kk, lane);
        else fa[i][kk] = frag_kcontig(base, wr * 64 + i * 16, kk, lane);
      }
  };
  auto read_b = [&](FragT (&fb)[JN][KS], int buf, int h) {
    const char* base = smem + buf * BUF + half_off<BN>(2 + h);
#pragma unroll
    for (int j = 0; j < JN; ++j)
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        const int cb = wc * (BN / 8) + j * 16;
        if constexpr (FP8) fb[j][kk] = frag_fp8x128(base, cb, lane);
        else if constexpr (BMD == OP_KOUTER && BN == 128) fb[j][kk] = frag_kouter<64>(base, cb, kk, lane);
        else if constexpr (BMD == OP_KOUTER) fb[j][kk] = frag_ko(base, cb, kk, lane);
        else fb[j][kk] = frag_kcontig(base, cb, kk, lane);
      }
  };
  auto mma = [&](const FragT (&fb)[JN][KS], int ha, int hb) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < KS; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          if constexpr (FP8)
            acc[ha * 4 + i][hb * JN + j] = mfma_fp8_ab<FP8>(fb[j][kk], fa[i][kk], acc[ha * 4 + i][hb * JN + j]);
          else
            acc[ha * 4 + i][hb * JN + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                fb[j][kk], fa[i][kk], acc[ha * 4 + i][hb * JN + j], 0, 0, 0);
        }
    __builtin_amdgcn_s_setprio(0);
  };

  // Schedule (phase index 4t+p, p = 0..3 for quadrants A0B0, A0B1, A1B1, A1B0). Each half of tile t is read
  // from LDS once (B0 stays in registers for phase 3): A0,B0 at 4t, B1 at 4t+1, A1 at 4t+2. Prefetch issues:
  // A0(t+1) at 4t-1, B0(t+1) at 4t, B1(t+1) at 4t+1, A1(t+1) at 4t+2 — each >= 2 phases after the previous
  // content of its half was last read (WAR) and >= 3 before its first read (RAW). The two 4-wave groups run
  // one phase apart (group 1 passes one extra barrier first), so group 1's MFMAs overlap group 0's LDS reads
  // and barrier waits on every SIMD. With that stagger a barrier must also publish the NEXT phase's halves,
  // so the wait before phase x covers the halves due at x and x+1: vmcnt(4|4|6|4).
  // counted waits: an A half is 2 glds per thread, a B half JN; the wait before phase x leaves in flight exactly
  // the halves issued after the ones due at phases x and x+1 (JN = 2: 6 | 4 4 6 4)
  constexpr int WP = JN + 4, W0 = 4, W1 = 2 + JN, W2 = 2 + 2 * JN, W3 = JN + 2;
  const int nk = kend > kbeg ? (kend - kbeg) / BK : 0;
  if (nk > 0) {
    issue(0, 0, 0);
    issue(2, 0, 0);
    issue(3, 0, 0);
    issue(1, 0, 0);
  }
  if (nk > 1) issue(0, 1, 1);
  if (wr == 1) {
    if (nk > 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WP) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();
  }
  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1, nb = buf ^ 1;
    const bool more = t + 1 < nk, more2 = t + 2 < nk;
    // phase 0: (A0, B0)
    if (more) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(W0) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();
    read_a(buf, 0);
    read_b(fb0, buf, 0);
    if (more) issue(2, t + 1, nb);
    mma(fb0, 0, 0);
    // phase 1: (A0, B1)
    if (more) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(W1) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();
    read_b(fb1, buf, 1);
    if (more) issue(3, t + 1, nb);
    mma(fb1, 0, 1);
    // phase 2: (A1, B1)
    if (more) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(W2) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();
    read_a(buf, 1);
    if (more) issue(1, t + 1, nb);
    mma(fb1, 1, 1);
    // phase 3: (A1, B0) from registers
    if (more) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(W3) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();
    if (more2) issue(0, t + 2, buf);
    mma(fb0, 1, 0);
  }
  if (wr == 0) barrier();

  // ---- epilogue (no glds outstanding: the last tile drained with vmcnt(0)) ----
  const float alpha = a.scales ? a.alpha * a.scales[0] * a.scales[1] : a.alpha;
  const long cbase = a.slab > 0 ? (long)z * a.slab : (long)bz * a.sC;
  // bf16 outputs (and the optional pre-activation side output) go through LDS, one 128-row half of the tile at
  // a time, so the global stores are whole 16-B chunks of 512-B row segments instead of 8-B pieces of 16 rows
  // beta (bf16 C, no aux/act): the old C is added to the bf16-rounded product in the store pass — exactly the
  // unfused GEMM followed by an elementwise add (a residual gradient joined in the branch's data-gradient GEMM)
  const bool staged = !a.out_f32 && (a.beta == 0.f || (!a.aux && !a.act)) && a.slab == 0 && !(a.N & 7) &&
                      !(a.ldc & 7) && !(reinterpret_cast<uintptr_t>(a.C) & 15) &&
                      !(reinterpret_cast<uintptr_t>(a.aux) & 15);
  if (staged) {
    constexpr int CS = BN + 8;  // LDS row stride (elements): conflict-free 8-B fragment writes
    bf16_t* ct = reinterpret_cast<bf16_t*>(smem);
    // fp8 copies of C (GemmArgs::q8*): the delayed scale, and this thread's running max |value|
    const bool q8on = a.q8 || a.q8T || a.q8col;
    const bool q8tp = a.q8T || a.q8col;  // the column pass over the LDS tile
    const float q8fmax = a.q8fmt ? 57344.f : 448.f;
    float q8inv = 0.f, q8max = 0.f;
    if (q8on) {
      const float ap = a.q8amax_prev ? a.q8amax_prev[0] : 0.f;
      const float sc = ap > 0.f ? ap / q8fmax : fmaxf(a.q8scale[0], 1e-30f);
      q8inv = 1.f / sc;
      if (a.q8used && blockIdx.x == 0 && blockIdx.z == 0 && tid == 0) {
        a.q8used[0] = sc;
        if (a.q8used2) a.q8used2[0] = sc;
      }
    }
    auto q8v = [&](float f) { return fminf(fmaxf(f * q8inv, -q8fmax), q8fmax); };
    const bool aux_nt = a.aux_nt & 1;
    // aux_nt bit 1: the pre-activation side output is stored straight from the fragments in the main pass (8-B
    // pieces, merged in L2) instead of a second LDS-staged pass
    // (fp8 kernels: a separate instantiation, AUXD — its extra live values cost 4 VGPR spills)
    const bool aux_direct = AUXD && (a.aux_nt & 2) && a.aux;
    // the tile's bias columns staged in LDS (past the C staging area) once, instead of a global float4 load per
    // row fragment in the loop below
    float* sbias = reinterpret_cast<float*>(smem + 128 * CS * 2);
    static_assert(128 * CS * 2 + BN * 4 <= 2 * BUF, "bias staging must fit past the C tile");
    __syncthreads();  // every wave is done with the operand buffers
    if (a.bias && tid < BN / 4)
      reinterpret_cast<float4*>(sbias)[tid] =
          n0 + 4 * tid < a.N ? *reinterpret_cast<const float4*>(a.bias + n0 + 4 * tid) : make_float4(0.f, 0.f, 0.f, 0.f);
    __syncthreads();
    for (int o = 0; o < ((a.aux && !aux_direct) ? 2 : 1); ++o) {
      bf16_t* dst = (o ? a.aux : reinterpret_cast<bf16_t*>(a.C)) + cbase;
      for (int h = 0; h < 2; ++h) {
        if (wr == h) {
#pragma unroll
          for (int i = 0; i < 8; ++i) {
#pragma unroll
            for (int j = 0; j < 2 * JN; ++j) {
              const int nl = wc * (BN / 4) + j * 16 + (lane >> 4) * 4;
              float v[4];
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] = alpha * acc[i][j][r];
              if (a.bias) {
                const float4 b = (a.aux_nt & 8) ? *reinterpret_cast<const float4*>(a.bias + n0 + nl)
                                                : reinterpret_cast<const float4*>(sbias)[nl >> 2];
                v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
              }
              if (aux_direct) {
                const int m = m0 + h * 128 + i * 16 + (lane & 15);
                if (m < a.M && n0 + nl < a.N)
                  *reinterpret_cast<uint2*>(a.aux + cbase + (long)m * a.ldc + n0 + nl) =
                      make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
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
        for (int c = threadIdx.x; c < 128 * (BN / 8); c += NT2) {
          const int row = c / (BN / 8), c8 = c % (BN / 8);
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
            if (o == 0 && a.dact) val = dact8(val, *reinterpret_cast<const uint4*>(a.dact_src + (long)m * a.ldc + n), a.dact);
            if (o != 0 && aux_nt) {  // the pre-activation is read again only by the backward: keep it out of L2
              typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
              __builtin_nontemporal_store(__builtin_bit_cast(u32x4, val),
                                          reinterpret_cast<u32x4*>(dst + (long)m * a.ldc + n));
            } else if (o != 0 || !a.no_c) {
              *reinterpret_cast<uint4*>(dst + (long)m * a.ldc + n) = val;
            }
            if (o == 0 && q8on) {
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
              // the column pass reads the final values from LDS (beta / dact changed them in registers)
              if (q8tp && (a.dact || a.beta != 0.f)) *reinterpret_cast<uint4*>(ct + row * CS + c8 * 8) = val;
            }
          }
        }
        __syncthreads();
        if (o == 0 && q8tp) {
          // column pass: thread -> one column of this 128-row half (16-row groups: 16 LDS reads, one 16-B store of
          // the transposed copy each; the column sum in a fixed row order: deterministic)
          for (int nl = tid; nl < BN; nl += NT2) {
            const int n = n0 + nl;
            float cs = 0.f;
#pragma unroll 2
            for (int rg = 0; rg < 8; ++rg) {
              float f[16];
#pragma unroll
              for (int i = 0; i < 16; ++i) f[i] = __uint_as_float((uint32_t)ct[(rg * 16 + i) * CS + nl] << 16);
#pragma unroll
              for (int i = 0; i < 16; ++i) cs += f[i];
              if (a.q8T) {
                uint4 qv;
                qv.x = q8pack4(a.q8fmt, q8v(f[0]), q8v(f[1]), q8v(f[2]), q8v(f[3]));
                qv.y = q8pack4(a.q8fmt, q8v(f[4]), q8v(f[5]), q8v(f[6]), q8v(f[7]));
                qv.z = q8pack4(a.q8fmt, q8v(f[8]), q8v(f[9]), q8v(f[10]), q8v(f[11]));
                qv.w = q8pack4(a.q8fmt, q8v(f[12]), q8v(f[13]), q8v(f[14]), q8v(f[15]));
                *reinterpret_cast<uint4*>(a.q8T + (long)n * a.M + m0 + h * 128 + rg * 16) = qv;
              }
            }
            if (a.q8col) a.q8col[(long)((m0 + h * 128) >> 7) * a.N + n] = cs;
          }
          __syncthreads();
        }
      }
    }
    if (q8on && a.q8amax) {  // block max |value| -> the amax slot (relaxed check first: most blocks lose)
      float mx = q8max;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
      float* red = reinterpret_cast<float*>(smem);
      if (lane == 0) red[w] = mx;
      __syncthreads();
      if (tid == 0) {
#pragma unroll
        for (int i = 1; i < NT2 / 64; ++i) mx = fmaxf(mx, red[i]);
        unsigned int* am = reinterpret_cast<unsigned int*>(a.q8amax);
        const unsigned int cur = __hip_atomic_load(am, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__float_as_uint(mx) > cur) atomicMax(am, __float_as_uint(mx));
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wr * 128 + i * 16 + (lane & 15);
    if (m >= a.M) continue;
#pragma unroll
    for (int j = 0; j < 2 * JN; ++j) {
      const int n = n0 + wc * (BN / 4) + j * 16 + (lane >> 4) * 4;
      if (n >= a.N) continue;  // N % 4 == 0 (host)
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = alpha * acc[i][j][r];
      const long off = cbase + (long)m * a.ldc + n;
      if (a.beta != 0.f) {
        if (a.out_f32) {
          float4 o = *reinterpret_cast<const float4*>(reinterpret_cast<float*>(a.C) + off);
          v[0] += a.beta * o.x; v[1] += a.beta * o.y; v[2] += a.beta * o.z; v[3] += a.beta * o.w;
        } else {
          uint2 o = *reinterpret_cast<const uint2*>(reinterpret_cast<bf16_t*>(a.C) + off);
          v[0] += a.beta * __uint_as_float(o.x << 16); v[1] += a.beta * __uint_as_float(o.x & 0xffff0000u);
          v[2] += a.beta * __uint_as_float(o.y << 16); v[3] += a.beta * __uint_as_float(o.y & 0xffff0000u);
        }
      }
      if (a.bias) {
        float4 b = *reinterpret_cast<const float4*>(a.bias + n);
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

template <int BN>
void launch256(GemmArgs& a, int amode, int bmode, hipStream_t st, int fp8) {
  dim3 grid(a.tiles_m * a.tiles_n, 1, a.batch * a.splitk);
  const bool auxd = a.aux && (a.aux_nt & 4);
  if (fp8 == 2 && auxd) hipLaunchKernelGGL((gemm256_kernel<OP_KCONTIG, OP_KCONTIG, 2, BN, true>), grid, dim3(NT2), 0, st, a);
  else if (fp8 == 2) hipLaunchKernelGGL((gemm256_kernel<OP_KCONTIG, OP_KCONTIG, 2, BN>), grid, dim3(NT2), 0, st, a);
  else if (fp8 && auxd) hipLaunchKernelGGL((gemm256_kernel<OP_KCONTIG, OP_KCONTIG, 1, BN, true>), grid, dim3(NT2), 0, st, a);
  else if (fp8) hipLaunchKernelGGL((gemm256_kernel<OP_KCONTIG, OP_KCONTIG, 1, BN>), grid, dim3(NT2), 0, st, a);
  else if (amode == OP_KCONTIG && bmode == OP_KCONTIG)
    hipLaunchKernelGGL((gemm256_kernel<OP_KCONTIG, OP_KCONTIG, 0, BN>), grid, dim3(NT2), 0, st, a);
  else if (amode == OP_KCONTIG)
    hipLaunchKernelGGL((gemm256_kernel<OP_KCONTIG, OP_KOUTER, 0, BN>), grid, dim3(NT2), 0, st, a);
  else if (bmode == OP_KCONTIG)
    hipLaunchKernelGGL((gemm256_kernel<OP_KOUTER, OP_KCONTIG, 0, BN>), grid, dim3(NT2), 0, st, a);
  else hipLaunchKernelGGL((gemm256_kernel<OP_KOUTER, OP_KOUTER, 0, BN>), grid, dim3(NT2), 0, st, a);
}

}  // namespace

// Used by dtf_gemm for eligible problems; returns 0 if launched, 1 if not eligible. bn: 256 or 128 (tile width).
int gemm256_try(GemmArgs& a, int amode, int bmode, hipStream_t st, int fp8, int bn) {
  if (a.kchunk % BK || a.kchunk < 2 * BK || (a.lda & 7) || (a.ldb & 7) || a.stats || a.atomic_out || a.crm ||
      a.betamask || a.bsrc)
    return 1;
  if ((a.splitk > 1 && a.K % a.kchunk && (a.K % a.kchunk) % BK) || a.K % BK) return 1;
  if (((uintptr_t)a.A & 15) || ((uintptr_t)a.B & 15)) return 1;
  if ((amode == OP_KOUTER && (a.M & 7)) || (bmode == OP_KOUTER && (a.N & 7))) return 1;
  if ((amode != OP_KCONTIG && amode != OP_KOUTER) || (bmode != OP_KCONTIG && bmode != OP_KOUTER)) return 1;
  if (bn != 256 && bn != 128) return 1;
  if (fp8 && (amode != OP_KCONTIG || bmode != OP_KCONTIG)) return 1;
  a.tiles_m = cdiv(a.M, 256);
  a.tiles_n = cdiv(a.N, bn);
  // pre-activation side output (aux, read again only by the backward), bits: 0 = nontemporal
  // stores (measured +-0); 1 = stored straight from the fragments in the main store pass instead of a second
  // LDS-staged pass (BERT-base +1.5%, GPT-2-medium +1.8%; FFN1 forward 167 -> 141 us / 123 -> 104 us); 2 = also
  // for the fp8 kernels (their own instantiation: 4 VGPR spills; GPT-2-medium fp8 erratic with it, 180-233k vs a
  // steady 231-234k tok/s without: off by default). Default 2 = bit 1
  a.aux_nt = 2;
  count_launch(fp8 ? LC_GEMM256_FP8 : LC_GEMM256);
  if (bn == 256) launch256<256>(a, amode, bmode, st, fp8);
  else launch256<128>(a, amode, bmode, st, fp8);
  return 0;
}

}  // namespace dtf

// Direct entry for benchmarks/tests: C[M][N] = A(m,k) . B(n,k) (A [M][K] or [K][M] when a_kouter; B [N][K] or
// [K][N] when b_kouter), bf16 in, bf16 or f32 out, optional split-K through f32 slabs in ws.
DTF_API int dtf_gemm256(const void* A, const void* B, void* C, int M, int N, int K, long lda, long ldb, long ldc,
                        int a_kouter, int b_kouter, int out_f32, int splitk, float* ws, long ws_elems,
                        void* stream) {
  dtf::GemmArgs a{};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.batch = 1; a.splitk = splitk < 1 ? 1 : splitk; a.alpha = 1.f; a.beta = 0.f; a.out_f32 = out_f32;
  if (N & 3) return -1;
  a.kchunk = (K / a.splitk + dtf::BK - 1) / dtf::BK * dtf::BK;
  hipStream_t st = (hipStream_t)stream;
  if (a.splitk > 1) {
    if (!out_f32 || ldc != N || !ws || ws_elems < (long)a.splitk * M * N) return -3;
    a.C = ws;
    a.slab = (long)M * N;
  }
  if (dtf::gemm256_try(a, a_kouter ? dtf::OP_KOUTER : dtf::OP_KCONTIG, b_kouter ? dtf::OP_KOUTER : dtf::OP_KCONTIG,
                       st, 0, 256))
    return -2;
  if (a.splitk > 1) dtf_sum_rows(ws, (long)M * N, a.splitk, (long)M * N, (float*)C, 0, stream);
  return (int)hipGetLastError();
}

// Direct entry with an explicit tile width (256 or 128) for tests and tile sweeps (no split-K).
DTF_API int dtf_gemm256_bn(const void* A, const void* B, void* C, int M, int N, int K, long lda, long ldb, long ldc,
                           int a_kouter, int b_kouter, int out_f32, int bn, void* stream) {
  dtf::GemmArgs a{};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.batch = 1; a.splitk = 1; a.alpha = 1.f; a.beta = 0.f; a.out_f32 = out_f32;
  if (N & 3) return -1;
  a.kchunk = (K + dtf::BK - 1) / dtf::BK * dtf::BK;
  if (dtf::gemm256_try(a, a_kouter ? dtf::OP_KOUTER : dtf::OP_KCONTIG, b_kouter ? dtf::OP_KOUTER : dtf::OP_KCONTIG,
                       (hipStream_t)stream, 0, bn))
    return -2;
  return (int)hipGetLastError();
}
