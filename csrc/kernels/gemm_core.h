// MFMA GEMM + implicit-GEMM convolution for gfx950 (MI355X / CDNA4).
//
// One kernel template covers every matmul-shaped op of the framework:
//   dense Linear fwd / dgrad / wgrad, batched attention products, and
//   NHWC Conv2D forward (im2col gather), data-gradient (dY gather) and
//   weight-gradient (X gather on a K-outer operand) — the TF MatMul /
//   Conv2D / Conv2DBackpropInput / Conv2DBackpropFilter family that the
//   reference drives through the TF runtime (call sites
//   reference trainer/task.py:69,137 for the ops the linear model issues).
//
// Design (MI355X-first, see /opt/skills/guides/cdna_hip_programming.md §5):
//  * C[m][n] = sum_k A(m,k) * B(n,k). Both operands are staged through LDS as
//    64-deep K tiles, double buffered, register staged (issue the next tile's
//    global loads before the MFMA block, write LDS after it: T14) so any gather
//    (conv padding, stride, dilation) and zero-fill is a per-lane address.
//  * K-contiguous operands live in LDS as [rows][64] with a 16-B chunk XOR
//    swizzle (c ^ ((row>>1)&7)) -> conflict-free ds_read_b128 fragment reads.
//  * K-outer operands (weight-gradient and dgrad-of-Linear cases) live in LDS
//    as [64][cols] with an 8-B granule swizzle and are read with the gfx950
//    transpose read ds_read_b64_tr_b16 (T10) — no transpose pass in HBM.
//  * v_mfma_f32_16x16x32_bf16, 4 waves (256 threads), 64-wide wave tiles.
//    The MFMA is issued with (B,A) swapped so each lane owns 4 consecutive
//    output columns -> 8-byte bf16 / 16-byte f32 stores.
//  * XCD-aware, bijective block remap + grouped tile order for L2 reuse (T1).
//  * Fused epilogue: alpha/beta, bias, ReLU/GELU, pre-activation side output,
//    per-column sum/sum^2 (BatchNorm statistics) and split-K f32 atomics.
#pragma once
#include "common.h"
#include <algorithm>
#include <type_traits>

namespace dtf {

enum OpMode : int {
  OP_KCONTIG = 0,  // X(r,k) = p[r*ld + k]
  OP_KOUTER = 1,   // X(r,k) = p[k*ld + r]
  OP_IM2COL = 2,   // conv fwd A: r = output pixel (n,p,q), k = (kh,kw,ci)
  OP_DGRAD = 3,    // conv dgrad A: r = input pixel (n,h,w), k = (kh,kw,co) gathered from dY
  OP_WGRADX = 4,   // conv wgrad B (k-outer): r = (kh,kw,ci), k = output pixel (n,p,q) gathered from X
  // Tap-uniform forms of IM2COL / DGRAD (C resp. Kout % 64 == 0, R*S <= 32, stride-1 DGRAD): every 64-wide
  // K-tile is ONE filter tap x 64 channels, so the per-K-tile gather is a wave-uniform tap offset added to
  // a per-row base offset, with a per-row bit mask of the taps that fall inside the image; loads go through
  // a buffer descriptor, masked rows get an out-of-range offset and read zeros (no per-row index math, no
  // selects on the 16-B data).
  OP_IM2COL_T = 5,
  OP_DGRAD_T = 6,
  // Row-mapped K-outer forms for the conv weight gradient (operands < 2 GiB): each thread owns ONE k-row
  // (pixel) of the 64-deep tile and R/32 of its 16-B chunks, so the pixel decode / row address is computed
  // once per thread per K-tile (not once per chunk row), loads go through a buffer descriptor with
  // immediate chunk offsets, and out-of-image taps or rows past K read zeros via the range check.
  OP_KOUTER_R = 7,   // A = dY [pixels][Kout]
  OP_WGRADX_R = 8,   // B = X gathered at (pixel, tap)
};

struct ConvGeom {
  int N, H, W, C;   // input NHWC
  int Kout, R, S;   // filter KRSC
  int P, Q;         // output spatial
  int sh, sw, ph, pw, dh, dw;
  FastDiv dPQ, dQ, dHW, dW, dC, dS, dK;
};

struct GemmArgs {
  const bf16_t* A;
  const bf16_t* B;
  void* C;
  bf16_t* aux;          // optional pre-activation output (bf16, ldc)
  const float* bias;    // optional [N]
  const float* scales;  // optional [2] device scales (fp8: dequant factors of A and B; alpha *= s0*s1)
  float* stats;         // optional [2*N]: column sum, sum of squares (f32 atomics)
  long lda, ldb, ldc;
  long sA, sB, sC;      // batch strides (elements)
  int M, N, K;
  int batch, splitk, kchunk;  // kchunk: K range per split (multiple of 64)
  int tiles_m, tiles_n;
  float alpha, beta;
  int act;              // 0 none, 1 relu, 2 gelu(tanh)
  int out_f32;          // C is float
  int atomic_out;       // atomicAdd into float C (split-K / accumulate)
  long slab;            // >0: split-K partials go to slab (blockIdx.z) of this many elements (plain stores)
  ConvGeom g;
  // optional output-row remap (strided dgrad phases): row m = (n, hh, ww) over an rmHs x rmWs grid is stored
  // at pixel (n, rmsh*hh + rmh0, rmsw*ww + rmw0) of an rmH x rmW image
  uint64_t g_rowrep;    // tap-uniform gathers: sum over kh < R of 2^(kh*S)
  // BatchNorm-backward statistics instead of forward ones (stats != nullptr and bnx != nullptr): the output is
  // the gradient dy of a BN(+ReLU) output; partial rows get sum(dz) and sum(dz * (x - mean)) with
  // dz = dy * relu_mask, x = the BN input [pixels][N] saved by the forward (ldc == N), mask 1 bit/element.
  const bf16_t* bnx;
  const uint8_t* bnmask;
  const float* bnmean;
  const uint8_t* betamask;  // optional 1-bit mask on the beta*C term (staged bf16 epilogue only)
  // optional activation backward applied to the (bf16-rounded) product: C = C * act'(dact_src), act 1 relu / 2 gelu
  // (a data-gradient GEMM that produces the gradient of an activation output hands on the pre-activation's)
  const bf16_t* dact_src;
  int dact;
  float* zero_slot;  // optional: block 0 clears this f32 (fp8 delayed scaling: the amax slot the next step fills)
  // optional beta source other than C, on a 2x-subsampled pixel grid (the compact data gradient of a stride-2 1x1
  // projection shortcut): output row m = pixel (n, h, w) of an H x W image adds bsrc[(n, h/2, w/2)] when h and w
  // are even, nothing otherwise (row stride ldc, same channels as C)
  const bf16_t* bsrc;
  FastDiv dBhw, dBw;
  int bH2, bW2;
  int crm;
  FastDiv dRm1, dRm2;
  int rmH, rmW, rmsh, rmsw, rmh0, rmw0;
  // fp8 copies of the (bf16-rounded, post-activation / post-dact) output written by the staged epilogue of
  // gemm256.hip (host-checked; the bf16 C store is skipped when no_c): q8 [M][N] row-major, q8T [N][M] transposed,
  // q8col [M/128][N] per-128-row column sums of the values (a bias gradient's partials). Delayed scaling as
  // gemm_fp8.hip's transposing quantizer: scale = q8amax_prev / fmax when > 0 (else *q8scale), published to
  // q8used / q8used2 by block 0; max |value| accumulated into q8amax. q8fmt 0 = e4m3, 1 = e5m2.
  uint8_t* q8;
  uint8_t* q8T;
  float* q8col;
  const float* q8scale;
  float* q8amax;
  const float* q8amax_prev;
  float* q8used;
  float* q8used2;
  int q8fmt;
  int no_c;
  int aux_nt;  // gemm256.hip staged epilogue: nontemporal stores for the aux (pre-activation) output
  // optional row sums of A over each split's K range (gemm_w4.hip, K-outer A, f32 out): rowsum[split][M] — the bias
  // gradient of a weight-gradient GEMM dW = dY^T X is the row sum of its A operand dY^T (written by the N-tile-0 blocks)
  float* rowsum;
};

// 4 floats -> 4 packed OCP fp8 bytes (fmt 0 e4m3, 1 e5m2), values already scaled and clamped
__device__ __forceinline__ uint32_t q8pack4(int fmt, float a0, float a1, float a2, float a3) {
  int r;
  if (fmt) {
    r = __builtin_amdgcn_cvt_pk_bf8_f32(a0, a1, 0, false);
    r = __builtin_amdgcn_cvt_pk_bf8_f32(a2, a3, r, true);
  } else {
    r = __builtin_amdgcn_cvt_pk_fp8_f32(a0, a1, 0, false);
    r = __builtin_amdgcn_cvt_pk_fp8_f32(a2, a3, r, true);
  }
  return (uint32_t)r;
}

__device__ __forceinline__ long out_row(const GemmArgs& a, int m) {
  if (!a.crm) return m;
  uint32_t n, hw, hh, ww;
  fdivmod((uint32_t)m, a.dRm1, n, hw);
  fdivmod(hw, a.dRm2, hh, ww);
  return ((long)n * a.rmH + (long)(a.rmsh * (int)hh + a.rmh0)) * a.rmW + (a.rmsw * (int)ww + a.rmw0);
}

constexpr int BK = 64;
constexpr int NT = 256;

// Beta operand of output element (row m, column n): C itself, or the stride-2 compact source (nullptr: zero)
__device__ __forceinline__ const bf16_t* beta_src(const GemmArgs& a, long m, int n, const bf16_t* cp) {
  if (!a.bsrc) return cp;
  uint32_t nn, hw, h, w;
  fdivmod((uint32_t)m, a.dBhw, nn, hw);
  fdivmod(hw, a.dBw, h, w);
  if ((h | w) & 1u) return nullptr;
  return a.bsrc + (((long)nn * a.bH2 + (h >> 1)) * a.bW2 + (w >> 1)) * a.ldc + n;
}

// Per-column statistics of 4 stored output values (columns n..n+3 of output pixel row mrow): forward BN
// (sum, sum of squares) or, with a.bnx, backward BN (sum dz, sum dz*(x - mean)).
__device__ __forceinline__ void stat_acc(const GemmArgs& a, long mrow, int n, const float (&v)[4], float (&cs)[4],
                                         float (&cq)[4]) {
  if (a.bnx) {
    const long e = mrow * a.ldc + n;
    const uint2 xr = *reinterpret_cast<const uint2*>(a.bnx + e);
    const float x[4] = {__uint_as_float(xr.x << 16), __uint_as_float(xr.x & 0xffff0000u),
                        __uint_as_float(xr.y << 16), __uint_as_float(xr.y & 0xffff0000u)};
    const uint32_t bits = a.bnmask ? ((uint32_t)a.bnmask[e >> 3] >> (e & 4)) : 0xFu;  // e % 8 is 0 or 4
    const float4 mu = *reinterpret_cast<const float4*>(a.bnmean + n);
    const float m4[4] = {mu.x, mu.y, mu.z, mu.w};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float dz = ((bits >> r) & 1u) ? v[r] : 0.f;
      cs[r] += dz;
      cq[r] = fmaf(dz, x[r] - m4[r], cq[r]);
    }
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) { cs[r] += v[r]; cq[r] = fmaf(v[r], v[r], cq[r]); }
  }
}

// 0.5 x (1 + tanh(u)) == x * sigmoid(2u): one exp and one reciprocal instead of a libm tanhf
__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float u = k0 * (x + k1 * x * x * x);
  return x * __builtin_amdgcn_rcpf(1.f + __expf(-2.f * u));
}

__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  // tanh(u) = 2 s - 1 with s = sigmoid(2u): one exp and one reciprocal instead of a libm tanhf
  const float u = k0 * (x + k1 * x * x * x);
  const float s = __builtin_amdgcn_rcpf(1.f + __expf(-2.f * u));
  return s + 2.f * x * s * (1.f - s) * k0 * (1.f + 3.f * k1 * x * x);
}
// 8 bf16 products (val) times act'(pre) of the 8 matching pre-activations, re-rounded to bf16
__device__ __forceinline__ uint4 dact8(uint4 val, uint4 pre, int act) {
  const uint32_t vw[4] = {val.x, val.y, val.z, val.w}, pw[4] = {pre.x, pre.y, pre.z, pre.w};
  uint32_t o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float f[2], p[2];
    f[0] = __uint_as_float(vw[q] << 16); f[1] = __uint_as_float(vw[q] & 0xffff0000u);
    p[0] = __uint_as_float(pw[q] << 16); p[1] = __uint_as_float(pw[q] & 0xffff0000u);
#pragma unroll
    for (int h = 0; h < 2; ++h) f[h] *= act == 1 ? (p[h] > 0.f ? 1.f : 0.f) : gelu_tanh_grad(p[h]);
    o[q] = pack2bf(f[0], f[1]);
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// Bit mask over the taps (kh * S + kw) of an R x S filter with kh in [h0, h1] and kw in [w0, w1] (empty when
// a range is empty), without a loop over taps: the kw range is one S-bit row pattern, replicated into the
// kept kh rows by a multiply with rowrep = sum_kh 2^(kh*S) (precomputed on the host) masked to [h0, h1].
__device__ __forceinline__ uint32_t tap_mask(int R, int S, int h0, int h1, int w0, int w1, uint64_t rowrep) {
  if (h0 > h1 || w0 > w1) return 0u;
  const uint64_t wm = (1ull << (w1 + 1)) - (1ull << w0);
  const uint64_t rows = ((rowrep >> (h0 * S)) << (h0 * S)) & ((1ull << ((h1 + 1) * S)) - 1);
  return (uint32_t)(wm * rows);
}

// ---- K-contiguous operand: LDS tile [R][64] bf16, 128-B rows ---------------
template <int R, int MODE>
struct KContigLoader {
  static constexpr int L = R / 32;  // 16-B loads per thread per K tile
  const bf16_t* base[L];
  int i0[L], i1[L], i2[L];  // per-row gather state
  bool rv[L];
  int chunk;
  uint4 reg[L];
  // tap-uniform modes: byte offset of the row's tap-(0,0) pixel and its in-image tap mask
  int roff[L];
  uint32_t tmask[L];
  __amdgpu_buffer_rsrc_t rsrc;

  __device__ __forceinline__ void init(const GemmArgs& a, const bf16_t* p, long ld, int r0, int Rtot) {
    const int t = threadIdx.x;
    chunk = t & 7;
    if constexpr (MODE == OP_IM2COL_T || MODE == OP_DGRAD_T) {
      const ConvGeom& g = a.g;
      // the host guarantees the gathered tensor is < 2 GiB, so byte offsets fit 31 bits
      const uint32_t bytes = MODE == OP_IM2COL_T ? (uint32_t)((long)g.N * g.H * g.W * g.C * 2)
                                                 : (uint32_t)((long)g.N * g.P * g.Q * g.Kout * 2);
      rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
#pragma unroll
      for (int i = 0; i < L; ++i) {
        const int r = r0 + (t >> 3) + 32 * i;
        uint32_t m = 0;
        int off = 0;
        if (r < Rtot) {
          uint32_t n, rem, y, x;
          if constexpr (MODE == OP_IM2COL_T) {
            fdivmod((uint32_t)r, g.dPQ, n, rem);
            fdivmod(rem, g.dQ, y, x);
            const int hb = (int)y * g.sh - g.ph, wb = (int)x * g.sw - g.pw;
            off = (((int)n * g.H + hb) * g.W + wb) * g.C * 2;
            if (g.dh == 1 && g.dw == 1) {  // taps in range: kh in [-hb, H-1-hb], kw in [-wb, W-1-wb]
              m = tap_mask(g.R, g.S, max(0, -hb), min(g.R - 1, g.H - 1 - hb), max(0, -wb), min(g.S - 1, g.W - 1 - wb),
                           a.g_rowrep);
            } else {
              for (int kh = 0; kh < g.R; ++kh)
                for (int kw = 0; kw < g.S; ++kw) {
                  const int hi = hb + kh * g.dh, wi = wb + kw * g.dw;
                  if ((unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W) m |= 1u << (kh * g.S + kw);
                }
            }
          } else {  // stride-1 dgrad: dX pixel (n, h, w) gathers dY(n, h + ph - kh*dh, w + pw - kw*dw)
            fdivmod((uint32_t)r, g.dHW, n, rem);
            fdivmod(rem, g.dW, y, x);
            const int hb = (int)y + g.ph, wb = (int)x + g.pw;
            off = (((int)n * g.P + hb) * g.Q + wb) * g.Kout * 2;
            if (g.dh == 1 && g.dw == 1) {  // taps in range: kh in [hb-P+1, hb], kw in [wb-Q+1, wb]
              m = tap_mask(g.R, g.S, max(0, hb - g.P + 1), min(g.R - 1, hb), max(0, wb - g.Q + 1), min(g.S - 1, wb),
                           a.g_rowrep);
            } else {
              for (int kh = 0; kh < g.R; ++kh)
                for (int kw = 0; kw < g.S; ++kw) {
                  const int ho = hb - kh * g.dh, wo = wb - kw * g.dw;
                  if ((unsigned)ho < (unsigned)g.P && (unsigned)wo < (unsigned)g.Q) m |= 1u << (kh * g.S + kw);
                }
            }
          }
        }
        roff[i] = off;
        tmask[i] = m;
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < L; ++i) {
      int row = (t >> 3) + 32 * i;
      int r = r0 + row;
      rv[i] = r < Rtot;
      if (!rv[i]) r = 0;
      if constexpr (MODE == OP_KCONTIG) {
        base[i] = p + (long)r * ld;
      } else if constexpr (MODE == OP_IM2COL) {
        uint32_t n, pq, pp, qq;
        fdivmod((uint32_t)r, a.g.dPQ, n, pq);
        fdivmod(pq, a.g.dQ, pp, qq);
        base[i] = p + (long)n * a.g.H * a.g.W * a.g.C;
        i0[i] = (int)pp * a.g.sh - a.g.ph;
        i1[i] = (int)qq * a.g.sw - a.g.pw;
      } else {  // OP_DGRAD: r indexes dX pixels, gather from dY [N][P][Q][Kout]
        uint32_t n, hw, h, w;
        fdivmod((uint32_t)r, a.g.dHW, n, hw);
        fdivmod(hw, a.g.dW, h, w);
        base[i] = p + (long)n * a.g.P * a.g.Q * a.g.Kout;
        i0[i] = (int)h + a.g.ph;
        i1[i] = (int)w + a.g.pw;
      }
    }
  }

  __device__ __forceinline__ void load(const GemmArgs& a, int k0, int Kend) {
    if constexpr (MODE == OP_IM2COL_T || MODE == OP_DGRAD_T) {
      // k0 is wave-uniform: the tap decomposition runs on the scalar unit
      const ConvGeom& g = a.g;
      uint32_t tap, c0, kh, kw;
      fdivmod((uint32_t)k0, MODE == OP_IM2COL_T ? g.dC : g.dK, tap, c0);
      fdivmod(tap, g.dS, kh, kw);
      const int toff = MODE == OP_IM2COL_T
                           ? (((int)kh * g.dh * g.W + (int)kw * g.dw) * g.C + (int)c0) * 2
                           : ((int)c0 - ((int)kh * g.dh * g.Q + (int)kw * g.dw) * g.Kout) * 2;
      const int lo = toff + chunk * 16;
#pragma unroll
      for (int i = 0; i < L; ++i) {
        const uint32_t off = ((tmask[i] >> tap) & 1u) ? (uint32_t)(roff[i] + lo) : 0x80000000u;
        reg[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0));
      }
      return;
    }
    const int k = k0 + chunk * 8;
    const bool kv = k < Kend;
    if constexpr (MODE == OP_KCONTIG) {
#pragma unroll
      for (int i = 0; i < L; ++i) {
        if (rv[i] && kv) reg[i] = *reinterpret_cast<const uint4*>(base[i] + k);
        else reg[i] = make_uint4(0, 0, 0, 0);
      }
    } else if constexpr (MODE == OP_IM2COL) {
      uint32_t rs, ci, kh, kw;
      fdivmod((uint32_t)k, a.g.dC, rs, ci);
      fdivmod(rs, a.g.dS, kh, kw);
      const int dh = (int)kh * a.g.dh, dw = (int)kw * a.g.dw;
#pragma unroll
      for (int i = 0; i < L; ++i) {
        int hi = i0[i] + dh, wi = i1[i] + dw;
        bool v = rv[i] && kv && (unsigned)hi < (unsigned)a.g.H && (unsigned)wi < (unsigned)a.g.W;
        if (v) reg[i] = *reinterpret_cast<const uint4*>(base[i] + ((long)hi * a.g.W + wi) * a.g.C + ci);
        else reg[i] = make_uint4(0, 0, 0, 0);
      }
    } else {  // OP_DGRAD
      uint32_t rs, co, kh, kw;
      fdivmod((uint32_t)k, a.g.dK, rs, co);
      fdivmod(rs, a.g.dS, kh, kw);
      const int dh = (int)kh * a.g.dh, dw = (int)kw * a.g.dw;
#pragma unroll
      for (int i = 0; i < L; ++i) {
        int th = i0[i] - dh, tw = i1[i] - dw;
        bool v = rv[i] && kv && th >= 0 && tw >= 0;
        int ho = th, wo = tw;
        if (a.g.sh != 1) { v = v && (th % a.g.sh) == 0; ho = th / a.g.sh; }
        if (a.g.sw != 1) { v = v && (tw % a.g.sw) == 0; wo = tw / a.g.sw; }
        v = v && ho < a.g.P && wo < a.g.Q;
        if (v) reg[i] = *reinterpret_cast<const uint4*>(base[i] + ((long)ho * a.g.Q + wo) * a.g.Kout + co);
        else reg[i] = make_uint4(0, 0, 0, 0);
      }
    }
  }

  __device__ __forceinline__ void store(char* lds) {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < L; ++i) {
      int row = (t >> 3) + 32 * i;
      int pc = chunk ^ ((row >> 1) & 7);
      *reinterpret_cast<uint4*>(lds + row * 128 + pc * 16) = reg[i];
    }
  }
};

// fragment read from a [R][64] tile: rows rb..rb+15, k-substep kk
__device__ __forceinline__ v8bf frag_kcontig(const char* lds, int rb, int kk, int lane) {
  int row = rb + (lane & 15);
  int c = (lane >> 4) + 4 * kk;
  int pc = c ^ ((row >> 1) & 7);
  return *reinterpret_cast<const v8bf*>(lds + row * 128 + pc * 16);
}

// ---- K-outer operand: LDS tile [64][R] bf16 -------------------------------
template <int R>
__device__ __forceinline__ int kouter_swz(int k) {
  if constexpr (R >= 128) return (k & 3) | (((k >> 3) & 1) << 2);  // 8 values, granule bits 2..4
  else return ((k >> 1) & 1) | (((k >> 3) & 1) << 1);               // R == 64: 4 values
}

template <int R, int MODE>
struct KOuterLoader {
  static constexpr int CPR = R / 8;       // 16-B chunks per k-row
  static constexpr int RPP = NT / CPR;    // k-rows per pass
  static constexpr int L = BK / RPP;      // loads per thread
  const bf16_t* p;
  long ld;
  int c, col;
  bool cv;
  int khoff, kwoff, ci;  // OP_WGRADX column decomposition
  uint4 reg[L];

  __device__ __forceinline__ void init(const GemmArgs& a, const bf16_t* ptr, long ld_, int r0, int Rtot) {
    const int t = threadIdx.x;
    p = ptr;
    ld = ld_;
    c = t % CPR;
    col = r0 + c * 8;
    cv = col < Rtot;
    if constexpr (MODE == OP_WGRADX) {
      uint32_t rs, cc, kh, kw;
      fdivmod((uint32_t)(cv ? col : 0), a.g.dC, rs, cc);
      fdivmod(rs, a.g.dS, kh, kw);
      ci = (int)cc;
      khoff = (int)kh * a.g.dh - a.g.ph;
      kwoff = (int)kw * a.g.dw - a.g.pw;
    }
  }

  __device__ __forceinline__ void load(const GemmArgs& a, int k0, int Kend) {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < L; ++i) {
      int kr = t / CPR + RPP * i;
      int k = k0 + kr;
      bool v = cv && k < Kend;
      if constexpr (MODE == OP_KOUTER) {
        if (v) reg[i] = *reinterpret_cast<const uint4*>(p + (long)k * ld + col);
        else reg[i] = make_uint4(0, 0, 0, 0);
      } else {  // OP_WGRADX: k is the output pixel
        uint32_t n, pq, pp, qq;
        fdivmod((uint32_t)(v ? k : 0), a.g.dPQ, n, pq);
        fdivmod(pq, a.g.dQ, pp, qq);
        int hi = (int)pp * a.g.sh + khoff, wi = (int)qq * a.g.sw + kwoff;
        v = v && (unsigned)hi < (unsigned)a.g.H && (unsigned)wi < (unsigned)a.g.W;
        if (v) reg[i] = *reinterpret_cast<const uint4*>(p + (((long)n * a.g.H + hi) * a.g.W + wi) * a.g.C + ci);
        else reg[i] = make_uint4(0, 0, 0, 0);
      }
    }
  }

  __device__ __forceinline__ void store(char* lds) {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < L; ++i) {
      int kr = t / CPR + RPP * i;
      int pc = c ^ (kouter_swz<R>(kr) << 1);
      *reinterpret_cast<uint4*>(lds + kr * (R * 2) + pc * 16) = reg[i];
    }
  }
};

template <int R, int MODE>
struct PixelRowLoader {
  static constexpr int CPT = R / 32;  // 16-B chunks per thread (4 threads per 64-deep k-row)
  int kr;
  int coff[CPT];                      // byte offset of the chunk's column within a pixel row (+ tap shift)
  int hoff[CPT], woff[CPT];           // OP_WGRADX_R: tap displacement kh*dh - ph, kw*dw - pw
  bool cv[CPT];
  bool one_tap;                       // every column of the tile belongs to one filter tap
  __amdgpu_buffer_rsrc_t rsrc;
  uint4 reg[CPT];

  __device__ __forceinline__ void init(const GemmArgs& a, const bf16_t* ptr, long ld, int r0, int Rtot) {
    const int t = threadIdx.x;
    const ConvGeom& g = a.g;
    kr = t >> 2;
    const uint32_t bytes = MODE == OP_WGRADX_R ? (uint32_t)((long)g.N * g.H * g.W * g.C * 2)
                                               : (uint32_t)((long)g.N * g.P * g.Q * g.Kout * 2);
    rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)ptr, (short)0, (int)bytes, 0x00020000);
    one_tap = MODE == OP_WGRADX_R && (g.C % R == 0);
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int col = r0 + chunk(t, i) * 8;
      cv[i] = col < Rtot;
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

  __device__ __forceinline__ void load(const GemmArgs& a, int k0, int Kend) {
    const ConvGeom& g = a.g;
    const int k = k0 + kr;
    const bool kv = k < Kend;
    if constexpr (MODE == OP_WGRADX_R) {
      uint32_t n, pq, pp, qq;
      fdivmod((uint32_t)(kv ? k : 0), g.dPQ, n, pq);
      fdivmod(pq, g.dQ, pp, qq);
      const int hb = (int)pp * g.sh, wb = (int)qq * g.sw;
      const int pix = (((int)n * g.H + hb) * g.W + wb) * g.C * 2;
      if (one_tap) {
        const int hi = hb + hoff[0], wi = wb + woff[0];
        const bool v = kv && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
          const uint32_t off = (v && cv[i]) ? (uint32_t)(pix + coff[i]) : 0x80000000u;
          reg[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0));
        }
      } else {
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
          const int hi = hb + hoff[i], wi = wb + woff[i];
          const bool v = kv && cv[i] && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
          const uint32_t off = v ? (uint32_t)(pix + coff[i]) : 0x80000000u;
          reg[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0));
        }
      }
    } else {  // dY rows: k = pixel, row stride ld = Kout
      const int rowb = k * g.Kout * 2;
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
        const uint32_t off = (kv && cv[i]) ? (uint32_t)(rowb + coff[i]) : 0x80000000u;
        reg[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0));
      }
    }
  }

  __device__ __forceinline__ void store(char* lds) {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int pc = chunk(t, i) ^ (kouter_swz<R>(kr) << 1);
      *reinterpret_cast<uint4*>(lds + kr * (R * 2) + pc * 16) = reg[i];
    }
  }

  // Logical 16-B chunk written by thread t in store instruction i. Odd k-rows take their chunks in the
  // other half-order (^4): a ds_write_b128 8-lane group spans two k-rows (4 lanes each), and this puts the
  // two rows' 64-B pieces on different banks (the rows are 256 B apart, i.e. the same bank set).
  __device__ __forceinline__ int chunk(int t, int i) const { return ((t & 3) + 4 * i) ^ ((kr & 1) << 2); }
};

// fragment read from a [64][R] tile via ds_read_b64_tr_b16: cols cb..cb+15, k-substep kk
template <int R>
__device__ __forceinline__ v8bf frag_kouter(const char* lds, int cb, int kk, int lane) {
  const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  v4s r[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    int k = 32 * kk + 8 * G + 4 * h + q;
    int g = (cb >> 2) + p;
    int pg = g ^ (kouter_swz<R>(k) << 2);
    r[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, lds + k * (R * 2) + pg * 8));
  }
  // whole-vector casts: per-element short->__bf16 extraction miscompiles (ROCm 7.2)
  v8s both = __builtin_shufflevector(r[0], r[1], 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(v8bf, both);
}

// K-contiguous operand staged straight into LDS (buffer_load_dwordx4 ... lds): no VGPR round trip, no
// ds_write. A wave instruction fills 1 KiB = 8 rows x 128 B of the [R][64] image lane-linearly, so each lane
// fetches the LOGICAL chunk that belongs at its physical slot (the XOR swizzle is undone on the source side).
// Rows past the operand, k past Kend and (tap-uniform gathers) out-of-image taps get an out-of-range offset
// and the range check writes zeros.
template <int R, int MODE>
struct GldsLoader {
  static_assert(MODE == OP_KCONTIG || MODE == OP_IM2COL_T || MODE == OP_DGRAD_T, "K-contiguous modes only");
  static constexpr int L = R / 32;  // wave instructions per thread per K-tile
  __amdgpu_buffer_rsrc_t rsrc;
  int roff[L];        // byte offset of the row (KCONTIG) / of the row's tap-(0,0) pixel (gathers)
  uint32_t tmask[L];  // KCONTIG: ~0 for valid rows; gathers: in-image tap mask
  int coff[L];        // byte offset of this lane's logical chunk in the 64-wide K-tile (the same for every i:
                      // rows 32 i + (t >> 3) share (row >> 1) & 7)

  __device__ __forceinline__ void init(const GemmArgs& a, const bf16_t* p, long ld, int r0, int Rtot) {
    const int t = threadIdx.x;
    const ConvGeom& g = a.g;
    uint32_t bytes;
    if constexpr (MODE == OP_KCONTIG) bytes = (uint32_t)((long)Rtot * ld * 2);  // host: < 2 GiB
    else if constexpr (MODE == OP_IM2COL_T) bytes = (uint32_t)((long)g.N * g.H * g.W * g.C * 2);
    else bytes = (uint32_t)((long)g.N * g.P * g.Q * g.Kout * 2);
    rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int row = 32 * i + (t >> 3);
      coff[i] = ((t & 7) ^ ((row >> 1) & 7)) * 16;
      const int r = r0 + row;
      uint32_t m = 0;
      int off = 0;
      if (r < Rtot) {
        if constexpr (MODE == OP_KCONTIG) {
          m = ~0u;
          off = (int)((long)r * ld * 2);
        } else {
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
      }
      roff[i] = off;
      tmask[i] = m;
    }
  }

  // instruction i of issue() alone, plain K-contiguous rows only (kernels that interleave the DMA with MFMAs)
  __device__ __forceinline__ void issue1(int k0, int Kend, char* lds, int i) {
    static_assert(MODE == OP_KCONTIG, "issue1: plain rows only");
    const int wave = threadIdx.x >> 6;
    const bool ok = tmask[i] != 0u && k0 + (coff[i] >> 1) < Kend;
    const uint32_t off = ok ? (uint32_t)(roff[i] + k0 * 2 + coff[i]) : 0x80000000u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)(lds + i * 4096 +
                                                                                            wave * 1024),
                                             16, off, 0, 0, 0);
  }

  __device__ __forceinline__ void issue(const GemmArgs& a, int k0, int Kend, char* lds) {
    const int wave = threadIdx.x >> 6;
    int toff;
    uint32_t tap = 0, c0 = (uint32_t)k0;
    if constexpr (MODE == OP_KCONTIG) {
      toff = k0 * 2;
    } else {
      const ConvGeom& g = a.g;
      uint32_t kh, kw;
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
      const uint32_t off = ok ? (uint32_t)(roff[i] + toff + coff[i]) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)(lds + i * 4096 +
                                                                                              wave * 1024),
                                               16, off, 0, 0, 0);
    }
  }
};

// K-outer operand ([64 k][R cols] image, read with ds_read_b64_tr_b16) staged by LDS-DMA: a wave instruction
// fills 1 KiB = 1024/(2R) consecutive k-rows lane-linearly; each lane fetches the logical 16-B column chunk that
// the XOR swizzle puts at its physical slot. OP_KOUTER_R: plain rows (dY of a weight gradient: row stride
// = Kout); OP_WGRADX_R: the row is an output pixel whose input pixel is decoded per K-tile, the column a
// (tap, channel) pair fixed per lane; out-of-image taps / rows past K read zeros via the range check.
template <int R, int MODE>
struct GldsKOuter {
  static_assert(MODE == OP_KOUTER_R || MODE == OP_WGRADX_R || MODE == OP_KOUTER, "K-outer operands only");
  static constexpr int L = R / 32;
  static constexpr int ROWB = R * 2;
  __amdgpu_buffer_rsrc_t rsrc;
  int ldb;          // row stride in bytes (OP_KOUTER: dense operand stored [K][rows])
  int kr[L];        // k-row of the tile this lane fills in instruction i
  int coff[L];      // byte offset of the lane's column chunk (+ tap shift for OP_WGRADX_R)
  int hoff[L], woff[L];
  bool cv[L];

  __device__ __forceinline__ void init(const GemmArgs& a, const bf16_t* ptr, long ld, int r0, int Rtot) {
    const int t = threadIdx.x;
    const ConvGeom& g = a.g;
    const uint32_t bytes = MODE == OP_WGRADX_R ? (uint32_t)((long)g.N * g.H * g.W * g.C * 2)
                           : MODE == OP_KOUTER_R ? (uint32_t)((long)g.N * g.P * g.Q * g.Kout * 2)
                                                 : (uint32_t)((long)a.K * ld * 2);  // host: < 2 GiB
    ldb = MODE == OP_KOUTER_R ? g.Kout * 2 : (int)(ld * 2);
    rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)ptr, (short)0, (int)bytes, 0x00020000);
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int P = i * 4096 + t * 16;
      kr[i] = P / ROWB;
      const int c = ((P % ROWB) >> 4) ^ (kouter_swz<R>(kr[i]) << 1);
      const int col = r0 + c * 8;
      cv[i] = col < Rtot;
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

  // instruction i of issue() alone, plain K-outer rows only (kernels that interleave the DMA with MFMAs)
  __device__ __forceinline__ void issue1(int k0, int Kend, char* lds, int i) {
    static_assert(MODE == OP_KOUTER, "issue1: plain rows only");
    const int wave = threadIdx.x >> 6;
    const int k = k0 + kr[i];
    const bool ok = cv[i] && k < Kend;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rsrc, (__attribute__((address_space(3))) void*)(lds + i * 4096 + wave * 1024), 16,
        ok ? (uint32_t)(k * ldb + coff[i]) : 0x80000000u, 0, 0, 0);
  }

  __device__ __forceinline__ void issue(const GemmArgs& a, int k0, int Kend, char* lds) {
    const ConvGeom& g = a.g;
    const int wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int k = k0 + kr[i];
      bool ok = cv[i] && k < Kend;
      int off;
      if constexpr (MODE == OP_WGRADX_R) {
        if (g.R == 1 && g.S == 1 && g.sh == 1 && g.sw == 1 && g.ph == 0 && g.pw == 0) {
          off = k * g.C * 2 + coff[i];  // pointwise: output pixel == input pixel
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
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsrc, (__attribute__((address_space(3))) void*)(lds + i * 4096 + wave * 1024), 16,
          ok ? (uint32_t)off : 0x80000000u, 0, 0, 0);
    }
  }
};

template <int R, int MODE>
using LoaderFor = typename std::conditional<
    (MODE == OP_KOUTER_R || MODE == OP_WGRADX_R), PixelRowLoader<R, MODE>,
    typename std::conditional<(MODE == OP_KOUTER || MODE == OP_WGRADX), KOuterLoader<R, MODE>,
                              KContigLoader<R, MODE>>::type>::type;

constexpr bool glds_kcontig(int m) { return m == OP_KCONTIG || m == OP_IM2COL_T || m == OP_DGRAD_T; }
constexpr bool glds_kouter(int m) { return m == OP_KOUTER_R || m == OP_WGRADX_R || m == OP_KOUTER; }
constexpr bool glds_mode(int m) { return glds_kcontig(m) || glds_kouter(m); }

template <int R, int MODE>
using GldsFor = typename std::conditional<glds_kouter(MODE), GldsKOuter<R, MODE>, GldsLoader<R, MODE>>::type;

constexpr bool kouter_mode(int m) {
  return m == OP_KOUTER || m == OP_WGRADX || m == OP_KOUTER_R || m == OP_WGRADX_R;
}

template <int R, int MODE>
__device__ __forceinline__ v8bf frag(const char* lds, int rb, int kk, int lane) {
  if constexpr (kouter_mode(MODE)) return frag_kouter<R>(lds, rb, kk, lane);
  else return frag_kcontig(lds, rb, kk, lane);
}

// FP8 (OCP e4m3) 128-deep fragment for the block-scaled v_mfma_scale_f32_16x16x128_f8f6f4: lane (G, i) holds the
// 32 consecutive k bytes 32 G .. 32 G + 31 of row rb + i of a [R][128 fp8] tile (two swizzled 16-B chunks). Any
// assignment of the 128 k values to the 4 lane groups x 32 bytes is a valid MFMA operand as long as A and B use
// the same one (the product sums over k): this one costs two ds_read_b128 per fragment.
__device__ __forceinline__ v8i frag_fp8x128(const char* lds, int rb, int lane) {
  const int row = rb + (lane & 15), G = lane >> 4, sw = (row >> 1) & 7;
  const uint4 lo = *reinterpret_cast<const uint4*>(lds + row * 128 + (((2 * G) ^ sw) << 4));
  const uint4 hi = *reinterpret_cast<const uint4*>(lds + row * 128 + (((2 * G + 1) ^ sw) << 4));
  return v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
}

// 8-bit float operands over 128 k with unit block scales (E8M0 127 = 2^0): twice the FLOP rate of the non-scaled
// fp8 and bf16 16x16 MFMAs (MI355X_MICROARCH.md, Matrix cores). Format codes (cbsz for the first operand, blgp for
// the second): 0 = e4m3 (OCP fp8), 1 = e5m2 (bf8).
template <int FA = 0, int FB = 0>
__device__ __forceinline__ v4f mfma_fp8x128(const v8i& a, const v8i& b, const v4f& c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, FA, FB, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
}
// FP8 template code of the GEMM kernels: 0 = bf16; 1 = A e4m3 x B e4m3; 2 = A e5m2 (gradients) x B e4m3.
// (the kernels issue the MFMA with (B, A) swapped, so B's format goes first)
template <int FP8>
__device__ __forceinline__ v4f mfma_fp8_ab(const v8i& fb, const v8i& fa, const v4f& c) {
  return mfma_fp8x128<0, FP8 == 2 ? 1 : 0>(fb, fa, c);
}

// Shared epilogue of the MFMA GEMM kernels (gemm_kernel here, conv256_kernel in conv256.hip): the block's
// BM x BN accumulator tile is held by WM x WN waves as acc[TM][TN] 16x16 fragments (wave (wm, wn) = (wave / WN,
// wave % WN) owns rows wm*BM/WM.., cols wn*BN/WN..); NTH threads; SMEMB bytes of LDS at smem are free.
// Fused: alpha/beta (+ deferred-ReLU beta mask), bias, activation, pre-activation side output, forward BN
// statistics or backward BN statistics (bnx), split-K slabs, f32 atomics, row remap.
template <int BM, int BN, int WM, int WN, int NTH, int SMEMB>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& a, v4f (&acc)[BM / WM / 16][BN / WN / 16], char* smem,
                                              int m0, int n0, int tile_m, int z, int bz) {
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / WN, wn = wave % WN;
  // ---- epilogue: lane owns row m = ..+(lane&15), cols n = ..+(lane>>4)*4 + r ----
  const long cbase = a.slab > 0 ? (long)z * a.slab : (long)bz * a.sC;
  const float alpha = a.scales ? a.alpha * a.scales[0] * a.scales[1] : a.alpha;
  float csum[TN][4], csq[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) csum[j][r] = csq[j][r] = 0.f;

  // bf16 outputs without beta/atomics: the tile goes through LDS so that the global stores are whole
  // 16-B chunks of contiguous row segments (a lane's MFMA fragment covers 4 columns x 1 row, i.e. 8-B
  // pieces of 16 different rows per store instruction). The main loop ended on a barrier: LDS is free.
  constexpr int CS = BN + 8;  // LDS row stride (elements): 16-B pad keeps the fragment writes conflict-free
  constexpr bool can_stage = BM * CS * 2 <= SMEMB;  // the C tile fits the LDS buffers
  // beta != 0 (accumulate into C) is staged too when there is no bias/activation/aux: the bf16 product goes
  // through LDS and the old C is added in the coalesced store pass (one extra bf16 rounding of the product).
  const bool staged = can_stage && !a.atomic_out && !a.out_f32 && !(a.N & 7) && !(a.ldc & 7) &&
                      !(reinterpret_cast<uintptr_t>(a.C) & 15) &&
                      (a.beta == 0.f || (!a.bias && !a.act && !a.aux && (!a.stats || a.bnx)));
  // BN-backward statistics are taken in the store pass from whole 16-B chunks (coalesced reads of the BN
  // input and one mask byte per 8 channels) instead of per fragment
  const bool bn_bwd = a.stats != nullptr && a.bnx != nullptr;
  if (staged) {
    bf16_t* ct = reinterpret_cast<bf16_t*>(smem);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int ml = wm * WTM + i * 16 + (lane & 15);
      const int m = m0 + ml;
      const bool mv = m < a.M;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int nl = wn * WTN + j * 16 + (lane >> 4) * 4;
        const int n = n0 + nl;
        const bool nv = n < a.N;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = alpha * acc[i][j][r];
        if (a.bias && nv) {
          float4 b = *reinterpret_cast<const float4*>(a.bias + n);
          v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
        }
        if (a.aux && mv && nv) {
          uint2 o;
          o.x = pack2bf(v[0], v[1]);
          o.y = pack2bf(v[2], v[3]);
          *reinterpret_cast<uint2*>(a.aux + cbase + out_row(a, m) * a.ldc + n) = o;
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
        if (a.stats && !bn_bwd && a.beta == 0.f && mv && nv) {  // statistics of the stored (bf16) values
          v[0] = __uint_as_float(o.x << 16); v[1] = __uint_as_float(o.x & 0xffff0000u);
          v[2] = __uint_as_float(o.y << 16); v[3] = __uint_as_float(o.y & 0xffff0000u);
          stat_acc(a, out_row(a, m), n, v, csum[j], csq[j]);
        }
      }
    }
    __syncthreads();
    constexpr int C8 = BN / 8;
    static_assert(NTH % C8 == 0, "a thread's channel chunk must stay fixed across the store pass");
    const int c8t = threadIdx.x % C8;  // this thread's 8-channel chunk (constant over the pass)
    float bs[8], bq[8], bmu[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) bs[r] = bq[r] = bmu[r] = 0.f;
    if (bn_bwd && n0 + c8t * 8 < a.N) {
      const float4 m0v = *reinterpret_cast<const float4*>(a.bnmean + n0 + c8t * 8);
      const float4 m1v = *reinterpret_cast<const float4*>(a.bnmean + n0 + c8t * 8 + 4);
      bmu[0] = m0v.x; bmu[1] = m0v.y; bmu[2] = m0v.z; bmu[3] = m0v.w;
      bmu[4] = m1v.x; bmu[5] = m1v.y; bmu[6] = m1v.z; bmu[7] = m1v.w;
    }
    // full tile, nothing to combine: U LDS reads back to back, then their U stores (the general loop below waits for
    // every read right before its store, behind the beta / dact / BN-backward branches)
    const bool plain = a.beta == 0.f && !a.dact && !bn_bwd && !a.crm && m0 + BM <= a.M && n0 + c8t * 8 < a.N;
    if (plain) {
      constexpr int RPP = NTH / C8, IT = BM / RPP, U = IT < 8 ? IT : 8;
      const int r0 = threadIdx.x / C8;
      bf16_t* cp = reinterpret_cast<bf16_t*>(a.C) + cbase + (long)(m0 + r0) * a.ldc + n0 + c8t * 8;
#pragma unroll
      for (int i0 = 0; i0 < IT; i0 += U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const uint4*>(ct + (r0 + RPP * (i0 + u)) * CS + c8t * 8);
#pragma unroll
        for (int u = 0; u < U; ++u) *reinterpret_cast<uint4*>(cp + (long)RPP * (i0 + u) * a.ldc) = v[u];
        __builtin_amdgcn_sched_group_barrier(0x100, U, 0);
        __builtin_amdgcn_sched_group_barrier(0x040, U, 0);
      }
    }
#pragma unroll 4
    for (int c = plain ? BM * C8 : threadIdx.x; c < BM * C8; c += NTH) {
      const int ml = c / C8;
      const int m = m0 + ml, n = n0 + c8t * 8;
      if (m >= a.M || n >= a.N) continue;
      uint4 val = *reinterpret_cast<const uint4*>(ct + ml * CS + c8t * 8);
      const long e = out_row(a, m) * a.ldc + n;
      bf16_t* cp = reinterpret_cast<bf16_t*>(a.C) + cbase + e;
      const bf16_t* bp = a.beta != 0.f ? beta_src(a, out_row(a, m), n, cp) : nullptr;
      if (bp) {
        const uint4 old = *reinterpret_cast<const uint4*>(bp);
        float f[8], g[8];
        const uint32_t vw[4] = {val.x, val.y, val.z, val.w}, ow[4] = {old.x, old.y, old.z, old.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          f[2 * q] = __uint_as_float(vw[q] << 16); f[2 * q + 1] = __uint_as_float(vw[q] & 0xffff0000u);
          g[2 * q] = __uint_as_float(ow[q] << 16); g[2 * q + 1] = __uint_as_float(ow[q] & 0xffff0000u);
        }
        // betamask: the old C is a BN(+ReLU) output gradient whose ReLU mask was not applied yet (the
        // residual shortcut's gradient, taken lazily instead of materialised by the BN backward)
        const uint32_t bm = a.betamask ? (uint32_t)a.betamask[(e + cbase) >> 3] : 0xFFu;  // e % 8 == 0
#pragma unroll
        for (int r = 0; r < 8; ++r) f[r] = ((bm >> r) & 1u) ? fmaf(a.beta, g[r], f[r]) : f[r];
        val.x = pack2bf(f[0], f[1]); val.y = pack2bf(f[2], f[3]);
        val.z = pack2bf(f[4], f[5]); val.w = pack2bf(f[6], f[7]);
      }
      if (a.dact) val = dact8(val, *reinterpret_cast<const uint4*>(a.dact_src + e), a.dact);
      *reinterpret_cast<uint4*>(cp) = val;
      if (bn_bwd) {
        const uint4 xr = *reinterpret_cast<const uint4*>(a.bnx + e);
        const uint32_t bits = a.bnmask ? (uint32_t)a.bnmask[e >> 3] : 0xFFu;  // e % 8 == 0
        const uint32_t vw[4] = {val.x, val.y, val.z, val.w}, xw[4] = {xr.x, xr.y, xr.z, xr.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int r = 2 * q + h;
            const float dv = __uint_as_float(h ? (vw[q] & 0xffff0000u) : (vw[q] << 16));
            const float xv = __uint_as_float(h ? (xw[q] & 0xffff0000u) : (xw[q] << 16));
            const float dz = ((bits >> r) & 1u) ? dv : 0.f;
            bs[r] += dz;
            bq[r] = fmaf(dz, xv - bmu[r], bq[r]);
          }
        }
      }
    }
    if (bn_bwd) {
      // reduce the NTH/C8 threads that share a channel chunk (fixed order: deterministic), one partial row
      __syncthreads();
      float* red = reinterpret_cast<float*>(smem);
#pragma unroll
      for (int r = 0; r < 8; ++r) { red[threadIdx.x * 16 + r] = bs[r]; red[threadIdx.x * 16 + 8 + r] = bq[r]; }
      __syncthreads();
      float* prow = a.stats + (long)tile_m * 2 * a.N;
      for (int nl = threadIdx.x; nl < BN; nl += NTH) {
        const int n = n0 + nl;
        if (n >= a.N) continue;
        float sv = 0.f, qv = 0.f;
        for (int t = nl >> 3; t < NTH; t += C8) { sv += red[t * 16 + (nl & 7)]; qv += red[t * 16 + 8 + (nl & 7)]; }
        prow[n] = sv;
        prow[a.N + n] = qv;
      }
    } else if (a.stats) {
      __syncthreads();  // the statistics reduction below reuses the LDS
    }
  } else
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * WTM + i * 16 + (lane & 15);
    const bool mv = m < a.M;
    const long mrow = out_row(a, mv ? m : 0);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * WTN + j * 16 + (lane >> 4) * 4;
      if (!mv || n >= a.N) continue;  // N % 4 == 0 is required by the host
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = alpha * acc[i][j][r];
      const long off = cbase + mrow * a.ldc + n;
      if (a.atomic_out) {
        float* Cf = reinterpret_cast<float*>(a.C) + off;
#pragma unroll
        for (int r = 0; r < 4; ++r) atomicAdd(Cf + r, v[r]);
        continue;
      }
      if (a.beta != 0.f) {
        if (a.out_f32) {
          float4 o = *reinterpret_cast<const float4*>(reinterpret_cast<float*>(a.C) + off);
          v[0] += a.beta * o.x; v[1] += a.beta * o.y; v[2] += a.beta * o.z; v[3] += a.beta * o.w;
        } else {
          const bf16_t* bp = beta_src(a, mrow, n, reinterpret_cast<bf16_t*>(a.C) + off);
          uint2 o = bp ? *reinterpret_cast<const uint2*>(bp) : make_uint2(0, 0);
          if (a.betamask) {  // zero the old values whose ReLU bit is clear (see the staged path)
            const uint32_t bm = ((uint32_t)a.betamask[off >> 3] >> (off & 4)) & 0xFu;  // off % 4 == 0
            o.x &= ((bm & 1u) ? 0x0000ffffu : 0u) | ((bm & 2u) ? 0xffff0000u : 0u);
            o.y &= ((bm & 4u) ? 0x0000ffffu : 0u) | ((bm & 8u) ? 0xffff0000u : 0u);
          }
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
          const uint2 pr = *reinterpret_cast<const uint2*>(a.dact_src + mrow * a.ldc + n);
          const uint4 d = dact8(make_uint4(o.x, o.y, 0, 0), make_uint4(pr.x, pr.y, 0, 0), a.dact);
          o.x = d.x; o.y = d.y;
        }
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(a.C) + off) = o;
        if (a.stats) {  // statistics of the stored (bf16-rounded) values
          v[0] = __uint_as_float(o.x << 16); v[1] = __uint_as_float(o.x & 0xffff0000u);
          v[2] = __uint_as_float(o.y << 16); v[3] = __uint_as_float(o.y & 0xffff0000u);
        }
      }
      if (a.stats) stat_acc(a, mrow, n, v, csum[j], csq[j]);
    }
  }
  if (a.stats && !(staged && bn_bwd)) {
    // Deterministic BN statistics: reduce the 16 rows of a lane group by shuffles, the WM wave rows of
    // the tile through LDS, then write ONE partial row per M-tile: stats[tile_m][0,N) = sum,
    // stats[tile_m][N,2N) = sum of squares (bn_finalize sums the tiles_m rows). No atomics.
    float* red = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float s = row16_sum(csum[j][r]), q = row16_sum(csq[j][r]);
        const int nl = wn * WTN + j * 16 + (lane >> 4) * 4 + r;
        if ((lane & 15) == 0) {
          red[wm * BN + nl] = s;
          red[WM * BN + wm * BN + nl] = q;
        }
      }
    }
    __syncthreads();
    float* prow = a.stats + (long)tile_m * 2 * a.N;
    for (int nl = threadIdx.x; nl < BN; nl += NTH) {
      const int n = n0 + nl;
      if (n >= a.N) continue;
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) { s += red[w * BN + nl]; q += red[WM * BN + w * BN + nl]; }
      prow[n] = s;
      prow[a.N + n] = q;
    }
  }
}

// Block -> (tile, z) over a grid of nwg tiles x gridDim.z (split-K slices / batch entries), gridDim.y == 1. The
// hardware deals workgroups to the 8 XCDs round-robin in dispatch order (x fastest, then z): the flat id is
// remapped bijectively so that each XCD gets one contiguous range of (z, tile) pairs — the tiles of one split
// (which read the same operand rows) share an XCD's L2 instead of being spread over all eight.
__device__ __forceinline__ void xcd_block(int nwg, int& bid, int& z) {
  const int total = nwg * (int)gridDim.z;
  int L = (int)blockIdx.z * nwg + (int)blockIdx.x;
  const int xcd = L & 7, qq = total >> 3, rr = total & 7;
  L = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (L >> 3);
  z = L / nwg;
  bid = L - z * nwg;
}

// Staging pipeline (PIPE):
//  1: register-staged, ONE LDS buffer (a second barrier before each restage) — half the LDS per block, so
//     twice the blocks (and bytes in flight) per CU; the default for 128-row tiles.
//  2: register-staged, double-buffered LDS (one barrier per K-tile).
//  3: LDS-DMA (GldsLoader), one buffer, synchronous per K-tile: no staging VGPRs, occupancy hides latency.
//  4: LDS-DMA, double-buffered: the next K-tile's DMA runs under this tile's MFMAs.
template <int BM, int BN, int WM, int WN, int AM, int BMODE, int FP8 = 0, int PIPE = 2>
__global__ void __launch_bounds__(NT, 2) gemm_kernel(GemmArgs a) {
  constexpr int NBUF = (PIPE == 2 || PIPE == 4) ? 2 : 1;
  constexpr bool GLDS = PIPE >= 3;
  constexpr int WTM = BM / WM, WTN = BN / WN;  // wave tile
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  __shared__ __attribute__((aligned(16))) char smem[NBUF * (A_BYTES + B_BYTES)];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / WN, wn = wave % WN;

  // ---- block -> tile (XCD-aware bijective remap, then grouped order) ----
  const int nwg = a.tiles_m * a.tiles_n;
  int bid, z;
  xcd_block(nwg, bid, z);
  constexpr int GROUP = 8;
  const int per_group = GROUP * a.tiles_n;
  const int grp = bid / per_group;
  const int first_m = grp * GROUP;
  const int gsize = min(a.tiles_m - first_m, GROUP);
  const int in_g = bid - grp * per_group;
  const int tile_m = first_m + in_g % gsize;
  const int tile_n = in_g / gsize;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  if (a.zero_slot && blockIdx.x == 0 && blockIdx.z == 0 && threadIdx.x == 0) *a.zero_slot = 0.f;
  const int bz = z / a.splitk, sk = z % a.splitk;
  const int kbeg = sk * a.kchunk;
  const int kend = min(a.K, kbeg + a.kchunk);
  if (kbeg >= kend && a.atomic_out) return;  // (slab mode writes zeros for empty splits)

  const bf16_t* Ap = a.A + (long)bz * a.sA;
  const bf16_t* Bp = a.B + (long)bz * a.sB;

  typename std::conditional<GLDS, GldsFor<BM, AM>, LoaderFor<BM, AM>>::type la;
  typename std::conditional<GLDS, GldsFor<BN, BMODE>, LoaderFor<BN, BMODE>>::type lb;
  la.init(a, Ap, a.lda, m0, a.M);
  lb.init(a, Bp, a.ldb, n0, a.N);

  v4f acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};

  const int nk = (kend - kbeg + BK - 1) / BK;
  char* sA0 = smem;
  char* sB0 = smem + A_BYTES;
  char* sA1 = NBUF == 2 ? smem + A_BYTES + B_BYTES : sA0;
  char* sB1 = NBUF == 2 ? sA1 + A_BYTES : sB0;

  auto compute = [&](const char* cA, const char* cB) {
    if constexpr (FP8) {
      // 128 fp8 of K per tile: ONE block-scaled 16x16x128 MFMA per fragment pair (2x the bf16 FLOP rate)
      v8i fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = frag_fp8x128(cA, wm * WTM + i * 16, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = frag_fp8x128(cB, wn * WTN + j * 16, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma_fp8_ab<FP8>(fb[j], fa[i], acc[i][j]);
    } else
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      v8bf fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = frag<BM, AM>(cA, wm * WTM + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = frag<BN, BMODE>(cB, wn * WTN + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
  };

  if constexpr (GLDS) {
    // (the loaders issue only LDS-DMA loads: no ordinary global load is waited for inside the loop)
    if constexpr (NBUF == 2) {
      if (nk > 0) {
        la.issue(a, kbeg, kend, sA0);
        lb.issue(a, kbeg, kend, sB0);
      }
      for (int kt = 0; kt < nk; ++kt) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // tile kt landed for every wave; every wave is done reading tile kt-1's buffer
        if (kt + 1 < nk) {
          la.issue(a, kbeg + (kt + 1) * BK, kend, (kt & 1) ? sA0 : sA1);
          lb.issue(a, kbeg + (kt + 1) * BK, kend, (kt & 1) ? sB0 : sB1);
        }
        compute((kt & 1) ? sA1 : sA0, (kt & 1) ? sB1 : sB0);
      }
    } else {
      for (int kt = 0; kt < nk; ++kt) {
        if (kt) __syncthreads();  // every wave is done reading the single buffer
        la.issue(a, kbeg + kt * BK, kend, sA0);
        lb.issue(a, kbeg + kt * BK, kend, sB0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        compute(sA0, sB0);
      }
    }
    __syncthreads();  // the epilogue may reuse the LDS
  } else {
    if (nk > 0) {
      la.load(a, kbeg, kend);
      lb.load(a, kbeg, kend);
      la.store(sA0);
      lb.store(sB0);
    }
    __syncthreads();

    for (int kt = 0; kt < nk; ++kt) {
      const bool more = kt + 1 < nk;
      if (more) {
        la.load(a, kbeg + (kt + 1) * BK, kend);
        lb.load(a, kbeg + (kt + 1) * BK, kend);
      }
      compute((kt & 1) ? sA1 : sA0, (kt & 1) ? sB1 : sB0);
      if (more) {
        if constexpr (NBUF == 1) __syncthreads();  // every wave is done reading the single buffer
        la.store((kt & 1) ? sA0 : sA1);
        lb.store((kt & 1) ? sB0 : sB1);
      }
      __syncthreads();
    }
  }

  gemm_epilogue<BM, BN, WM, WN, NT, NBUF * (A_BYTES + B_BYTES)>(a, acc, smem, m0, n0, tile_m, z, bz);
}

}  // namespace dtf
