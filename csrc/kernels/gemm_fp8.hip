// FP8 (OCP e4m3, gfx950 native) GEMM + quantization for the GPT-2-medium fp8 config
// (BASELINE.json: "GPT-2-medium fp8 weights (CDNA4 fp8 MFMA)").
//
//  * dtf_quant_fp8: x (bf16) -> e4m3 with a per-tensor scale; the SAME pass computes amax(|x|) into
//    a device float (atomicMax on the bit pattern; values are non-negative) so the next step can use
//    it ("delayed scaling": no extra reduction pass on the critical path).
//  * dtf_gemm_fp8: C[M][N] = (sa*sb) * A_q[M][K] . B_q[N][K]^T (+bias, act, pre-activation aux), bf16 out,
//    on v_mfma_f32_16x16x32_fp8_fp8 with the same LDS-staged, swizzled pipeline as the bf16 GEMM
//    (gemm_core.h) — half the staged bytes per FLOP.
#include <cstdlib>

#include "gemm_core.h"

namespace {

__device__ __forceinline__ float fp8_max() { return 448.f; }

// 8 bf16 -> 8 e4m3 bytes (x * inv, saturated to +-448)
__device__ __forceinline__ uint2 quant8(const float* f, float inv) {
  uint32_t w[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float a0 = fminf(fmaxf(f[4 * h + 0] * inv, -fp8_max()), fp8_max());
    float a1 = fminf(fmaxf(f[4 * h + 1] * inv, -fp8_max()), fp8_max());
    float a2 = fminf(fmaxf(f[4 * h + 2] * inv, -fp8_max()), fp8_max());
    float a3 = fminf(fmaxf(f[4 * h + 3] * inv, -fp8_max()), fp8_max());
    int r = __builtin_amdgcn_cvt_pk_fp8_f32(a0, a1, 0, false);
    r = __builtin_amdgcn_cvt_pk_fp8_f32(a2, a3, r, true);
    w[h] = (uint32_t)r;
  }
  return make_uint2(w[0], w[1]);
}

// Grid-stride passes over 8-element chunks, QU chunks per thread per trip with every load issued before any use
// (a trip keeps 4 x 16 B per lane in flight: the pass is HBM-latency bound otherwise).
constexpr int QU = 4;

// x (bf16) -> e4m3 with scale; amax(|x|) of the pass is max-ed into *amax (delayed scaling)
__global__ void __launch_bounds__(256) quant_fp8_kernel(const bf16_t* __restrict__ x, uint8_t* __restrict__ q, long n8,
                                                        const float* __restrict__ scale, float* __restrict__ amax) {
  __shared__ float red[16];
  const float inv = 1.f / fmaxf(scale[0], 1e-30f);
  float m = 0.f;
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (QU - 1) * stride < n8; i += QU * stride) {
    float f[QU][8];
#pragma unroll
    for (int u = 0; u < QU; ++u) load8(x + (i + u * stride) * 8, f[u]);
#pragma unroll
    for (int u = 0; u < QU; ++u) {
      *reinterpret_cast<uint2*>(q + (i + u * stride) * 8) = quant8(f[u], inv);
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(f[u][j]));
    }
  }
  for (; i < n8; i += stride) {
    float f[8];
    load8(x + i * 8, f);
    *reinterpret_cast<uint2*>(q + i * 8) = quant8(f, inv);
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(f[j]));
  }
  if (amax) {
    m = block_max(m, red);
    // only blocks that can raise the running maximum issue the atomic: thousands of same-address atomics
    // serialise at the memory side, and most blocks' maxima are below the first few published ones
    if (threadIdx.x == 0) {
      unsigned int* a = reinterpret_cast<unsigned int*>(amax);
      const unsigned int cur = __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__float_as_uint(m) > cur) atomicMax(a, __float_as_uint(m));
    }
  }
}

// new scale from the amax of the previous step: scale = amax / 448 * 2^-margin  (history length 1); the amax
// accumulator is reset here, so the next quantize pass needs no memset
__global__ void fp8_update_scale_kernel(float* amax, float* scale, float margin) {
  float a = amax[0];
  scale[0] = a > 0.f ? a / 448.f * exp2f(margin) : 1.f;
  amax[0] = 0.f;
}

// exact per-tensor scale, pass 1: per-block max |x| partials (no atomics, no zeroing)
__global__ void __launch_bounds__(256) absmax_part_kernel(const bf16_t* __restrict__ x, long n8,
                                                          float* __restrict__ part) {
  __shared__ float red[16];
  float m = 0.f;
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (QU - 1) * stride < n8; i += QU * stride) {
    float f[QU][8];
#pragma unroll
    for (int u = 0; u < QU; ++u) load8(x + (i + u * stride) * 8, f[u]);
#pragma unroll
    for (int u = 0; u < QU; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(f[u][j]));
  }
  for (; i < n8; i += stride) {
    float f[8];
    load8(x + i * 8, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(f[j]));
  }
  m = block_max(m, red);
  if (threadIdx.x == 0) part[blockIdx.x] = m;
}

// pass 2: every block folds the partials into the scale (amax / 448), block 0 publishes it, then quantizes
__global__ void __launch_bounds__(256) quant_fp8_exact_kernel(const bf16_t* __restrict__ x, uint8_t* __restrict__ q,
                                                              long n8, const float* __restrict__ part, int nparts,
                                                              float* __restrict__ scale_out) {
  __shared__ float red[16];
  float m = 0.f;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) m = fmaxf(m, part[i]);
  m = block_max(m, red);
  const float scale = fmaxf(m, 1e-12f) / fp8_max();
  if (blockIdx.x == 0 && threadIdx.x == 0) scale_out[0] = scale;
  const float inv = 1.f / scale;
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (QU - 1) * stride < n8; i += QU * stride) {
    float f[QU][8];
#pragma unroll
    for (int u = 0; u < QU; ++u) load8(x + (i + u * stride) * 8, f[u]);
#pragma unroll
    for (int u = 0; u < QU; ++u) *reinterpret_cast<uint2*>(q + (i + u * stride) * 8) = quant8(f[u], inv);
  }
  for (; i < n8; i += stride) {
    float f[8];
    load8(x + i * 8, f);
    *reinterpret_cast<uint2*>(q + i * 8) = quant8(f, inv);
  }
}

// ---- transposing quantizer (fp8 backward) ----
// One pass over a [M][N] bf16 tensor (M, N multiples of 64) produces any of: the row-major fp8 copy q [M][N], the
// transposed fp8 copy qT [N][M] (the K-contiguous operand of a weight-gradient GEMM over M), per-64-row-tile
// column sums of the f32 values (bias gradient partials) and the running amax (delayed scaling). With `pre` the
// value is dy * act'(pre) (the activation backward folded in: the bf16 gradient is never written).
struct QtArgs {
  const bf16_t* x;
  const bf16_t* pre;
  uint8_t* q;
  uint8_t* qT;
  float* colpart;
  const float* scale;
  float* amax;
  const float* part;  // exact scaling: per-block absmax partials of x (scale = max / fmax, written to scale_out)
  int nparts;
  float* scale_out;
  // delayed scaling without an update launch: scale = amax_prev / fmax when amax_prev > 0 (else *scale); the scale
  // used is published to scale_used / scale_used2 (block (0, 0))
  const float* amax_prev;
  float* scale_used;
  float* scale_used2;
  int M, N, act;
};

__device__ __forceinline__ float gelu_grad_q(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  // tanh(u) = 2 s - 1 with s = sigmoid(2u): one exp and one reciprocal instead of a libm tanhf
  const float u = k0 * (x + k1 * x * x * x);
  const float s = __builtin_amdgcn_rcpf(1.f + __expf(-2.f * u));
  return s + 2.f * x * s * (1.f - s) * k0 * (1.f + 3.f * k1 * x * x);
}

template <int FMT>
__device__ __forceinline__ uint32_t cvt4(float a0, float a1, float a2, float a3) {
  int r;
  if constexpr (FMT == 1) {
    r = __builtin_amdgcn_cvt_pk_bf8_f32(a0, a1, 0, false);
    r = __builtin_amdgcn_cvt_pk_bf8_f32(a2, a3, r, true);
  } else {
    r = __builtin_amdgcn_cvt_pk_fp8_f32(a0, a1, 0, false);
    r = __builtin_amdgcn_cvt_pk_fp8_f32(a2, a3, r, true);
  }
  return (uint32_t)r;
}

// block (x, y) = columns [64x, 64x+64) x rows [QT_ROWS y, QT_ROWS (y+1)), walked as 64-row tiles; thread (wave w,
// lane l): row 16w + (l & 15) of each tile, the 16 columns 16 (l >> 4) .. +15 (the 16 lanes of a DPP row share
// the columns: the column sums, kept in registers over the strip, are row16_sum reductions at the end). All tiles'
// loads are issued before the first quantize / transpose.
constexpr int QT_ROWS = 256;

template <int FMT>
__global__ void __launch_bounds__(256) quant_t_kernel(QtArgs a) {
  constexpr float FMAX = FMT == 1 ? 57344.f : 448.f;
  constexpr int LDT = 80;  // transposed tile row stride (bytes): 16-B aligned rows
  __shared__ __attribute__((aligned(16))) uint8_t sT[2][64 * LDT];
  __shared__ float red[4][64];
  __shared__ float redm[16];
  const int t = threadIdx.x, w = t >> 6, l = t & 63, cc = l >> 4, r = 16 * w + (l & 15);
  const int n0 = blockIdx.x * 64, mb = blockIdx.y * QT_ROWS;
  const int ntile = min(QT_ROWS, a.M - mb) / 64;
  float scale;
  if (a.part) {
    float m = 0.f;
    for (int i = t; i < a.nparts; i += 256) m = fmaxf(m, a.part[i]);
    m = block_max(m, redm);
    scale = fmaxf(m, 1e-12f) / FMAX;
    if (blockIdx.x == 0 && blockIdx.y == 0 && t == 0) a.scale_out[0] = scale;
  } else {
    const float ap = a.amax_prev ? a.amax_prev[0] : 0.f;
    scale = ap > 0.f ? ap / FMAX : fmaxf(a.scale[0], 1e-30f);
    if (a.scale_used && blockIdx.x == 0 && blockIdx.y == 0 && t == 0) {
      a.scale_used[0] = scale;
      if (a.scale_used2) a.scale_used2[0] = scale;
    }
  }
  const float inv = 1.f / scale;
  float cs[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) cs[j] = 0.f;
  float mx = 0.f;
  // every tile's loads are issued before the first use (QT_ROWS / 64 tiles: up to 8 x 16 B per thread in flight;
  // one tile ahead left the pass latency-bound at ~2.5 TB/s on GPT-2-medium's activations)
  constexpr int NTL = QT_ROWS / 64;
  uint4 xa[NTL][2], pa[NTL][2];
#pragma unroll
  for (int tile = 0; tile < NTL; ++tile) {
    if (tile < ntile) {
      const long e = (long)(mb + 64 * tile + r) * a.N + n0 + 16 * cc;
      xa[tile][0] = *reinterpret_cast<const uint4*>(a.x + e);
      xa[tile][1] = *reinterpret_cast<const uint4*>(a.x + e + 8);
      if (a.pre) {
        pa[tile][0] = *reinterpret_cast<const uint4*>(a.pre + e);
        pa[tile][1] = *reinterpret_cast<const uint4*>(a.pre + e + 8);
      }
    }
  }
#pragma unroll
  for (int tile = 0; tile < NTL; ++tile) {
    if (tile >= ntile) break;
    const int m0 = mb + 64 * tile;
    const uint4* xr = xa[tile];
    const uint4* pr = pa[tile];
    float f[16];
    {
      const uint32_t xw[8] = {xr[0].x, xr[0].y, xr[0].z, xr[0].w, xr[1].x, xr[1].y, xr[1].z, xr[1].w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        f[2 * k] = __uint_as_float(xw[k] << 16);
        f[2 * k + 1] = __uint_as_float(xw[k] & 0xffff0000u);
      }
      if (a.pre) {
        const uint32_t pw[8] = {pr[0].x, pr[0].y, pr[0].z, pr[0].w, pr[1].x, pr[1].y, pr[1].z, pr[1].w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float p0 = __uint_as_float(pw[k] << 16), p1 = __uint_as_float(pw[k] & 0xffff0000u);
          f[2 * k] *= a.act == 1 ? (p0 > 0.f ? 1.f : 0.f) : gelu_grad_q(p0);
          f[2 * k + 1] *= a.act == 1 ? (p1 > 0.f ? 1.f : 0.f) : gelu_grad_q(p1);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      mx = fmaxf(mx, fabsf(f[j]));
      cs[j] += f[j];
    }
    uint32_t qw[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = fminf(fmaxf(f[4 * h + j] * inv, -FMAX), FMAX);
      qw[h] = cvt4<FMT>(v[0], v[1], v[2], v[3]);
    }
    const long e = (long)(m0 + r) * a.N + n0 + 16 * cc;
    if (a.q) *reinterpret_cast<uint4*>(a.q + e) = make_uint4(qw[0], qw[1], qw[2], qw[3]);
    if (a.qT) {
      uint8_t* st = sT[tile & 1];
#pragma unroll
      for (int j = 0; j < 16; ++j) st[(16 * cc + j) * LDT + r] = (uint8_t)(qw[j >> 2] >> (8 * (j & 3)));
      __syncthreads();  // (double-buffered: the tile before last is no longer read)
      const int c = t >> 2, rq = (t & 3) * 16;
      *reinterpret_cast<uint4*>(a.qT + (long)(n0 + c) * a.M + m0 + rq) =
          *reinterpret_cast<const uint4*>(st + c * LDT + rq);
    }
  }
  if (a.colpart) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float sj = row16_sum(cs[j]);
      if ((l & 15) == 0) red[w][16 * cc + j] = sj;
    }
    __syncthreads();
    if (t < 64) a.colpart[(long)blockIdx.y * a.N + n0 + t] = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
  }
  if (a.amax) {
    mx = block_max(mx, redm);
    if (t == 0) {
      unsigned int* am = reinterpret_cast<unsigned int*>(a.amax);
      const unsigned int cur = __hip_atomic_load(am, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__float_as_uint(mx) > cur) atomicMax(am, __float_as_uint(mx));
    }
  }
}

// scale <- amax / fmax * 2^margin (unchanged when amax is 0), prev (optional) <- the replaced scale, amax <- 0
__global__ void fp8_update_scale2_kernel(float* amax, float* scale, float* prev, float fmax, float margin) {
  const float am = amax[0], old = scale[0];
  if (prev) prev[0] = old;
  scale[0] = am > 0.f ? am / fmax * exp2f(margin) : old;
  amax[0] = 0.f;
}

}  // namespace

DTF_API void dtf_sum_rows(float* rows, long stride, int nrows, long W, float* out, int accumulate, void* stream);

namespace dtf {
int gemm256_try(GemmArgs& a, int amode, int bmode, hipStream_t st, int fp8, int bn);  // gemm256.hip
}  // namespace dtf

using namespace dtf;

// Tile policy of the fp8 GEMMs: the 256-row pipelined kernel whenever it has >= 128 tiles, 256x128 tiles whenever
// 256x256 would leave CUs idle in its last round and 256x128 fill whole rounds. The scaled fp8 MFMA does twice the
// work per staged byte of bf16, so the 128-row register-staged tiles are relatively more load/latency bound.
// Measured on GPT-2-medium fp8 (interleaved A/B): 35.25 / 35.27 ms/step vs 35.75 / 35.60 with the bf16 rule and
// 35.84 / 35.94 without the 256x128 preference.
namespace dtf {
int gemm_w4_fp8_try(GemmArgs& a, int fp8, hipStream_t st, int bn);  // gemm_w4_fp8.hip
}
// The 4-wave fp8 kernel (gemm_w4_fp8.hip) first: DTF_FP8_W4=0 keeps the 8-wave gemm256 / 128-row kernels (A/B).
// 0 off, 1 every fp8 GEMM, 2 (default) every one except the producer-quantizing (q8) GEMMs: their epilogue (LDS
// transposes for the K-outer copy, column sums, amax) on the 4-wave kernel is faster standalone (FFN1 forward 87 vs
// 106 us, FFN2 data gradient 54 vs 65 us: tools/bench_fp8_gemms.py) but 1.7% slower in the GPT-2-medium fp8 step next
// to the side-stream weight gradients (interleaved, 246.7-247.2k vs 251.0-251.2k tok/s: profiles/r5_fp8_w4.txt)
static int g_fp8_w4 = -1;
static bool fp8_w4_on() {
  if (g_fp8_w4 < 0) {
    const char* e = getenv("DTF_FP8_W4");
    g_fp8_w4 = e ? atoi(e) : 2;
  }
  return g_fp8_w4 != 0;
}
// A/B switch for benchmarks and tests (-1: back to DTF_FP8_W4 / the default)
DTF_API void dtf_fp8_w4_enable(int on) { g_fp8_w4 = on; }
// Its tile width: 256x256 unless 256x128 tiles fill the 256 CUs' rounds clearly better (as pick_w4 in gemm.hip).
static int pick_w4_fp8(long M, long N, long batch_splits) {
  const long t256 = (long)cdiv(M, 256) * cdiv(N, 256) * batch_splits, t2x1 = (long)cdiv(M, 256) * cdiv(N, 128) * batch_splits;
  auto eff = [](long t, long slots) { return (double)t / (double)(((t + slots - 1) / slots) * slots); };
  const double s256 = N > 128 ? eff(t256, 256) : 0.0, s2x1 = 0.8 * eff(t2x1, 256);
  return s256 >= s2x1 ? 256 : 128;
}

static int pick256_fp8(long M, long N, long K) {
  (void)K;
  const long t256 = (long)cdiv(M, 256) * cdiv(N, 256), t2x1 = (long)cdiv(M, 256) * cdiv(N, 128);
  if (t2x1 >= 128 && (t256 % 256) != 0 && t2x1 % 256 == 0) return 128;
  if (t256 >= 128 && t256 % 256 == 0) return 256;
  if (t2x1 >= 128) return 128;
  return 0;
}

DTF_API int dtf_quant_fp8(const void* x, void* q, long n, const float* scale, float* amax, int zero_amax,
                          void* stream) {
  if (n & 7) return -1;
  hipStream_t st = (hipStream_t)stream;
  if (amax && zero_amax) (void)hipMemsetAsync(amax, 0, sizeof(float), st);
  int grid = stream_grid(n / 8 / QU, 256);
  hipLaunchKernelGGL(quant_fp8_kernel, dim3(grid), dim3(256), 0, st, (const bf16_t*)x, (uint8_t*)q, n / 8, scale,
                     amax);
  return (int)hipGetLastError();
}

// Exact per-tensor quantization (weights): scale_out = amax(|x|)/448 computed on the device, two launches,
// ws >= 2048 floats of scratch for the per-block partials.
DTF_API int dtf_quant_fp8_exact(const void* x, void* q, long n, float* scale_out, float* ws, void* stream) {
  if (n & 7) return -1;
  hipStream_t st = (hipStream_t)stream;
  int grid = stream_grid(n / 8 / QU, 256);  // <= 2048 partials
  hipLaunchKernelGGL(absmax_part_kernel, dim3(grid), dim3(256), 0, st, (const bf16_t*)x, n / 8, ws);
  hipLaunchKernelGGL(quant_fp8_exact_kernel, dim3(grid), dim3(256), 0, st, (const bf16_t*)x, (uint8_t*)q, n / 8, ws,
                     grid, scale_out);
  return (int)hipGetLastError();
}

DTF_API int dtf_fp8_update_scale(float* amax, float* scale, float margin, void* stream) {
  hipLaunchKernelGGL(fp8_update_scale_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, amax, scale, margin);
  return (int)hipGetLastError();
}

// Transposing quantizer (see quant_t_kernel; column-sum partials: one row per 256 rows of x). fmt 0 = e4m3, 1 = e5m2. exact: the scale is amax(|x|)/fmax computed
// on the device (two launches; ws >= 2048 floats; written to scale_out), else x is quantized with *scale and
// amax (optional) records max |value|. pre (optional, exact = 0 only): x is dy of act(pre), act 1 relu / 2 gelu.
DTF_API int dtf_quant_fp8_t2(const void* x, const void* pre, int act, void* q, void* qT, float* colpart,
                             const float* scale, float* amax, int M, int N, int fmt, int exact, float* ws,
                             float* scale_out, const float* amax_prev, float* scale_used, float* scale_used2,
                             void* stream);
DTF_API int dtf_quant_fp8_t(const void* x, const void* pre, int act, void* q, void* qT, float* colpart,
                            const float* scale, float* amax, int M, int N, int fmt, int exact, float* ws,
                            float* scale_out, void* stream) {
  return dtf_quant_fp8_t2(x, pre, act, q, qT, colpart, scale, amax, M, N, fmt, exact, ws, scale_out, nullptr, nullptr,
                          nullptr, stream);
}

// dtf_quant_fp8_t with delayed scaling folded in: scale = amax_prev / fmax (when > 0, else *scale), published to
// scale_used (and scale_used2); amax accumulates this pass's max for the next step (the caller's consumer GEMM
// clears amax_prev through GemmArgs::zero_slot so that the slot can accumulate again a step later).
DTF_API int dtf_quant_fp8_t2(const void* x, const void* pre, int act, void* q, void* qT, float* colpart,
                             const float* scale, float* amax, int M, int N, int fmt, int exact, float* ws,
                             float* scale_out, const float* amax_prev, float* scale_used, float* scale_used2,
                             void* stream) {
  if ((M & 63) || (N & 63) || M <= 0 || N <= 0 || (exact && (pre || !ws || !scale_out))) return -1;
  hipStream_t st = (hipStream_t)stream;
  QtArgs a{};
  a.x = (const bf16_t*)x; a.pre = (const bf16_t*)pre; a.act = act;
  a.q = (uint8_t*)q; a.qT = (uint8_t*)qT; a.colpart = colpart;
  a.scale = scale; a.amax = amax; a.M = M; a.N = N;
  a.amax_prev = amax_prev; a.scale_used = scale_used; a.scale_used2 = scale_used2;
  if (exact) {
    const long n8 = (long)M * N / 8;
    const int grid = stream_grid(n8 / QU, 256);
    hipLaunchKernelGGL(absmax_part_kernel, dim3(grid), dim3(256), 0, st, (const bf16_t*)x, n8, ws);
    a.part = ws; a.nparts = grid; a.scale_out = scale_out;
  }
  dim3 g(N / 64, (M + QT_ROWS - 1) / QT_ROWS);
  if (fmt == 1) hipLaunchKernelGGL(quant_t_kernel<1>, g, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(quant_t_kernel<0>, g, dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

// out[W] (+)= sum of nrows rows [nrows][stride] (deterministic; the bias-gradient partials of dtf_quant_fp8_t)
DTF_API int dtf_reduce_rows(float* rows, long stride, int nrows, long W, float* out, int accumulate, void* stream) {
  dtf_sum_rows(rows, stride, nrows, W, out, accumulate, stream);
  return (int)hipGetLastError();
}

DTF_API int dtf_fp8_update_scale2(float* amax, float* scale, float* prev, float fmax, float margin, void* stream) {
  hipLaunchKernelGGL(fp8_update_scale2_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, amax, scale, prev, fmax,
                     margin);
  return (int)hipGetLastError();
}

// General fp8 GEMM: C[M][N] = (s0*s1) * A_q[M][K] . B_q[N][K]^T; A e4m3 (fmt_a 0) or e5m2 (fmt_a 1, gradients), B
// e4m3. bf16 out (+bias, act, aux) or f32 out with beta in {0, 1}; splitk > 1 (f32 out only) goes through f32
// slabs in ws (>= splitk*M*N floats) reduced by dtf_sum_rows (accumulating into C when beta = 1).
DTF_API int dtf_gemm_fp8_ex(const void* A, const void* B, void* C, void* aux, const float* bias, const float* scales,
                            int M, int N, int K, long lda, long ldb, long ldc, int act, int fmt_a, int out_f32,
                            float beta, int splitk, float* ws, long ws_elems, float* zero_slot, void* stream) {
  if ((N & 7) || (K & 127) || (lda & 15) || (ldb & 15) || M <= 0) return -1;
  if (beta != 0.f && beta != 1.f) return -2;
  if (!out_f32 && (beta != 0.f || splitk > 1)) return -3;
  hipStream_t st = (hipStream_t)stream;
  const int fp8 = fmt_a == 1 ? 2 : 1;
  GemmArgs a{};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C; a.aux = (bf16_t*)aux;
  a.bias = bias; a.scales = scales;
  a.M = M; a.N = N; a.K = K / 2;
  a.lda = lda / 2; a.ldb = ldb / 2; a.ldc = ldc;
  a.batch = 1; a.alpha = 1.f; a.beta = beta; a.act = act; a.out_f32 = out_f32;
  a.zero_slot = zero_slot;
  if (splitk < 1) splitk = 1;
  if (splitk > 1) {
    if (!ws || ws_elems < (long)splitk * M * N || ldc != N || bias || act || aux) return -4;
    a.splitk = splitk;
    a.kchunk = ((a.K + splitk - 1) / splitk + BK - 1) / BK * BK;
    a.C = ws;
    a.slab = (long)M * N;
    a.beta = 0.f;
    if (!(fp8_w4_on() && gemm_w4_fp8_try(a, fp8, st, pick_w4_fp8(M, N, splitk)) == 0) &&
        gemm256_try(a, OP_KCONTIG, OP_KCONTIG, st, fp8, 256))
      return -5;
    dtf_sum_rows(ws, (long)M * N, splitk, (long)M * N, (float*)C, beta != 0.f ? 1 : 0, stream);
    return (int)hipGetLastError();
  }
  a.splitk = 1;
  a.kchunk = (a.K + BK - 1) / BK * BK;
  if (fp8_w4_on() && gemm_w4_fp8_try(a, fp8, st, pick_w4_fp8(M, N, 1)) == 0) return (int)hipGetLastError();
  const int bn = pick256_fp8(M, N, K);
  if (bn && gemm256_try(a, OP_KCONTIG, OP_KCONTIG, st, fp8, bn) == 0) return (int)hipGetLastError();
  const long b128 = (long)cdiv(M, 128) * cdiv(N, 128);
  const bool big = b128 >= 256;
  a.tiles_m = cdiv(M, 128);
  a.tiles_n = cdiv(N, big ? 128 : 64);
  dim3 grid(a.tiles_m * a.tiles_n, 1, 1);
  // staging of the 128-row tiles: 2 = register-staged double-buffered LDS, 3 / 4 = LDS-DMA single /
  // double buffered (both operand rows are 16-B aligned: host-checked above). 3 measured fastest standalone on the
  // GPT-2-medium projections (tools/bench_fp8_gemms.py: 0.602 vs 0.631 ms per layer for 2, 0.615 for 4) but slower in
  // the model step (35.89 vs 35.17 ms: the side-stream weight gradients share the CUs), so 2 stays the default
  constexpr int pipe = 2;
#define FP8_LAUNCH(BN_, F_, P_) hipLaunchKernelGGL((gemm_kernel<128, BN_, 2, 2, OP_KCONTIG, OP_KCONTIG, F_, P_>), grid, \
                                                  dim3(NT), 0, st, a)
#define FP8_PIPE_LAUNCH(BN_, F_)                  \
  if (pipe == 4) FP8_LAUNCH(BN_, F_, 4);     \
  else if (pipe == 3) FP8_LAUNCH(BN_, F_, 3); \
  else FP8_LAUNCH(BN_, F_, 2);
  if (big && fp8 == 2) { FP8_PIPE_LAUNCH(128, 2) }
  else if (big) { FP8_PIPE_LAUNCH(128, 1) }
  else if (fp8 == 2) { FP8_PIPE_LAUNCH(64, 2) }
  else { FP8_PIPE_LAUNCH(64, 1) }
#undef FP8_PIPE_LAUNCH
#undef FP8_LAUNCH
  return (int)hipGetLastError();
}

// A: [M][K] e4m3 (lda bytes), B: [N][K] e4m3 (ldb bytes); scales: device [sa, sb]; C bf16 [M][ldc]
DTF_API int dtf_gemm_fp8(const void* A, const void* B, void* C, void* aux, const float* bias, const float* scales,
                         int M, int N, int K, long lda, long ldb, long ldc, int act, int tile, void* stream) {
  if ((N & 3) || (K & 15) || (lda & 1) || (ldb & 1) || M <= 0) return -1;
  GemmArgs a{};
  // the loaders move 16-B chunks: view fp8 rows as bf16_t pairs (K/2, ld/2)
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C; a.aux = (bf16_t*)aux;
  a.bias = bias; a.scales = scales;
  a.M = M; a.N = N; a.K = K / 2;
  a.lda = lda / 2; a.ldb = ldb / 2; a.ldc = ldc;
  a.batch = 1; a.splitk = 1; a.kchunk = (a.K + BK - 1) / BK * BK;
  a.alpha = 1.f; a.beta = 0.f; a.act = act; a.out_f32 = 0;
  if (tile < 0 && fp8_w4_on() && gemm_w4_fp8_try(a, 1, (hipStream_t)stream, pick_w4_fp8(M, N, 1)) == 0)
    return (int)hipGetLastError();
  // the 256x256 glds pipeline when its tiling fills the chip (fp8 halves its staged bytes per FLOP)
  const int bn = tile < 0 ? pick256_fp8(M, N, K) : 0;
  if (bn && gemm256_try(a, OP_KCONTIG, OP_KCONTIG, (hipStream_t)stream, 1, bn) == 0)
    return (int)hipGetLastError();
  if (tile < 0) {
    long b128 = (long)cdiv(M, 128) * cdiv(N, 128);
    tile = b128 >= 256 ? 0 : 2;
  }
  a.tiles_m = cdiv(M, tile == 0 ? 128 : 128);
  a.tiles_n = cdiv(N, tile == 0 ? 128 : 64);
  dim3 grid(a.tiles_m * a.tiles_n, 1, 1);
  if (tile == 0)
    hipLaunchKernelGGL((gemm_kernel<128, 128, 2, 2, OP_KCONTIG, OP_KCONTIG, 1>), grid, dim3(NT), 0,
                       (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL((gemm_kernel<128, 64, 2, 2, OP_KCONTIG, OP_KCONTIG, 1>), grid, dim3(NT), 0,
                       (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

// fp8 GEMM whose epilogue also writes fp8 copies of its (bf16-rounded) output for the next fp8 layer (GemmArgs::q8*):
// C[M][N] = (s0*s1) * A_q . B_q^T (+bias, act with the pre-activation to aux; dact_src/dact: the output is the
// gradient of act(dact_src) — the activation backward applied in the store pass). C may be null (only the fp8
// copies are written). Runs on the 256-row pipelined kernel only: returns -6 (nothing launched) when that kernel
// cannot take the shape, and the caller falls back to the bf16 output + a quantize pass.
DTF_API int dtf_gemm_fp8_q8(const void* A, const void* B, void* C, void* aux, const float* bias, const float* scales,
                            int M, int N, int K, long lda, long ldb, int act, int fmt_a, const void* dact_src,
                            int dact, float* zero_slot, void* q8, void* q8T, float* q8col, int q8fmt,
                            const float* q8scale, float* q8amax, const float* q8amax_prev, float* q8used,
                            float* q8used2, void* stream) {
  if ((N & 7) || (K & 127) || (lda & 15) || (ldb & 15) || M <= 0) return -1;
  if ((M & 255) || !q8scale || (C && ((uintptr_t)C & 15)) || (aux && ((uintptr_t)aux & 15)) ||
      (dact_src && ((uintptr_t)dact_src & 15)) || (q8T && (M & 15)) || (q8 && ((uintptr_t)q8 & 7)) ||
      (q8T && ((uintptr_t)q8T & 15)))
    return -6;
  int bn = pick256_fp8(M, N, K);
  if (!bn) bn = (N % 256 == 0) ? 256 : 128;
  if (N % bn) return -6;
  GemmArgs a{};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C; a.aux = (bf16_t*)aux;
  a.bias = bias; a.scales = scales;
  a.M = M; a.N = N; a.K = K / 2;
  a.lda = lda / 2; a.ldb = ldb / 2; a.ldc = N;
  a.batch = 1; a.splitk = 1; a.kchunk = (a.K + BK - 1) / BK * BK;
  a.alpha = 1.f; a.beta = 0.f; a.act = act; a.out_f32 = 0;
  a.dact_src = (const bf16_t*)dact_src; a.dact = dact_src ? dact : 0;
  a.zero_slot = zero_slot;
  a.q8 = (uint8_t*)q8; a.q8T = (uint8_t*)q8T; a.q8col = q8col; a.q8fmt = q8fmt;
  a.q8scale = q8scale; a.q8amax = q8amax; a.q8amax_prev = q8amax_prev; a.q8used = q8used; a.q8used2 = q8used2;
  a.no_c = C ? 0 : 1;
  if (fp8_w4_on() && g_fp8_w4 != 2 &&
      gemm_w4_fp8_try(a, fmt_a == 1 ? 2 : 1, (hipStream_t)stream, pick_w4_fp8(M, N, 1)) == 0)
    return (int)hipGetLastError();
  if (gemm256_try(a, OP_KCONTIG, OP_KCONTIG, (hipStream_t)stream, fmt_a == 1 ? 2 : 1, bn)) return -6;
  return (int)hipGetLastError();
}
