// FP8 (OCP e4m3, gfx950 native) GEMM + quantization for the GPT-2-medium fp8 config
// (BASELINE.json: "GPT-2-medium fp8 weights (CDNA4 fp8 MFMA)").
//
//  * dtf_quant_fp8: x (bf16) -> e4m3 with a per-tensor scale; the SAME pass computes amax(|x|) into
//    a device float (atomicMax on the bit pattern; values are non-negative) so the next step can use
//    it ("delayed scaling": no extra reduction pass on the critical path).
//  * dtf_gemm_fp8: C[M][N] = (sa*sb) * A_q[M][K] . B_q[N][K]^T (+bias, act, pre-activation aux), bf16 out,
//    on v_mfma_f32_16x16x32_fp8_fp8 with the same LDS-staged, swizzled pipeline as the bf16 GEMM
//    (gemm_core.h) — half the staged bytes per FLOP.
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

}  // namespace

namespace dtf {
int gemm256_try(GemmArgs& a, int amode, int bmode, hipStream_t st, int fp8);  // gemm256.hip
bool prefer256(long M, long N, long K, long batch);                           // gemm.hip
}  // namespace dtf

using namespace dtf;

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
  // the 256x256 glds pipeline when its tiling fills the chip (fp8 halves its staged bytes per FLOP)
  if (tile < 0 && prefer256(M, N, 2L * K, 1) && gemm256_try(a, OP_KCONTIG, OP_KCONTIG, (hipStream_t)stream, 1) == 0)
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
