// Shared device helpers for the gfx950 (CDNA4) kernels of distributed_tensorflow_amd.
//
// Everything here is written for 64-lane wavefronts and the MI355X memory system:
// 16-byte vector accesses, bf16 <-> f32 bit conversions, wave reductions via
// __shfl_xor over 64 lanes, and a magic-number divmod for the implicit-GEMM
// index math (integer division is ~20 VALU ops on CDNA; the magic form is 3).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DTF_API extern "C" __attribute__((visibility("default")))

typedef unsigned short bf16_t;  // raw bf16 bits in memory
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef int v8i __attribute__((ext_vector_type(8)));

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// gfx950 converts f32 -> bf16 in hardware (v_cvt_pk_bf16_f32, round-to-nearest-even, NaN kept quiet):
// one VALU op per pair instead of the 4-5 op software rounding sequence.
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2bf(float a, float b) {
  f32x2_t v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}
__device__ __forceinline__ bf16_t f2bf(float f) {
  return __builtin_bit_cast(bf16_t, (__bf16)f);
}

// Load/store 8 bf16 (16 bytes) <-> 8 floats.
__device__ __forceinline__ void load8(const bf16_t* p, float* f) {
  uint4 v = *reinterpret_cast<const uint4*>(p);
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}
__device__ __forceinline__ void store8(bf16_t* p, const float* f) {
  uint4 v;
  v.x = pack2bf(f[0], f[1]); v.y = pack2bf(f[2], f[3]);
  v.z = pack2bf(f[4], f[5]); v.w = pack2bf(f[6], f[7]);
  *reinterpret_cast<uint4*>(p) = v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Sum over the 16 lanes of each DPP row (lanes 16r..16r+15), result in every lane of the row: four
// VALU adds with DPP operands (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror) instead of
// ds_bpermute shuffles.
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}

// Block-wide sum for blockDim.x multiple of 64 (<= 1024). `red` needs 16 floats.
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int nw = blockDim.x >> 6;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int nw = blockDim.x >> 6;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, red[i]);
  return t;
}

// Unsigned magic-number division for n < 2^31 (Granlund–Montgomery).
struct FastDiv {
  uint32_t d, mul, shr;
};
static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.shr = s;
  f.mul = (uint32_t)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  uint32_t hi = __umulhi(n, f.mul);
  return (hi + n) >> f.shr;
}
__device__ __forceinline__ void fdivmod(uint32_t n, const FastDiv& f, uint32_t& q, uint32_t& r) {
  q = fdiv(n, f);
  r = n - q * f.d;
}

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// Grid size for grid-stride memory-bound kernels: enough blocks to fill 256 CUs.
static inline int stream_grid(long work_items, int block) {
  long g = (work_items + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

// Sum groups of `sg` consecutive rows of a [rows][W] f32 matrix (row stride `stride` elements).
// Group g's sum is written either into its first row (in place, leaders at stride sg*stride) or,
// when `out` is given (single group), into out (+= when accumulate). grid = (ceil(W/256), ngroups).
__global__ void __launch_bounds__(256) dtf_group_rows_kernel(float* __restrict__ rows, long stride, int nrows,
                                                             int sg, long W, float* __restrict__ out,
                                                             int accumulate);

// Deterministic two-level reduction of `nrows` f32 rows (stride `stride`) into out (+= when accumulate);
// the rows are used as scratch. Defined in gemm.hip.
DTF_API void dtf_sum_rows(float* rows, long stride, int nrows, long W, float* out, int accumulate, void* stream);



// Host-side launch counters: which GEMM kernel a call reached (read by the tests through dtf_launch_counts, so a
// test named for a kernel fails when a dispatch change routes its call elsewhere). Incremented at launch sites on
// the host only; no device code touches them.
enum LaunchCounter : int {
  LC_W4_256 = 0,      // gemm_w4.hip, 256x256 tiles
  LC_W4_128 = 1,      // gemm_w4.hip, 256x128 tiles
  LC_GEMM256 = 2,     // gemm256.hip (8-wave)
  LC_GEMM_TILE = 3,   // gemm_core.h gemm_kernel (128/64-row tiles)
  LC_GEMM_DACT = 4,   // dtf_gemm_dact (activation backward in the data-gradient epilogue)
  LC_BETA_BF16 = 5,   // bf16 GEMM accumulating into C (beta != 0)
  LC_SPLITK = 6,      // split-K GEMM (f32 slabs + ordered reduction)
  LC_W4F8_256 = 7,    // gemm_w4_fp8.hip, 256x256 tiles
  LC_W4F8_128 = 8,    // gemm_w4_fp8.hip, 256x128 tiles
  LC_GEMM256_FP8 = 9, // gemm256.hip with fp8 operands
  LC_COUNT = 16
};
DTF_API long* dtf_launch_counters();
inline void count_launch(int c) { dtf_launch_counters()[c]++; }
