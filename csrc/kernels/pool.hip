// NHWC pooling for gfx950: MaxPool (with 1-byte argmax for a deterministic
// gather-form backward) and global average pool.
#include "common.h"

namespace {

// One thread = 8 channels of one output pixel.
// Index decomposition is 32-bit with multiply-shift division (launchers require < 2^31 work items).
struct PoolDivs {
  FastDiv c8, a, b;  // chunks per pixel, then the two spatial extents (Q,P for fwd; W,H for bwd)
};

__global__ void __launch_bounds__(256) maxpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                          uint8_t* __restrict__ arg, int N, int H, int W, int C,
                                                          int P, int Q, int R, int S, int sh, int sw, int ph,
                                                          int pw, PoolDivs dv) {
  const uint32_t total = (uint32_t)N * P * Q * (C / 8);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    uint32_t pix, cc, t, q, n, p;
    fdivmod(i, dv.c8, pix, cc);
    fdivmod(pix, dv.a, t, q);
    fdivmod(t, dv.b, n, p);
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
    for (int r = 0; r < R; ++r) {
      int hi = p * sh - ph + r;
      if ((unsigned)hi >= (unsigned)H) continue;
      for (int s = 0; s < S; ++s) {
        int wi = q * sw - pw + s;
        if ((unsigned)wi >= (unsigned)W) continue;
        float f[8];
        load8(x + ((long)(n * H + hi) * W + wi) * C + cc * 8, f);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (f[j] > best[j]) { best[j] = f[j]; bi[j] = (uint8_t)(r * S + s); }
      }
    }
    store8(y + (long)i * 8, best);
    if (arg) {
      uint2 a;
      a.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
      a.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
      *reinterpret_cast<uint2*>(arg + (long)i * 8) = a;
    }
  }
}

// Gather backward: each input pixel sums dy over the outputs whose argmax is it.
__global__ void __launch_bounds__(256) maxpool_bwd_kernel(const bf16_t* __restrict__ dy,
                                                          const uint8_t* __restrict__ arg, bf16_t* __restrict__ dx,
                                                          int N, int H, int W, int C, int P, int Q, int R, int S,
                                                          int sh, int sw, int ph, int pw, PoolDivs dv) {
  const uint32_t total = (uint32_t)N * H * W * (C / 8);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    uint32_t pix, cc, t, w, n, h;
    fdivmod(i, dv.c8, pix, cc);
    fdivmod(pix, dv.a, t, w);
    fdivmod(t, dv.b, n, h);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int r = 0; r < R; ++r) {
      int th = (int)h + ph - r;
      if (th < 0 || th % sh) continue;
      int p = th / sh;
      if (p >= P) continue;
      for (int s = 0; s < S; ++s) {
        int tw = (int)w + pw - s;
        if (tw < 0 || tw % sw) continue;
        int q = tw / sw;
        if (q >= Q) continue;
        long o = ((long)(n * P + p) * Q + q) * C + cc * 8;
        uint2 a = *reinterpret_cast<const uint2*>(arg + o);
        uint8_t bi[8] = {(uint8_t)a.x, (uint8_t)(a.x >> 8), (uint8_t)(a.x >> 16), (uint8_t)(a.x >> 24),
                         (uint8_t)a.y, (uint8_t)(a.y >> 8), (uint8_t)(a.y >> 16), (uint8_t)(a.y >> 24)};
        float g[8];
        load8(dy + o, g);
        const uint8_t me = (uint8_t)(r * S + s);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (bi[j] == me) acc[j] += g[j];
      }
    }
    store8(dx + (long)i * 8, acc);
  }
}

// Global average pool [N,HW,C] -> [N,C] (f32 or bf16 out): block per (n, 8*256 channel slab)
__global__ void __launch_bounds__(256) gap_fwd_kernel(const bf16_t* __restrict__ x, void* __restrict__ y, int HW,
                                                      int C, int out_f32) {
  const int n = blockIdx.y;
  const int c = (blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (c >= C) return;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const bf16_t* xp = x + (long)n * HW * C + c;
  for (int i = 0; i < HW; ++i) {
    float f[8];
    load8(xp + (long)i * C, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += f[j];
  }
  const float inv = 1.f / HW;
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] *= inv;
  if (out_f32) {
    float* yp = reinterpret_cast<float*>(y) + (long)n * C + c;
    *reinterpret_cast<float4*>(yp) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    *reinterpret_cast<float4*>(yp + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
  } else {
    store8(reinterpret_cast<bf16_t*>(y) + (long)n * C + c, acc);
  }
}

__global__ void __launch_bounds__(256) gap_bwd_kernel(const void* __restrict__ dy, int dy_f32,
                                                      bf16_t* __restrict__ dx, long N, int HW, int C) {
  const int c8 = C / 8;
  const long total = N * HW * c8;
  const float inv = 1.f / HW;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int cc = (int)(i % c8);
    long n = i / c8 / HW;
    float g[8];
    if (dy_f32) {
      const float* p = reinterpret_cast<const float*>(dy) + n * C + cc * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = p[j] * inv;
    } else {
      load8(reinterpret_cast<const bf16_t*>(dy) + n * C + cc * 8, g);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] *= inv;
    }
    store8(dx + i * 8, g);
  }
}

}  // namespace

DTF_API int dtf_maxpool_fwd(const void* x, void* y, void* argmax, int N, int H, int W, int C, int P, int Q, int R,
                            int S, int sh, int sw, int ph, int pw, void* stream) {
  if (C & 7) return -1;
  long total = (long)N * P * Q * (C / 8);
  if (total >= (1L << 31) || R * S > 256) return -1;
  PoolDivs dv{make_fastdiv(C / 8), make_fastdiv(Q), make_fastdiv(P)};
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)x, (bf16_t*)y, (uint8_t*)argmax, N, H, W, C, P, Q, R, S, sh, sw, ph, pw, dv);
  return (int)hipGetLastError();
}

DTF_API int dtf_maxpool_bwd(const void* dy, const void* argmax, void* dx, int N, int H, int W, int C, int P, int Q,
                            int R, int S, int sh, int sw, int ph, int pw, void* stream) {
  if (C & 7) return -1;
  long total = (long)N * H * W * (C / 8);
  if (total >= (1L << 31) || R * S > 256) return -1;
  PoolDivs dv{make_fastdiv(C / 8), make_fastdiv(W), make_fastdiv(H)};
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)dy, (const uint8_t*)argmax, (bf16_t*)dx, N, H, W, C, P, Q, R, S, sh, sw, ph,
                     pw, dv);
  return (int)hipGetLastError();
}

DTF_API int dtf_gap_fwd(const void* x, void* y, int N, int HW, int C, int out_f32, void* stream) {
  if (C & 7) return -1;
  dim3 grid(cdiv(C / 8, 256), N);
  hipLaunchKernelGGL(gap_fwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, y, HW, C, out_f32);
  return (int)hipGetLastError();
}

DTF_API int dtf_gap_bwd(const void* dy, int dy_f32, void* dx, int N, int HW, int C, void* stream) {
  if (C & 7) return -1;
  long total = (long)N * HW * (C / 8);
  hipLaunchKernelGGL(gap_bwd_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, (hipStream_t)stream, dy, dy_f32,
                     (bf16_t*)dx, (long)N, HW, C);
  return (int)hipGetLastError();
}
