// Elementwise / layout / reduction / embedding / loss kernels for gfx950
// (SURVEY §2.4.b K1, K2, K7, K8, K17, K18). Every kernel is 16-B vectorized and
// grid-stride (Guideline 13: scalar bf16 loads cost 2-2.5x on CDNA).
#include "common.h"
#include "dropout_mask.h"

namespace {

__device__ __forceinline__ float gelu_f(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
}
__device__ __forceinline__ float gelu_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  // tanh(u) = 2 s - 1 with s = sigmoid(2u): one exp and one reciprocal instead of a libm tanhf
  const float u = k0 * (x + k1 * x * x * x);
  const float s = __builtin_amdgcn_rcpf(1.f + __expf(-2.f * u));
  return s + 2.f * x * s * (1.f - s) * k0 * (1.f + 3.f * k1 * x * x);
}


__global__ void cast_f32_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, long n) {
  long n8 = n / 8;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float4 a = reinterpret_cast<const float4*>(x)[2 * i], b = reinterpret_cast<const float4*>(x)[2 * i + 1];
    float f[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    store8(y + i * 8, f);
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 7)) y[n8 * 8 + threadIdx.x] = f2bf(x[n8 * 8 + threadIdx.x]);
}

__global__ void cast_bf16_f32_kernel(const bf16_t* __restrict__ x, float* __restrict__ y, long n) {
  long n8 = n / 8;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float f[8];
    load8(x + i * 8, f);
    reinterpret_cast<float4*>(y)[2 * i] = make_float4(f[0], f[1], f[2], f[3]);
    reinterpret_cast<float4*>(y)[2 * i + 1] = make_float4(f[4], f[5], f[6], f[7]);
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 7)) y[n8 * 8 + threadIdx.x] = bf2f(x[n8 * 8 + threadIdx.x]);
}

// NCHW f32 image batch -> NHWC bf16 with channels zero-padded to Cp (input pipeline on device)
__global__ void nchw_to_nhwc_pad_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, int N, int C, int HW,
                                        int Cp) {
  long total = (long)N * HW;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    long n = i / HW, s = i % HW;
    for (int c0 = 0; c0 < Cp; c0 += 8) {
      float f[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        int c = c0 + j;
        f[j] = c < C ? x[(n * C + c) * HW + s] : 0.f;
      }
      store8(y + i * Cp + c0, f);
    }
  }
}

// f32 NCHW images (C <= 4, even H, W) -> bf16 2x2 space-to-depth image [N, H/2+3, W/2+3, 16] with channel index
// (dh*2 + dw)*4 + c and 2 zero rows/cols of padding before, 1 after: the ResNet stem's 7x7/2 pad-3 conv is then a
// 4x4/1 unpadded conv over it (K = 256 instead of 7*7*8 = 392, ops.conv.stem_s2d_filter). One thread = one
// s2d pixel (two 16-B stores).
__global__ void nchw_to_s2d_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, int N, int C, int H, int W) {
  const int Hs = H / 2 + 3, Ws = W / 2 + 3;
  const long total = (long)N * Hs * Ws;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int v = (int)(i % Ws);
    const long t = i / Ws;
    const int u = (int)(t % Hs);
    const long n = t / Hs;
    float f[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int dh = k >> 3, dw = (k >> 2) & 1, c = k & 3;
      const int h = 2 * (u - 2) + dh, w = 2 * (v - 2) + dw;
      f[k] = (c < C && h >= 0 && h < H && w >= 0 && w < W) ? x[((n * C + c) * H + h) * W + w] : 0.f;
    }
    store8(y + i * 16, f);
    store8(y + i * 16 + 8, f + 8);
  }
}

// Filter KRSC (f32 master or bf16) -> bf16 CRSK (the dgrad operand layout).
__global__ void filter_krsc_to_crsk_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ o, int K, int RS,
                                           int C) {
  long total = (long)K * RS * C;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    // i indexes the OUTPUT [c][rs][k] so writes are contiguous
    int k = (int)(i % K);
    long t = i / K;
    int rs = (int)(t % RS);
    int c = (int)(t / RS);
    o[i] = w[((long)k * RS + rs) * C + c];
  }
}

// Batched KRSC -> CRSK for many filters in ONE launch (every conv filter of a model after each optimizer
// step): table[f] = {src, dst, K, RS, C, first_tile}; block = one 64(k) x 64(c) tile of one tap rs, transposed
// through LDS so both the reads (along c) and the writes (along k) are contiguous.
__global__ void __launch_bounds__(256) filters_to_crsk_kernel(const long* __restrict__ table, int nf) {
  __shared__ bf16_t tile[64][66];
  const int b = blockIdx.x;
  int f = 0;
  while (f + 1 < nf && table[(f + 1) * 6 + 5] <= b) ++f;
  const long* d = table + f * 6;
  const bf16_t* __restrict__ w = reinterpret_cast<const bf16_t*>(d[0]);
  bf16_t* __restrict__ o = reinterpret_cast<bf16_t*>(d[1]);
  const int K = (int)d[2], RS = (int)d[3], C = (int)d[4];
  const int kt_n = (K + 63) / 64, ct_n = (C + 63) / 64;
  int t = b - (int)d[5];
  const int ct = t % ct_n; t /= ct_n;
  const int kt = t % kt_n;
  const int rs = t / kt_n;
  const int k0 = kt * 64, c0 = ct * 64;
#pragma unroll 4
  for (int i = 0; i < 16; ++i) {
    const int e = threadIdx.x + 256 * i, kl = e >> 6, cl = e & 63;
    const int k = k0 + kl, c = c0 + cl;
    tile[kl][cl] = (k < K && c < C) ? w[((long)k * RS + rs) * C + c] : (bf16_t)0;
  }
  __syncthreads();
#pragma unroll 4
  for (int i = 0; i < 16; ++i) {
    const int e = threadIdx.x + 256 * i, cl = e >> 6, kl = e & 63;
    const int k = k0 + kl, c = c0 + cl;
    if (k < K && c < C) o[((long)c * RS + rs) * K + k] = tile[kl][cl];
  }
}

__global__ void add_bf16_kernel(const bf16_t* a, const bf16_t* b, bf16_t* y, long n8, float alpha, float beta) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float fa[8], fb[8];
    load8(a + i * 8, fa);
    load8(b + i * 8, fb);
#pragma unroll
    for (int j = 0; j < 8; ++j) fa[j] = alpha * fa[j] + beta * fb[j];
    store8(y + i * 8, fa);
  }
}

// act: 1 relu, 2 gelu. fwd: y = act(x); bwd: dx = dy * act'(x)
__global__ void act_kernel(const bf16_t* x, const bf16_t* dy, bf16_t* y, long n8, int act, int bwd) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float f[8], g[8];
    load8(x + i * 8, f);
    if (bwd) load8(dy + i * 8, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (!bwd) f[j] = act == 1 ? fmaxf(f[j], 0.f) : gelu_f(f[j]);
      else f[j] = g[j] * (act == 1 ? (f[j] > 0.f ? 1.f : 0.f) : gelu_grad(f[j]));
    }
    store8(y + i * 8, f);
  }
}

// Per-step dropout stream: the host seed identifies the call site within a step, the device counter `ctr`
// (advanced once per training step by dtf_rng_advance, inside the captured graph when the step is a hipGraph)
// identifies the step, so a replayed graph draws fresh masks although its kernel arguments are frozen.
__global__ void rng_advance_kernel(uint64_t* ctr) { *ctr += 1; }

// dropout: y = x * mask / keep ; mask regenerated from (seed, chunk index)
__global__ void dropout_kernel(const bf16_t* x, bf16_t* y, long n8, uint32_t thr, uint64_t seed, const uint64_t* ctr) {
  const float inv = 65536.f / (float)thr;
  seed = step_seed(seed, ctr);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float f[8];
    load8(x + i * 8, f);
    const uint32_t kb = keep_bits8(seed, i, thr);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = ((kb >> j) & 1u) ? f[j] * inv : 0.f;
    store8(y + i * 8, f);
  }
}

// Residual add of a dropped-out branch: y = x + dropout(f) in one pass, the same mask as dropout_kernel(f)
// (so the backward of the branch is dropout_kernel(dy) with the same seed) and the same bf16 rounding as the
// two-kernel form (the dropped branch value is rounded before the add).
__global__ void add_dropout_kernel(const bf16_t* x, const bf16_t* f, bf16_t* y, long n8, uint32_t thr, uint64_t seed,
                                   const uint64_t* ctr) {
  const float inv = 65536.f / (float)thr;
  seed = step_seed(seed, ctr);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float a[8], b[8];
    load8(x + i * 8, a);
    load8(f + i * 8, b);
    const uint32_t kb = keep_bits8(seed, i, thr);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += ((kb >> j) & 1u) ? bf2f(f2bf(b[j] * inv)) : 0.f;
    store8(y + i * 8, a);
  }
}

// Column partial sums of a bf16 [M][N] matrix (BiasAddGrad core), N % 8 == 0. Block (bx, by) owns columns
// [256 bx, 256 bx + 256) (32 lanes x 8 columns, 512 contiguous bytes per row) and rows [by rpb, by rpb + rpb)
// (8 row-threads); it writes its partial sums to part[by][N]. No atomics: dtf_sum_rows finishes the reduction
// deterministically.
__global__ void __launch_bounds__(256) colsum_part_kernel(const bf16_t* __restrict__ x, long M, int N, long rpb,
                                                          float* __restrict__ part) {
  __shared__ float red[8][257];
  const int tc = threadIdx.x & 31, tr = threadIdx.x >> 5;
  const long c0 = ((long)blockIdx.x * 32 + tc) * 8;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c0 < N) {
    const long r0 = (long)blockIdx.y * rpb, r1 = min(M, r0 + rpb);
    const bf16_t* p = x + c0;
    long r = r0 + tr;
    for (; r + 8 < r1; r += 16) {  // two independent rows in flight per thread
      float f[8], g[8];
      load8(p + r * N, f);
      load8(p + (r + 8) * N, g);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += f[j] + g[j];
    }
    if (r < r1) {
      float f[8];
      load8(p + r * N, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += f[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[tr][tc * 8 + j] = s[j];
  __syncthreads();
  const long col = (long)blockIdx.x * 256 + threadIdx.x;
  if (col < N) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) t += red[i][threadIdx.x];
    part[(long)blockIdx.y * N + col] = t;
  }
}

// Embedding lookup: out[t] = table[idx[t]] (+ table2[idx2[t]]) (+ table3[idx3[t]]), bf16 rows, D % 8 == 0
__global__ void embed_fwd_kernel(const bf16_t* __restrict__ t1, const long* __restrict__ i1,
                                 const bf16_t* __restrict__ t2, const long* __restrict__ i2,
                                 const bf16_t* __restrict__ t3, const long* __restrict__ i3, bf16_t* __restrict__ out,
                                 long T, int D, int pos_mod) {
  const int d8 = D / 8;
  long total = T * d8;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    long t = i / d8;
    int c = (int)(i % d8) * 8;
    float f[8];
    load8(t1 + i1[t] * D + c, f);
    if (t2) {
      float g[8];
      long r = i2 ? i2[t] : (t % pos_mod);
      load8(t2 + r * D + c, g);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] += g[j];
    }
    if (t3) {
      float g[8];
      long r = i3 ? i3[t] : 0;
      load8(t3 + r * D + c, g);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] += g[j];
    }
    store8(out + t * D + c, f);
  }
}

// Embedding gradient over SORTED token ids (large vocabularies): each wave walks a slice of the sorted
// positions; at every segment start (id differs from its predecessor) it sums the rows of the whole segment
// (perm gives the source token) in registers and writes dtable[id] once. Deterministic, no atomics; rows of
// untouched ids are left as they are (zeroed by the caller).
__global__ void __launch_bounds__(256) embed_bwd_sorted_kernel(const bf16_t* __restrict__ dy,
                                                               const long* __restrict__ sid,
                                                               const long* __restrict__ perm,
                                                               float* __restrict__ dt, long T, int D) {
  const int lane = threadIdx.x & 63;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  const int d8 = D / 8;
  for (long i = wave; i < T; i += nw) {
    const long id = sid[i];
    if (i > 0 && sid[i - 1] == id) continue;
    long e = i + 1;
    while (e < T && sid[e] == id) ++e;
    for (int c = lane; c < d8; c += 64) {
      float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (long k = i; k < e; ++k) {
        float f[8];
        load8(dy + perm[k] * D + c * 8, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += f[j];
      }
      float* o = dt + id * D + c * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] += s[j];
    }
  }
}

// Embedding gradient for small tables (V <= 16 rows, e.g. BERT's token types): one wave per block, each lane's
// columns (NC 8-column chunks) accumulated in registers per table row over the block's tokens in token order, 4
// tokens' loads in flight, then the wave's partial rows to part[block][V][D] — deterministic (no atomics; dtf_sum_rows
// finishes in a fixed order). One launch covers table rows [vbase, vbase + VR); larger tables take ceil(V / 4)
// launches. (Round 4's form accumulated in LDS with float atomics raced by 4 waves on the same rows, 257 us for
// BERT-base b128's 65k tokens: 28 us now.)
template <int VR, int NC>
__global__ void __launch_bounds__(64) embed_bwd_regs_kernel(const bf16_t* __restrict__ dy,
                                                            const long* __restrict__ idx, long T, int D, int V,
                                                            int vbase, long rpb, float* __restrict__ part) {
  const int lane = threadIdx.x;
  const int d8 = D / 8;
  float acc[VR][NC][8];
#pragma unroll
  for (int u = 0; u < VR; ++u)
#pragma unroll
    for (int k = 0; k < NC; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[u][k][j] = 0.f;
  const long r0 = (long)blockIdx.x * rpb, r1 = min(T, r0 + rpb);
  long t = r0;
  for (; t + 4 <= r1; t += 4) {
    int vv[4];
    float f[4][NC][8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      vv[q] = (int)idx[t + q] - vbase;
#pragma unroll
      for (int k = 0; k < NC; ++k) {
        const int c = lane + 64 * k;
        if (c < d8) load8(dy + (t + q) * D + c * 8, f[q][k]);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int u = 0; u < VR; ++u)
        if (vv[q] == u) {
#pragma unroll
          for (int k = 0; k < NC; ++k)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[u][k][j] += f[q][k][j];
        }
  }
  for (; t < r1; ++t) {
    const int v = (int)idx[t] - vbase;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const int c = lane + 64 * k;
      if (c >= d8) continue;
      float f[8];
      load8(dy + t * D + c * 8, f);
#pragma unroll
      for (int u = 0; u < VR; ++u)
        if (v == u) {
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[u][k][j] += f[j];
        }
    }
  }
  float* prow = part + (long)blockIdx.x * V * D + (long)vbase * D;
#pragma unroll
  for (int u = 0; u < VR; ++u) {
    if (vbase + u >= V) break;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const int c = lane + 64 * k;
      if (c >= d8) continue;
      float4* o = reinterpret_cast<float4*>(prow + (long)u * D + c * 8);
      o[0] = make_float4(acc[u][k][0], acc[u][k][1], acc[u][k][2], acc[u][k][3]);
      o[1] = make_float4(acc[u][k][4], acc[u][k][5], acc[u][k][6], acc[u][k][7]);
    }
  }
}

// Fused softmax cross-entropy over rows (logits f32 or bf16), int64 labels.
// loss[r] = logsumexp(x) - x[label]; dlogits = (softmax - onehot) * gscale (written in the fwd pass).
// label < 0 => ignored row (loss 0, grad 0). label_smoothing eps spreads eps/V over all classes.
__global__ void __launch_bounds__(256) softmax_ce_kernel(const void* __restrict__ logits, int in_f32,
                                                         const long* __restrict__ labels, float* __restrict__ loss,
                                                         void* __restrict__ dlogits, int grad_f32, int V,
                                                         float gscale, float smooth) {
  __shared__ float red[16];
  const long r = blockIdx.x;
  const float* xf = in_f32 ? reinterpret_cast<const float*>(logits) + r * V : nullptr;
  const bf16_t* xb = in_f32 ? nullptr : reinterpret_cast<const bf16_t*>(logits) + r * V;
  auto ld = [&](int i) { return xf ? xf[i] : bf2f(xb[i]); };
  float m = -INFINITY;
  for (int i = threadIdx.x; i < V; i += blockDim.x) m = fmaxf(m, ld(i));
  m = block_max(m, red);
  float s = 0.f, sx = 0.f;
  for (int i = threadIdx.x; i < V; i += blockDim.x) {
    float v = ld(i);
    s += __expf(v - m);
    sx += v;
  }
  s = block_sum(s, red);
  sx = block_sum(sx, red);
  const long lab = labels[r];
  const float lse = m + __logf(s);
  if (threadIdx.x == 0) {
    float l = 0.f;
    if (lab >= 0) {
      float xl = ld((int)lab);
      l = (1.f - smooth) * (lse - xl) + smooth * (lse - sx / V);
    }
    loss[r] = l;
  }
  if (!dlogits) return;
  const float inv = 1.f / s;
  for (int i = threadIdx.x; i < V; i += blockDim.x) {
    float p = __expf(ld(i) - m) * inv;
    float tgt = (i == lab ? 1.f - smooth : 0.f) + smooth / V;
    float gval = lab >= 0 ? (p - tgt) * gscale : 0.f;
    if (grad_f32) reinterpret_cast<float*>(dlogits)[r * V + i] = gval;
    else reinterpret_cast<bf16_t*>(dlogits)[r * V + i] = f2bf(gval);
  }
}

// Two-pass softmax cross-entropy (the gradient is produced in the backward, where dloss is known):
//   fwd: one online pass per row -> loss[r], lse[r];  bwd: dlogits = (exp(x - lse) - target) * dloss[r].
// bf16 rows are read with 16-B vector loads between a scalar head (rows of odd length V start at any element
// offset) and a scalar tail; one 256-thread block per row.
__device__ __forceinline__ void ce_online(float v, float& m, float& s) {
  if (v > m) {
    s = s * __expf(m - v) + 1.f;
    m = v;
  } else {
    s += __expf(v - m);
  }
}

__global__ void __launch_bounds__(256) softmax_ce_fwd_kernel(const void* __restrict__ logits, int in_f32,
                                                             const long* __restrict__ labels, float* __restrict__ loss,
                                                             float* __restrict__ lse_out, int V, float smooth) {
  __shared__ float red[16];
  const long r = blockIdx.x;
  const int t = threadIdx.x;
  float m = -INFINITY, s = 0.f, sx = 0.f;
  if (in_f32) {
    const float* xf = reinterpret_cast<const float*>(logits) + r * V;
    for (int i = t; i < V; i += blockDim.x) { const float v = xf[i]; ce_online(v, m, s); sx += v; }
  } else {
    const bf16_t* xb = reinterpret_cast<const bf16_t*>(logits) + r * V;
    const int head = min(V, (int)((8 - ((reinterpret_cast<uintptr_t>(xb) >> 1) & 7)) & 7));
    const int nvec = (V - head) >> 3;
    if (t < head) { const float v = bf2f(xb[t]); ce_online(v, m, s); sx += v; }
    const bf16_t* xv = xb + head;
    for (int c = t; c < nvec; c += blockDim.x) {
      float f[8];
      load8(xv + c * 8, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) { ce_online(f[j], m, s); sx += f[j]; }
    }
    for (int i = head + nvec * 8 + t; i < V; i += blockDim.x) { const float v = bf2f(xb[i]); ce_online(v, m, s); sx += v; }
  }
  const float M = block_max(m, red);
  const float S = block_sum(m == -INFINITY ? 0.f : s * __expf(m - M), red);
  const float SX = block_sum(sx, red);
  if (t == 0) {
    const float lse = M + __logf(S);
    const long lab = labels[r];
    float l = 0.f;
    if (lab >= 0) {
      const float xl = in_f32 ? reinterpret_cast<const float*>(logits)[r * V + lab]
                              : bf2f(reinterpret_cast<const bf16_t*>(logits)[r * V + lab]);
      l = (1.f - smooth) * (lse - xl) + smooth * (lse - SX / V);
    }
    loss[r] = l;
    lse_out[r] = lse;
  }
}

__global__ void __launch_bounds__(256) softmax_ce_bwd_kernel(const void* __restrict__ logits, int in_f32,
                                                             const long* __restrict__ labels,
                                                             const float* __restrict__ lse_in,
                                                             const float* __restrict__ dloss, void* __restrict__ dl,
                                                             int V, float smooth) {
  const long r = blockIdx.x;
  const int t = threadIdx.x;
  const long lab = labels[r];
  const float g = lab >= 0 ? dloss[r] : 0.f, lse = lse_in[r];
  const float off = smooth / V, hit = 1.f - smooth;
  auto grad = [&](float v, int i) { return (__expf(v - lse) - ((i == lab ? hit : 0.f) + off)) * g; };
  if (in_f32) {
    const float* xf = reinterpret_cast<const float*>(logits) + r * V;
    float* o = reinterpret_cast<float*>(dl) + r * V;
    for (int i = t; i < V; i += blockDim.x) o[i] = grad(xf[i], i);
    return;
  }
  const bf16_t* xb = reinterpret_cast<const bf16_t*>(logits) + r * V;
  bf16_t* ob = reinterpret_cast<bf16_t*>(dl) + r * V;
  const int head = min(V, (int)((8 - ((reinterpret_cast<uintptr_t>(xb) >> 1) & 7)) & 7));
  const bool vec = ((reinterpret_cast<uintptr_t>(ob) ^ reinterpret_cast<uintptr_t>(xb)) & 15) == 0;
  const int nvec = vec ? (V - head) >> 3 : 0;
  if (vec && t < head) ob[t] = f2bf(grad(bf2f(xb[t]), t));
  for (int c = t; c < nvec; c += blockDim.x) {
    float f[8];
    const int i0 = head + c * 8;
    load8(xb + i0, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = grad(f[j], i0 + j);
    store8(ob + i0, f);
  }
  for (int i = (vec ? head + nvec * 8 : 0) + t; i < V; i += blockDim.x) ob[i] = f2bf(grad(bf2f(xb[i]), i));
}

// Row softmax over bf16 scores with scale and optional causal mask (attention probabilities).
// rows are [batch][Sq] with row length Sk; causal: col > (row % Sq) + (Sk - Sq) masked.
__global__ void __launch_bounds__(256) softmax_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                          int Sq, int Sk, float scale, int causal,
                                                          const float* __restrict__ add_mask) {
  __shared__ float red[16];
  const long r = blockIdx.x;
  const int qi = (int)(r % Sq);
  const long bidx = r / Sq;
  const bf16_t* xr = x + r * Sk;
  const int lim = causal ? qi + (Sk - Sq) : Sk - 1;
  const float* am = add_mask ? add_mask + bidx * Sk : nullptr;  // [batch][Sk] additive mask
  float m = -INFINITY;
  for (int i = threadIdx.x; i < Sk; i += blockDim.x) {
    float v = i <= lim ? bf2f(xr[i]) * scale + (am ? am[i] : 0.f) : -INFINITY;
    m = fmaxf(m, v);
  }
  m = block_max(m, red);
  float s = 0.f;
  for (int i = threadIdx.x; i < Sk; i += blockDim.x) {
    float v = i <= lim ? bf2f(xr[i]) * scale + (am ? am[i] : 0.f) : -INFINITY;
    s += v == -INFINITY ? 0.f : __expf(v - m);
  }
  s = block_sum(s, red);
  const float inv = s > 0.f ? 1.f / s : 0.f;
  for (int i = threadIdx.x; i < Sk; i += blockDim.x) {
    float v = i <= lim ? bf2f(xr[i]) * scale + (am ? am[i] : 0.f) : -INFINITY;
    y[r * Sk + i] = f2bf(v == -INFINITY ? 0.f : __expf(v - m) * inv);
  }
}

// dx = scale * y * (dy - sum(dy*y))
__global__ void __launch_bounds__(256) softmax_bwd_kernel(const bf16_t* __restrict__ y, const bf16_t* __restrict__ dy,
                                                          bf16_t* __restrict__ dx, int Sk, float scale) {
  __shared__ float red[16];
  const long r = blockIdx.x;
  float s = 0.f;
  for (int i = threadIdx.x; i < Sk; i += blockDim.x) s += bf2f(y[r * Sk + i]) * bf2f(dy[r * Sk + i]);
  s = block_sum(s, red);
  for (int i = threadIdx.x; i < Sk; i += blockDim.x) {
    float yv = bf2f(y[r * Sk + i]);
    dx[r * Sk + i] = f2bf(scale * yv * (bf2f(dy[r * Sk + i]) - s));
  }
}

}  // namespace

#define GRID(n) dim3(stream_grid((n), 256)), dim3(256), 0, (hipStream_t)stream


DTF_API int dtf_cast_f32_bf16(const float* x, void* y, long n, void* stream) {
  hipLaunchKernelGGL(cast_f32_bf16_kernel, GRID(n / 8 + 1), x, (bf16_t*)y, n);
  return (int)hipGetLastError();
}
DTF_API int dtf_cast_bf16_f32(const void* x, float* y, long n, void* stream) {
  hipLaunchKernelGGL(cast_bf16_f32_kernel, GRID(n / 8 + 1), (const bf16_t*)x, y, n);
  return (int)hipGetLastError();
}
DTF_API int dtf_nchw_to_nhwc_pad(const float* x, void* y, int N, int C, int HW, int Cp, void* stream) {
  if (Cp & 7) return -1;
  hipLaunchKernelGGL(nchw_to_nhwc_pad_kernel, GRID((long)N * HW), x, (bf16_t*)y, N, C, HW, Cp);
  return (int)hipGetLastError();
}
DTF_API int dtf_nchw_to_s2d(const float* x, void* y, int N, int C, int H, int W, void* stream) {
  if (C > 4 || (H & 1) || (W & 1)) return -1;
  hipLaunchKernelGGL(nchw_to_s2d_kernel, GRID((long)N * (H / 2 + 3) * (W / 2 + 3)), x, (bf16_t*)y, N, C, H, W);
  return (int)hipGetLastError();
}
DTF_API int dtf_filter_to_crsk(const void* w, void* o, int K, int RS, int C, void* stream) {
  hipLaunchKernelGGL(filter_krsc_to_crsk_kernel, GRID((long)K * RS * C), (const bf16_t*)w, (bf16_t*)o, K, RS, C);
  return (int)hipGetLastError();
}
DTF_API int dtf_filters_to_crsk(const long* table, int nfilters, int total_tiles, void* stream) {
  if (nfilters <= 0 || total_tiles <= 0) return 0;
  hipLaunchKernelGGL(filters_to_crsk_kernel, dim3(total_tiles), dim3(256), 0, (hipStream_t)stream, table, nfilters);
  return (int)hipGetLastError();
}
DTF_API int dtf_add_bf16(const void* a, const void* b, void* y, long n, float alpha, float beta, void* stream) {
  if (n & 7) return -1;
  hipLaunchKernelGGL(add_bf16_kernel, GRID(n / 8), (const bf16_t*)a, (const bf16_t*)b, (bf16_t*)y, n / 8, alpha,
                     beta);
  return (int)hipGetLastError();
}
DTF_API int dtf_act(const void* x, const void* dy, void* y, long n, int act, int bwd, void* stream) {
  if (n & 7) return -1;
  hipLaunchKernelGGL(act_kernel, GRID(n / 8), (const bf16_t*)x, (const bf16_t*)dy, (bf16_t*)y, n / 8, act, bwd);
  return (int)hipGetLastError();
}
// ctr: optional device step counter (see step_seed); nullptr = the host seed alone
DTF_API int dtf_add_dropout(const void* x, const void* f, void* y, long n, float keep, unsigned long long seed,
                            const void* ctr, void* stream) {
  if (n & 7) return -1;
  hipLaunchKernelGGL(add_dropout_kernel, GRID(n / 8), (const bf16_t*)x, (const bf16_t*)f, (bf16_t*)y, n / 8,
                     keep_threshold(keep), (uint64_t)seed, (const uint64_t*)ctr);
  return (int)hipGetLastError();
}
DTF_API int dtf_dropout(const void* x, void* y, long n, float keep, unsigned long long seed, const void* ctr,
                        void* stream) {
  if (n & 7) return -1;
  hipLaunchKernelGGL(dropout_kernel, GRID(n / 8), (const bf16_t*)x, (bf16_t*)y, n / 8, keep_threshold(keep),
                     (uint64_t)seed, (const uint64_t*)ctr);
  return (int)hipGetLastError();
}
DTF_API int dtf_rng_advance(void* ctr, void* stream) {
  hipLaunchKernelGGL(rng_advance_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, (uint64_t*)ctr);
  return (int)hipGetLastError();
}
// Column sums (BiasAddGrad): partial rows into ws, then a deterministic row reduction into out.
DTF_API int dtf_colsum(const void* x, long M, int N, float* out, int accumulate, float* ws, long ws_elems,
                       void* stream) {
  if (N & 7) return -1;
  hipStream_t st = (hipStream_t)stream;
  const long gx = (N + 255) / 256;
  long splits = std::max<long>(1, std::min<long>((M + 31) / 32, std::max<long>(1, 2048 / gx)));
  splits = std::min<long>(splits, std::max<long>(1, ws_elems / N));
  const long rpb = (M + splits - 1) / splits;
  splits = (M + rpb - 1) / rpb;
  if (M == 0) {
    if (!accumulate) (void)hipMemsetAsync(out, 0, sizeof(float) * N, st);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(colsum_part_kernel, dim3((unsigned)gx, (unsigned)splits), dim3(256), 0, st, (const bf16_t*)x,
                     M, N, rpb, ws);
  dtf_sum_rows(ws, N, (int)splits, N, out, accumulate, stream);
  return (int)hipGetLastError();
}
DTF_API int dtf_embed_fwd(const void* t1, const long* i1, const void* t2, const long* i2, const void* t3,
                          const long* i3, void* out, long T, int D, int pos_mod, void* stream) {
  if (D & 7) return -1;
  hipLaunchKernelGGL(embed_fwd_kernel, GRID(T * (D / 8)), (const bf16_t*)t1, i1, (const bf16_t*)t2, i2,
                     (const bf16_t*)t3, i3, (bf16_t*)out, T, D, pos_mod < 1 ? 1 : pos_mod);
  return (int)hipGetLastError();
}
// Large-table embedding gradient from sorted ids (see embed_bwd_sorted_kernel); dt must be pre-zeroed.
DTF_API int dtf_embed_bwd_sorted(const void* dy, const long* sid, const long* perm, float* dt, long T, int D,
                                 void* stream) {
  if (D & 7) return -1;
  long blocks = std::min<long>((T + 3) / 4, 4096);
  hipLaunchKernelGGL(embed_bwd_sorted_kernel, dim3((unsigned)std::max<long>(blocks, 1)), dim3(256), 0,
                     (hipStream_t)stream, (const bf16_t*)dy, sid, perm, dt, T, D);
  return (int)hipGetLastError();
}
// Small-table (V <= 16) embedding gradient: out[V][D] (+)= sum over tokens.
DTF_API int dtf_embed_bwd_small(const void* dy, const long* idx, float* out, long T, int D, int V, int accumulate,
                                float* ws, long ws_elems, void* stream) {
  if ((D & 7) || V < 1 || V > 16 || D > 2048 || T <= 0) return T <= 0 ? 0 : -1;
  hipStream_t st = (hipStream_t)stream;
  const long VD = (long)V * D;
  if (ws_elems < VD) return -1;
  long blocks = std::max<long>(1, std::min<long>((T + 31) / 32, 2048));
  blocks = std::min<long>(blocks, std::max<long>(1, ws_elems / VD));
  const long rpb = (T + blocks - 1) / blocks;
  blocks = (T + rpb - 1) / rpb;
  const int nc = (D / 8 + 63) / 64;
#define EBR(VR, NC) \
  hipLaunchKernelGGL((embed_bwd_regs_kernel<VR, NC>), dim3((unsigned)blocks), dim3(64), 0, st, (const bf16_t*)dy, idx, \
                     T, D, V, vb, rpb, ws)
#define EBR_NC(VR) \
  if (nc == 1) EBR(VR, 1); else if (nc == 2) EBR(VR, 2); else EBR(VR, 4)
  for (int vb = 0; vb < V; vb += 4) {
    const int vr = V - vb;
    if (vr == 1) EBR_NC(1);
    else if (vr == 2) EBR_NC(2);
    else EBR_NC(4);
  }
#undef EBR_NC
#undef EBR
  dtf_sum_rows(ws, VD, (int)blocks, VD, out, accumulate, stream);
  return (int)hipGetLastError();
}
DTF_API int dtf_softmax_ce(const void* logits, int in_f32, const long* labels, float* loss, void* dlogits,
                           int grad_f32, long rows, int V, float gscale, float smooth, void* stream) {
  hipLaunchKernelGGL(softmax_ce_kernel, dim3(rows), dim3(256), 0, (hipStream_t)stream, logits, in_f32, labels, loss,
                     dlogits, grad_f32, V, gscale, smooth);
  return (int)hipGetLastError();
}
DTF_API int dtf_softmax_ce_fwd(const void* logits, int in_f32, const long* labels, float* loss, float* lse, long rows,
                               int V, float smooth, void* stream) {
  if ((reinterpret_cast<uintptr_t>(logits) & 1) || rows <= 0) return rows <= 0 ? 0 : -1;
  hipLaunchKernelGGL(softmax_ce_fwd_kernel, dim3(rows), dim3(256), 0, (hipStream_t)stream, logits, in_f32, labels, loss,
                     lse, V, smooth);
  return (int)hipGetLastError();
}
DTF_API int dtf_softmax_ce_bwd(const void* logits, int in_f32, const long* labels, const float* lse,
                               const float* dloss, void* dl, long rows, int V, float smooth, void* stream) {
  if (rows <= 0) return 0;
  hipLaunchKernelGGL(softmax_ce_bwd_kernel, dim3(rows), dim3(256), 0, (hipStream_t)stream, logits, in_f32, labels, lse,
                     dloss, dl, V, smooth);
  return (int)hipGetLastError();
}
DTF_API int dtf_softmax_fwd(const void* x, void* y, long rows, int Sq, int Sk, float scale, int causal,
                            const float* add_mask, void* stream) {
  hipLaunchKernelGGL(softmax_fwd_kernel, dim3(rows), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                     (bf16_t*)y, Sq, Sk, scale, causal, add_mask);
  return (int)hipGetLastError();
}
DTF_API int dtf_softmax_bwd(const void* y, const void* dy, void* dx, long rows, int Sk, float scale, void* stream) {
  hipLaunchKernelGGL(softmax_bwd_kernel, dim3(rows), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)y,
                     (const bf16_t*)dy, (bf16_t*)dx, Sk, scale);
  return (int)hipGetLastError();
}
