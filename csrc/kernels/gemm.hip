// MFMA GEMM + implicit-GEMM convolution for gfx950: host API (kernels in gemm_core.h).
#include <cstdlib>

#include "gemm_core.h"

// Deterministic grouped row sums (split-K slabs, BN partial rows): see common.h.
__global__ void __launch_bounds__(256) dtf_group_rows_kernel(float* __restrict__ rows, long stride, int nrows,
                                                             int sg, long W, float* __restrict__ out,
                                                             int accumulate) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= W) return;
  const int r0 = blockIdx.y * sg;
  const int r1 = min(nrows, r0 + sg);
  float a8[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // independent chains: the loads stay in flight
  int r = r0;
  for (; r + 8 <= r1; r += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) a8[u] += rows[(long)(r + u) * stride + i];
  }
  for (; r < r1; ++r) a8[0] += rows[(long)r * stride + i];
  const float acc = ((a8[0] + a8[1]) + (a8[2] + a8[3])) + ((a8[4] + a8[5]) + (a8[6] + a8[7]));
  if (out) out[i] = accumulate ? out[i] + acc : acc;
  else rows[(long)r0 * stride + i] = acc;
}

// float4 form (W, stride multiples of 4, 16-B aligned rows): 4 columns per thread
__global__ void __launch_bounds__(256) dtf_group_rows4_kernel(float* __restrict__ rows, long stride, int nrows,
                                                              int sg, long W4, float* __restrict__ out,
                                                              int accumulate) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= W4) return;
  const int r0 = blockIdx.y * sg;
  const int r1 = min(nrows, r0 + sg);
  const float4* R = reinterpret_cast<const float4*>(rows);
  const long s4 = stride / 4;
  float4 a[4] = {};
  int r = r0;
  for (; r + 4 <= r1; r += 4) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = R[(long)(r + u) * s4 + i];
#pragma unroll
    for (int u = 0; u < 4; ++u) { a[u].x += v[u].x; a[u].y += v[u].y; a[u].z += v[u].z; a[u].w += v[u].w; }
  }
  for (; r < r1; ++r) {
    const float4 v = R[(long)r * s4 + i];
    a[0].x += v.x; a[0].y += v.y; a[0].z += v.z; a[0].w += v.w;
  }
  float4 acc;
  acc.x = (a[0].x + a[1].x) + (a[2].x + a[3].x);
  acc.y = (a[0].y + a[1].y) + (a[2].y + a[3].y);
  acc.z = (a[0].z + a[1].z) + (a[2].z + a[3].z);
  acc.w = (a[0].w + a[1].w) + (a[2].w + a[3].w);
  float4* dst = out ? reinterpret_cast<float4*>(out) + i : reinterpret_cast<float4*>(rows) + (long)r0 * s4 + i;
  if (out && accumulate) {
    const float4 o = *dst;
    acc.x += o.x; acc.y += o.y; acc.z += o.z; acc.w += o.w;
  }
  *dst = acc;
}

// Narrow rows (W <= 1024 floats, W % 4 == 0: the BatchNorm / LayerNorm / bias partial rows): each block sums one
// group of rows with ALL its 256 threads — W/4 float4 columns x 256/(W/4) row lanes, each lane striding the
// group's rows with 4 loads in flight — and combines the row lanes through LDS in a fixed order (deterministic).
// The one-thread-per-column form left 7/8 of a block idle and walked ~200 rows per thread serially.
__global__ void __launch_bounds__(256) dtf_group_rows_narrow_kernel(const float* __restrict__ rows, long stride,
                                                                    int nrows, int sg, int W4,
                                                                    float* __restrict__ dst, long dst_stride,
                                                                    int accumulate) {
  __shared__ float4 red[256];
  const int t = threadIdx.x, RL = 256 / W4, c = t % W4, rl = t / W4;
  const int r0 = blockIdx.y * sg, r1 = min(nrows, r0 + sg);
  float4 a[4] = {};
  if (rl < RL) {
    const float4* R = reinterpret_cast<const float4*>(rows);
    const long s4 = stride / 4;
    int r = r0 + rl;
    for (; r + 3 * RL < r1; r += 4 * RL) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = R[(long)(r + u * RL) * s4 + c];
#pragma unroll
      for (int u = 0; u < 4; ++u) { a[u].x += v[u].x; a[u].y += v[u].y; a[u].z += v[u].z; a[u].w += v[u].w; }
    }
    for (; r < r1; r += RL) {
      const float4 v = R[(long)r * s4 + c];
      a[0].x += v.x; a[0].y += v.y; a[0].z += v.z; a[0].w += v.w;
    }
  }
  float4 s;
  s.x = (a[0].x + a[1].x) + (a[2].x + a[3].x);
  s.y = (a[0].y + a[1].y) + (a[2].y + a[3].y);
  s.z = (a[0].z + a[1].z) + (a[2].z + a[3].z);
  s.w = (a[0].w + a[1].w) + (a[2].w + a[3].w);
  red[t] = s;
  __syncthreads();
  if (t < W4) {
    float4 acc = red[t];
    for (int k = 1; k < RL; ++k) {
      const float4 v = red[k * W4 + t];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    float4* o = reinterpret_cast<float4*>(dst + (long)blockIdx.y * dst_stride) + t;
    if (accumulate) {
      const float4 p = *o;
      acc.x += p.x; acc.y += p.y; acc.z += p.z; acc.w += p.w;
    }
    *o = acc;
  }
}

static bool narrow_rows_ok(const float* rows, long stride, long W) {
  return !(W & 3) && W <= 1024 && !(stride & 3) && !((uintptr_t)rows & 15);
}

// One launch: sum groups of rows into leader rows so that <= target leaders remain; returns their count
// and (via out_stride) their row stride.
DTF_API int dtf_group_rows_once(float* rows, long stride, int nrows, long W, int target, long* out_stride,
                                void* stream) {
  *out_stride = stride;
  if (nrows <= target) return nrows;
  const int sg = (nrows + target - 1) / target;
  const int groups = (nrows + sg - 1) / sg;
  if (narrow_rows_ok(rows, stride, W)) {
    hipLaunchKernelGGL(dtf_group_rows_narrow_kernel, dim3(1, groups), dim3(256), 0, (hipStream_t)stream, rows,
                       stride, nrows, sg, (int)(W / 4), rows, stride * sg, 0);
  } else {
    hipLaunchKernelGGL(dtf_group_rows_kernel, dim3((unsigned)((W + 255) / 256), groups), dim3(256), 0,
                       (hipStream_t)stream, rows, stride, nrows, sg, W, (float*)nullptr, 0);
  }
  *out_stride = stride * sg;
  return groups;
}


DTF_API long* dtf_launch_counters() {
  static long c[LC_COUNT] = {};
  return c;
}
// copies the first n counters into out (tests: ops._util.launch_counts)
DTF_API int dtf_launch_counts(long* out, int n) {
  for (int i = 0; i < n && i < LC_COUNT; ++i) out[i] = dtf_launch_counters()[i];
  return 0;
}

// Two-level deterministic reduction of `nrows` rows into out (or into row 0 if out == nullptr).
// Returns nothing; stream-ordered.
DTF_API void dtf_sum_rows(float* rows, long stride, int nrows, long W, float* out, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (W >= (1l << 16) && !(W & 3) && !(stride & 3) && !((uintptr_t)rows & 15) && !((uintptr_t)out & 15) &&
      nrows <= 64) {
    // wide rows (split-K slabs of a weight gradient): ONE float4 pass, each thread sums its 4 columns over all
    // rows with 4 interleaved accumulators (a fixed association: deterministic)
    const long W4 = W / 4;
    hipLaunchKernelGGL(dtf_group_rows4_kernel, dim3((unsigned)((W4 + 255) / 256), 1), dim3(256), 0, st, rows, stride,
                       nrows, nrows, W4, out, accumulate);
    return;
  }
  const int gx = (int)((W + 255) / 256);
  long s = stride;
  int n = nrows;
  if (out && narrow_rows_ok(rows, stride, W) && !((uintptr_t)out & 15)) {
    const int W4 = (int)(W / 4);
    if (n > 64) {  // one pass to <= 64 leader rows (written over the group's first row), ~16+ rows per group
      const int groups = std::min(64, std::max(1, n / 16));
      const int sg = (n + groups - 1) / groups;
      const int g2 = (n + sg - 1) / sg;
      hipLaunchKernelGGL(dtf_group_rows_narrow_kernel, dim3(1, g2), dim3(256), 0, st, rows, s, n, sg, W4, rows,
                         s * sg, 0);
      s *= sg;
      n = g2;
    }
    hipLaunchKernelGGL(dtf_group_rows_narrow_kernel, dim3(1, 1), dim3(256), 0, st, rows, s, n, n, W4, out, 0L,
                       accumulate);
    return;
  }
  if (gx < 64 && n > 32) {
    // narrow rows (LayerNorm/bias partials: W of a few thousand): ONE grouping pass to <= 32 leader rows,
    // then the final pass — two launches instead of a cascade of small ones
    const int sg = (n + 31) / 32;
    const int groups = (n + sg - 1) / sg;
    hipLaunchKernelGGL(dtf_group_rows_kernel, dim3(gx, groups), dim3(256), 0, st, rows, s, n, sg, W,
                       (float*)nullptr, 0);
    s *= sg;
    n = groups;
  }
  // stage 1: enough groups to fill the chip, each summing sg rows into its leader row
  while (n > 8 && gx < 2048 && gx >= 64) {
    int groups = (int)std::min<long>(n, std::max<long>(1, 1024 / gx));
    int sg = std::max(8, (n + groups - 1) / groups);
    groups = (n + sg - 1) / sg;
    hipLaunchKernelGGL(dtf_group_rows_kernel, dim3(gx, groups), dim3(256), 0, st, rows, s, n, sg, W,
                       (float*)nullptr, 0);
    s *= sg;
    n = groups;
    if (n <= 8) break;
  }
  hipLaunchKernelGGL(dtf_group_rows_kernel, dim3(gx, 1), dim3(256), 0, st, rows, s, n, n, W, out, accumulate);
}

namespace dtf {

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN, int AM, int BMODE, int PIPE = 2>
static void launch_t(GemmArgs& a, hipStream_t st) {
  a.tiles_m = cdiv(a.M, BM);
  a.tiles_n = cdiv(a.N, BN);
  dim3 grid(a.tiles_m * a.tiles_n, 1, a.batch * a.splitk);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, AM, BMODE, 0, PIPE>), grid, dim3(NT), 0, st, a);
}

template <int AM, int BMODE>
static void launch_modes(GemmArgs& a, int tile, hipStream_t st) {
  switch (tile) {
    // 128-row tiles use ONE LDS buffer: the register-staged prefetch already overlaps the next tile's loads
    // with the MFMAs, and half the LDS per block doubles the blocks (and bytes in flight) per CU — faster
    // on every ResNet-50 conv measured (tools/conv_roofline.py --tiles; tiles 5/6 = the double-buffered forms)
    case 0: launch_t<128, 128, 2, 2, AM, BMODE, 1>(a, st); break;
    case 1: launch_t<256, 64, 4, 1, AM, BMODE>(a, st); break;
    case 2: launch_t<128, 64, 2, 2, AM, BMODE, 1>(a, st); break;
    case 4: launch_t<64, 256, 1, 4, AM, BMODE>(a, st); break;
    case 5: launch_t<128, 64, 2, 2, AM, BMODE, 2>(a, st); break;
    case 6: launch_t<128, 128, 2, 2, AM, BMODE, 2>(a, st); break;
    case 7: case 8: case 9: case 10:  // LDS-DMA staging (K-contiguous operands only; callers check)
      if constexpr (glds_mode(AM) && glds_mode(BMODE)) {
        if (tile == 7) launch_t<128, 128, 2, 2, AM, BMODE, 3>(a, st);
        else if (tile == 8) launch_t<128, 64, 2, 2, AM, BMODE, 3>(a, st);
        else if (tile == 9) launch_t<128, 128, 2, 2, AM, BMODE, 4>(a, st);
        else launch_t<128, 64, 2, 2, AM, BMODE, 4>(a, st);
      } else {
        launch_t<128, 128, 2, 2, AM, BMODE, 1>(a, st);
      }
      break;
    case 15: case 16:  // 64 x 256 LDS-DMA (one block covers 256 output channels: the A rows are read once)
      if constexpr (glds_mode(AM) && glds_mode(BMODE)) {
        if (tile == 15) launch_t<64, 256, 1, 4, AM, BMODE, 3>(a, st);
        else launch_t<64, 256, 1, 4, AM, BMODE, 4>(a, st);
      } else {
        launch_t<64, 256, 1, 4, AM, BMODE>(a, st);
      }
      break;
    default: launch_t<64, 64, 2, 2, AM, BMODE>(a, st); break;
  }
}

// Tile choice: prefer the largest tile that still yields >= ~2 waves of blocks on
// 256 CUs (2 blocks/CU at ~64 KB LDS each); narrow N -> 256x64.
static int pick_tile(long M, long N, long batch_splits, long K = 1 << 30) {
  auto blocks = [&](int bm, int bn) { return (long)cdiv(M, bm) * cdiv(N, bn) * batch_splits; };
  if (N <= 64) {
    if (blocks(128, 64) >= 512) return 2;
    if (blocks(256, 64) >= 512) return 1;
    if (blocks(128, 64) >= 256) return 2;
    return 3;
  }
  // short K (the memory-bound 1x1 convolutions): 128x64 keeps the most blocks in flight per CU
  if (K <= 256 && blocks(128, 64) >= 1024) return 2;
  if (blocks(128, 128) >= 256) return 0;
  if (blocks(128, 64) >= 256) return 2;
  return 3;
}

int gemm256_try(GemmArgs& a, int amode, int bmode, hipStream_t st, int fp8 = 0, int bn = 256);  // gemm256.hip
int gemm_w4_try(GemmArgs& a, int amode, int bmode, hipStream_t st, int bn);  // gemm_w4.hip
// 256-row tiles: the 4-wave kernel (gemm_w4.hip: 1.0-1.25x gemm256 on every transformer shape, profiles/
// r5_gemm_vs_hipblaslt.txt) when its epilogue covers the call, else the 8-wave gemm256 kernel.
static int tile256_try(GemmArgs& a, int amode, int bmode, hipStream_t st, int bn = 256) {
  if (gemm_w4_try(a, amode, bmode, st, bn) == 0) return 0;
  return gemm256_try(a, amode, bmode, st, 0, bn);
}
int conv256_try(GemmArgs& a, int amode, int bmode, int cfg, hipStream_t st, bool force);  // conv256.hip
bool conv256_on();
int pwconv_try(const void* X, const void* W, void* Y, float* stats, long M, int C, int K, hipStream_t st);  // pwconv.hip

// The 256-row pipelined LDS-DMA kernel (conv256.hip) for a convolution GEMM: forced by tiles 11-14 (variant
// tile - 11, see conv256.hip launch_cfg); by default whenever it is eligible and fills the chip. True if launched.
static bool try_conv256(GemmArgs& a, int am, int bm, int& tile, hipStream_t st) {
  if (tile >= 11 && tile <= 14) {
    if (conv256_try(a, am, bm, tile - 11, st, true) == 0) return true;
    tile = -1;
  }
  return tile < 0 && conv256_try(a, am, bm, -1, st, false) == 0;
}

// 256-row pipelined tiles (1 block/CU, ~1.12-1.24x faster per tile than 128x128, more so at long K) vs the
// 128x128 kernel (2 blocks/CU): compare the wave-quantisation efficiency of the tilings on 256 CUs. Returns the
// 256-row tile width to use (256 or 128), or 0 for the 128x128 kernel.
int pick256(long M, long N, long K, long batch) {
  const long t256 = (long)cdiv(M, 256) * cdiv(N, 256) * batch, t2x1 = (long)cdiv(M, 256) * cdiv(N, 128) * batch,
             t128 = (long)cdiv(M, 128) * cdiv(N, 128) * batch;
  // (the 8-wave kernel's 256x128 tiles are LDS-read bound with its 2x4 wave layout: GPT-2-medium 218.5k -> 210.4k
  // tok/s with them: not used)
  auto eff = [](long t, long slots) { return (double)t / (double)(((t + slots - 1) / slots) * slots); };
  const double base = 1.12 + 0.12 * (double)std::min<long>(K, 4096) / 4096.0;
  const double s256 = t256 >= 128 ? base * eff(t256, 256) : 0.0;
  const double s128 = eff(t128, 512);
  (void)t2x1;
  return s256 > s128 ? 256 : 0;
}
bool prefer256(long M, long N, long K, long batch) { return pick256(M, N, K, batch) == 256; }

// Tile rule of the bf16 GEMMs: the 4-wave kernels (gemm_w4.hip) with 256x256 or 256x128 tiles, or the 128x128 kernel
// (2 blocks/CU), by the wave-quantisation efficiency of each tiling on 256 CUs times its per-tile speed (256x128: 0.8
// of the 256x256 FLOP rate, 128x128: 0.6 — tools/bench_gemm_w4.py, profiles/r5_gemm_vs_hipblaslt.txt; e.g. M=8192
// N=1024: 128 tiles of 256x256 (half the chip) 523 TF vs 256 tiles of 256x128 761 TF). Returns 256, 128 or 0.
static int pick_w4(long M, long N, long batch) {
  const long t256 = (long)cdiv(M, 256) * cdiv(N, 256) * batch, t2x1 = (long)cdiv(M, 256) * cdiv(N, 128) * batch,
             t128 = (long)cdiv(M, 128) * cdiv(N, 128) * batch;
  auto eff = [](long t, long slots) { return (double)t / (double)(((t + slots - 1) / slots) * slots); };
  const double s256 = N > 128 ? eff(t256, 256) : 0.0;
  const double s2x1 = 0.8 * eff(t2x1, 256);
  const double s128 = 0.6 * eff(t128, 512);
  if (s256 >= s2x1 && s256 >= s128) return 256;
  if (s2x1 >= s128) return 128;
  return 0;
}

// LDS-DMA staged tiles for K-contiguous operands (both operand images filled by buffer_load ... lds):
// 128x64 synchronous (occupancy hides the DMA) almost everywhere, 128x128 double-buffered when there are
// few tiles and a long K (ResNet-50 stage 4). Measured per layer: tools/conv_roofline.py --tiles.
static int pick_glds_tile(const GemmArgs& a, int amode, int bmode) {
  if (!glds_mode(amode) || !glds_mode(bmode) || a.atomic_out) return -1;
  if (amode == OP_KCONTIG && (long)a.M * a.lda * 2 >= (1l << 31)) return -1;
  if (bmode == OP_KCONTIG && (long)a.N * a.ldb * 2 >= (1l << 31)) return -1;
  if (amode == OP_KOUTER && ((long)a.K * a.lda * 2 >= (1l << 31) || (a.M & 7))) return -1;
  if (bmode == OP_KOUTER && ((long)a.K * a.ldb * 2 >= (1l << 31) || (a.N & 7))) return -1;
  const long blocks = (long)cdiv(a.M, 128) * cdiv(a.N, 64) * a.batch * a.splitk;
  return (blocks <= 1600 && a.kchunk >= 1024) ? 9 : 8;
}

static void dispatch(GemmArgs& a, int amode, int bmode, int tile, hipStream_t st) {
  count_launch(LC_GEMM_TILE);
  if (tile < 0) tile = pick_tile(a.M, a.N, (long)a.batch * a.splitk, a.kchunk);
  if (amode == OP_KCONTIG && bmode == OP_KCONTIG) launch_modes<OP_KCONTIG, OP_KCONTIG>(a, tile, st);
  else if (amode == OP_KCONTIG && bmode == OP_KOUTER) launch_modes<OP_KCONTIG, OP_KOUTER>(a, tile, st);
  else if (amode == OP_KOUTER && bmode == OP_KOUTER) launch_modes<OP_KOUTER, OP_KOUTER>(a, tile, st);
  else if (amode == OP_KOUTER && bmode == OP_KCONTIG) launch_modes<OP_KOUTER, OP_KCONTIG>(a, tile, st);
  else if (amode == OP_IM2COL && bmode == OP_KCONTIG) launch_modes<OP_IM2COL, OP_KCONTIG>(a, tile, st);
  else if (amode == OP_DGRAD && bmode == OP_KCONTIG) launch_modes<OP_DGRAD, OP_KCONTIG>(a, tile, st);
  else if (amode == OP_IM2COL_T && bmode == OP_KCONTIG) launch_modes<OP_IM2COL_T, OP_KCONTIG>(a, tile, st);
  else if (amode == OP_DGRAD_T && bmode == OP_KCONTIG) launch_modes<OP_DGRAD_T, OP_KCONTIG>(a, tile, st);
  else if (amode == OP_KOUTER && bmode == OP_WGRADX) launch_modes<OP_KOUTER, OP_WGRADX>(a, tile, st);
  else if (amode == OP_KOUTER_R && bmode == OP_WGRADX_R) launch_modes<OP_KOUTER_R, OP_WGRADX_R>(a, tile, st);
  else if (amode == OP_WGRADX_R && bmode == OP_KOUTER_R) launch_modes<OP_WGRADX_R, OP_KOUTER_R>(a, tile, st);
}

// dst[c][r] (+)= src[r][c] for an f32 [R][C] matrix (the transposed weight gradient of dtf_conv_wgrad)
__global__ void __launch_bounds__(256) transpose_acc_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                            int R, int C, int accumulate) {
  __shared__ float tile[32][33];
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int y = ty; y < 32; y += 8)
    if (r0 + y < R && c0 + tx < C) tile[y][tx] = src[(long)(r0 + y) * C + c0 + tx];
  __syncthreads();
  for (int y = ty; y < 32; y += 8) {
    const int c = c0 + y, r = r0 + tx;
    if (c < C && r < R) {
      float* d = dst + (long)c * R + r;
      *d = accumulate ? *d + tile[tx][y] : tile[tx][y];
    }
  }
}

static ConvGeom make_geom(int N, int H, int W, int C, int K, int R, int S, int P, int Q, int sh, int sw,
                          int ph, int pw, int dh, int dw) {
  ConvGeom g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.Kout = K; g.R = R; g.S = S; g.P = P; g.Q = Q;
  g.sh = sh; g.sw = sw; g.ph = ph; g.pw = pw; g.dh = dh; g.dw = dw;
  g.dPQ = make_fastdiv(P * Q); g.dQ = make_fastdiv(Q); g.dHW = make_fastdiv(H * W);
  g.dW = make_fastdiv(W); g.dC = make_fastdiv(C); g.dS = make_fastdiv(S); g.dK = make_fastdiv(K);
  return g;
}

static uint64_t rowrep(int R, int S) {
  uint64_t r = 0;
  for (int kh = 0; kh < R && kh * S < 64; ++kh) r |= 1ull << (kh * S);
  return r;
}

// Tap-uniform gather eligibility (OP_IM2COL_T / OP_DGRAD_T): 64-channel K-tiles never straddle a tap, the tap
// mask fits 32 bits, the gathered tensor's byte offsets fit 31 bits.
static bool tap_uniform(int chans, int taps, long gathered_elems) {
  return chans % 64 == 0 && taps <= 32 && gathered_elems * 2 < (1l << 31);
}

// Split-K plan of an f32-output GEMM (a weight gradient: few output tiles over a long token K) on the 4-wave
// kernels: per tile width (256x256 at speed 1, 256x128 at 0.8, see pick_w4) the split count s (<= K/1024, <= 16)
// that maximises speed x the wave-quantisation efficiency of tiles x s blocks on 256 CUs, less 3% per extra split
// (the f32 slab round trip and its reduction). Returns s (1 = no split) and the tile width in bn; bn = 0 when K is
// too short to consider splitting (the caller's usual rule then applies).
static double g_split_penalty = 0.03;  // per extra split (dtf_set_split_penalty: A/B runs)
static int plan_w4_split(long M, long N, long K, long batch, int& bn) {
  bn = 0;
  if (K < 2048) return 0;
  auto eff = [](long t, long slots) { return (double)t / (double)(((t + slots - 1) / slots) * slots); };
  double best = -1.0;
  int best_s = 1;
  for (int w : {256, 128}) {
    if (w == 256 && N <= 128) continue;
    const long t = (long)cdiv(M, 256) * cdiv(N, w) * batch;
    const double speed = w == 256 ? 1.0 : 0.8;
    for (long sp = 1; sp <= std::min<long>(16, K / 1024); ++sp) {
      const double sc = speed * eff(t * sp, 256) - g_split_penalty * (double)(sp - 1);
      if (sc > best) { best = sc; best_s = (int)sp; bn = w; }
    }
  }
  return best_s;
}

// Split-K plan for a very long K (a 1x1-conv weight gradient over up to millions of pixels) on the 4-wave
// kernels: the tile width (256x256 or 256x128) and split count s (<= 64) that minimise a time model —
//   rounds of 1-block/CU tiles  x  K-tiles per split  x  per-K-tile time (256 CUs at ~1.5 PF: 1.43 us for a
//   256x256x64 tile, 256x128 at 0.8 of that rate)  +  for s > 1 the f32 slab round trip (8 s M N bytes at 5 TB/s)
//   and the reduction launch (5 us).
// Returns s (1 = no split) and the tile width in bn; bn = 0 when K is too short to consider splitting (the caller's
// usual rule then applies).
}  // namespace dtf
// (profiles/r5_gemm_vs_hipblaslt.txt: 0.005-0.2 measured, 0.03 kept)
DTF_API int dtf_set_split_penalty(int permille) {
  dtf::g_split_penalty = permille / 1000.0;
  return 0;
}
namespace dtf {

static int plan_w4_split_long(long M, long N, long K, long batch, int& bn) {
  bn = 0;
  if (K < 2048) return 0;
  const long kt = (K + BK - 1) / BK;
  double best = 1e30;
  int best_s = 1;
  for (int w : {256, 128}) {
    if (w == 256 && N <= 128) continue;
    const long t = (long)cdiv(M, 256) * cdiv(N, w) * batch;
    const double tau = w == 256 ? 1.43e-6 : 0.89e-6;
    for (long sp = 1; sp <= std::min<long>(64, kt / 16); ++sp) {
      const double rounds = (double)((t * sp + 255) / 256);
      double tm = rounds * (double)((kt + sp - 1) / sp) * tau;
      if (sp > 1) tm += 8.0 * (double)sp * (double)M * (double)N * (double)batch / 5e12 + 5e-6;
      if (tm < best) { best = tm; best_s = (int)sp; bn = w; }
    }
  }
  return best_s;
}

static int choose_splitk(long M, long N, long K, int tile_m, int tile_n, long batch) {
  long tiles = (long)cdiv(M, tile_m) * cdiv(N, tile_n) * batch;
  // aim for 2 blocks per CU; no split from 256 128x128 tiles on (measured: more / less splitting lost on BERT
  // and GPT-2, README "Measured and not adopted")
  constexpr long target = 512, full = 256;
  if (tiles >= full || K <= 1024) return 1;
  long want = (target + tiles - 1) / tiles;
  if (want > 256) want = 256;
  long maxs = K / 512;  // keep >= 512 of K per split
  if (want > maxs) want = maxs;
  return want < 1 ? 1 : (int)want;
}

}  // namespace dtf

using namespace dtf;

// Generic (batched) GEMM: C[b][m][n] = alpha * sum_k A(m,k) B(n,k) + beta*C (+bias, act)
//   a_kouter: A stored [K][M] (ld=lda) instead of [M][K]; b_kouter: B stored [K][N] instead of [N][K].
// stats (optional): per-M-tile partial rows [tiles_m][2N] (capacity ceil(M/64) rows); *stat_rows = tiles_m.
static int gemm_impl(const void* A, const void* B, void* C, void* aux, const float* bias, float* stats,
                     int* stat_rows, int M, int N, int K, long lda, long ldb, long ldc, int a_kouter, int b_kouter,
                     int batch, long sA, long sB, long sC, float alpha, float beta, int act, int out_f32,
                     int splitk, int tile, float* ws, long ws_elems, void* stream, const void* dact_src = nullptr,
                     int dact = 0);

DTF_API int dtf_gemm(const void* A, const void* B, void* C, void* aux, const float* bias, float* stats,
                     int* stat_rows, int M, int N, int K, long lda, long ldb, long ldc, int a_kouter, int b_kouter,
                     int batch, long sA, long sB, long sC, float alpha, float beta, int act, int out_f32,
                     int splitk, int tile, float* ws, long ws_elems, void* stream) {
  return gemm_impl(A, B, C, aux, bias, stats, stat_rows, M, N, K, lda, ldb, ldc, a_kouter, b_kouter, batch, sA, sB,
                   sC, alpha, beta, act, out_f32, splitk, tile, ws, ws_elems, stream);
}

// Weight gradient with its bias gradient fused (the BiasAddGrad of a dense layer): dW[M][N] (f32, += when beta = 1)
// = dY^T X over K tokens with dY [K][M] and X [K][N] both K-outer, and db[M] += the column sums of dY, taken by the
// 4-wave kernel from the dY fragments it already holds (GemmArgs::rowsum: 4 v_dot2c per fragment, no separate pass
// over dY). Split-K by plan_w4_split into f32 slabs of ws (splitk * M * N, then splitk * M row-sum partials), both
// reduced in a fixed order. Returns -1 when the 4-wave kernel cannot take the shape (nothing launched: the caller runs
// the plain GEMM + a column-sum pass).
DTF_API int dtf_gemm_wgrad_bias(const void* dY, const void* X, float* dW, float* db, int M, int N, int K, long lda,
                                long ldb, long ldc, float beta, float* ws, long ws_elems, void* stream) {
  if (!db || (beta != 0.f && beta != 1.f) || (M & 7) || (N & 7) || (K % BK) || ldc != N) return -1;
  hipStream_t st = (hipStream_t)stream;
  GemmArgs a{};
  a.A = (const bf16_t*)dY; a.B = (const bf16_t*)X; a.C = dW;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.batch = 1; a.alpha = 1.f; a.beta = beta; a.out_f32 = 1;
  int bn = 0;
  int s = plan_w4_split(M, N, K, 1, bn);
  if (s <= 0 || !bn) {
    s = 1;
    bn = pick_w4(M, N, 1);
    if (!bn) bn = 128;
  }
  const long mn = (long)M * N;
  if (!ws || (long)s * mn + (long)s * M > ws_elems) s = 1;
  if (!ws || (long)M > ws_elems - (s > 1 ? (long)s * mn : 0)) return -1;
  a.splitk = s;
  a.kchunk = ((K + s - 1) / s + BK - 1) / BK * BK;
  float* rows = ws + (s > 1 ? (long)s * mn : 0);
  a.rowsum = rows;
  if (s > 1) {
    a.C = ws;
    a.slab = mn;
    a.beta = 0.f;
  }
  if (gemm_w4_try(a, OP_KOUTER, OP_KOUTER, st, bn)) return -1;
  if (s > 1) {
    count_launch(LC_SPLITK);
    dtf_sum_rows(ws, mn, s, mn, dW, beta != 0.f ? 1 : 0, stream);
  }
  dtf_sum_rows(rows, M, s, M, db, 1, stream);
  return (int)hipGetLastError();
}

// Data-gradient GEMM with the activation backward fused: C[M][N] (bf16) = (A . B^T) * act'(pre), pre [M][N] with
// row stride ldc (act 1 relu, 2 gelu-tanh). The product is rounded to bf16 before the multiply, exactly as the
// unfused GEMM + dtf_act pair would.
DTF_API int dtf_gemm_dact(const void* A, const void* B, void* C, const void* pre, int act, int M, int N, int K, long lda,
                          long ldb, long ldc, int a_kouter, int b_kouter, void* stream) {
  if (!pre || (act != 1 && act != 2)) return -1;
  return gemm_impl(A, B, C, nullptr, nullptr, nullptr, nullptr, M, N, K, lda, ldb, ldc, a_kouter, b_kouter, 1, 0, 0, 0,
                   1.f, 0.f, 0, 0, 1, -1, nullptr, 0, stream, pre, act);
}

static int gemm_impl(const void* A, const void* B, void* C, void* aux, const float* bias, float* stats,
                     int* stat_rows, int M, int N, int K, long lda, long ldb, long ldc, int a_kouter, int b_kouter,
                     int batch, long sA, long sB, long sC, float alpha, float beta, int act, int out_f32,
                     int splitk, int tile, float* ws, long ws_elems, void* stream, const void* dact_src, int dact) {
  if ((N & 3) || (K & 7) || M <= 0 || N <= 0) return -1;
  if (a_kouter && (M & 7)) return -2;
  if (b_kouter && (N & 7)) return -3;
  if (dact && (out_f32 || beta != 0.f || act || aux || splitk > 1 || batch > 1)) return -8;
  if (dact) count_launch(LC_GEMM_DACT);
  if (beta != 0.f && !out_f32) count_launch(LC_BETA_BF16);
  GemmArgs a{};
  a.dact_src = (const bf16_t*)dact_src;
  a.dact = dact;
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C; a.aux = (bf16_t*)aux;
  a.bias = bias; a.stats = stats;
  a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.sA = sA; a.sB = sB; a.sC = sC;
  a.M = M; a.N = N; a.K = K; a.batch = batch < 1 ? 1 : batch;
  a.alpha = alpha; a.beta = beta; a.act = act; a.out_f32 = out_f32;
  const bool split_ok = out_f32 && (beta == 0.f || beta == 1.f) && !bias && !act && !aux && !stats && !dact;
  int w4bn = 0;  // the 4-wave kernel's tile width for a split-K plan made for it (f32 outputs: weight gradients)
  // (plan_w4_split_long's time model measured equal on BERT-base b128 / GPT-2-medium b32, 1,021-1,024k / 308.3-308.5k
  // tok/s either way: the dense weight gradients keep this plan)
  if (splitk <= 0 && split_ok && tile < 0 && K % BK == 0) splitk = plan_w4_split(M, N, K, a.batch, w4bn);
  if (splitk <= 0) splitk = split_ok ? choose_splitk(M, N, K, 128, 128, a.batch) : 1;
  a.splitk = splitk;
  a.kchunk = ((K + splitk - 1) / splitk + BK - 1) / BK * BK;
  if (splitk > 1) {
    // split-K: per-split f32 slabs + deterministic reduce (C = alpha*AB + beta*C, beta in {0,1})
    const long mn = (long)a.batch * M * N;
    if (!out_f32 || ldc != N || (a.batch > 1 && sC != (long)M * N) || (beta != 0.f && beta != 1.f)) return -4;
    if (ws == nullptr || ws_elems < 2 * mn) {
      a.splitk = splitk = 1;
      a.kchunk = (K + BK - 1) / BK * BK;
    } else {
      if ((long)splitk * mn > ws_elems) splitk = (int)(ws_elems / mn);
      a.splitk = splitk;
      a.kchunk = ((K + splitk - 1) / splitk + BK - 1) / BK * BK;
      a.C = ws;
      a.slab = (long)M * N;  // z = batch*splitk + split -> slab index
      a.beta = 0.f;
      bool big = false;
      if (w4bn) {  // the split chosen for the 4-wave kernel
        GemmArgs b = a;
        if (tile256_try(b, a_kouter ? OP_KOUTER : OP_KCONTIG, b_kouter ? OP_KOUTER : OP_KCONTIG, (hipStream_t)stream,
                        w4bn) == 0)
          big = true;
      }
      if (!big && tile < 0 && M >= 256 && N >= 256) {  // 256x256 tiles: re-split for them (>= ~1 block per CU)
        GemmArgs b = a;
        const long t256 = (long)cdiv(M, 256) * cdiv(N, 256) * a.batch;
        // one round of 1-block/CU tiles: splits so that tiles x splits <= 256 CUs, >= 1024 of K per split
        int s2 = (int)std::min<long>(std::max<long>(1, 256 / t256), std::max<long>(1, K / 1024));
        if (t256 * s2 >= 200 && (long)s2 * mn <= ws_elems) {
          b.splitk = s2;
          b.kchunk = ((K + s2 - 1) / s2 + BK - 1) / BK * BK;
          if (tile256_try(b, a_kouter ? OP_KOUTER : OP_KCONTIG, b_kouter ? OP_KOUTER : OP_KCONTIG,
                          (hipStream_t)stream) == 0) {
            big = true;
            splitk = s2;
          }
        }
      }
      if (!big) {
        const int am = a_kouter ? OP_KOUTER : OP_KCONTIG, bm = b_kouter ? OP_KOUTER : OP_KCONTIG;
        int t = tile;
        dispatch(a, am, bm, t, (hipStream_t)stream);
      }
      count_launch(LC_SPLITK);
      // slabs are [batch][splitk][M*N]: reduce each batch separately
      for (int b = 0; b < a.batch; ++b)
        dtf_sum_rows(ws + (long)b * splitk * M * N, (long)M * N, splitk, (long)M * N, (float*)C + (long)b * M * N,
                     beta != 0.f ? 1 : 0, stream);
      return (int)hipGetLastError();
    }
  }
  if (stats && (a.batch > 1 || a.splitk > 1)) return -7;
  // large K-contiguous problems: the 256x256 glds-pipelined kernel when it fills the chip
  const int bn256 = (tile < 0 && !stats && a.splitk == 1) ? pick_w4(M, N, a.batch) : 0;
  if (bn256 && tile256_try(a, a_kouter ? OP_KOUTER : OP_KCONTIG, b_kouter ? OP_KOUTER : OP_KCONTIG, (hipStream_t)stream,
                           bn256) == 0)
    return (int)hipGetLastError();
  const int am = a_kouter ? OP_KOUTER : OP_KCONTIG, bm = b_kouter ? OP_KOUTER : OP_KCONTIG;
  dispatch(a, am, bm, tile, (hipStream_t)stream);
  if (stat_rows) *stat_rows = a.tiles_m;
  return (int)hipGetLastError();
}

DTF_API int dtf_stem_fwd(const void* X, const void* Wt, void* Y, float* part, int* rows, int N, int Hs, int Ws, int C,
                         int K, int R, int S, int P, int Q, void* stream);  // stem.hip
// NHWC conv forward: Y[N,P,Q,K] = X[N,H,W,C] * W[K,R,S,C] (+bias, act, BN stats of Y)
// stats (optional): BN partial rows [tiles_m][2K] (capacity ceil(N*P*Q/64) rows); *stat_rows = tiles_m.
static int conv_fwd_impl(const void* X, const void* Wt, void* Y, const float* bias, float* stats, int* stat_rows,
                         int N, int H, int W, int C, int K, int R, int S, int P, int Q, int sh, int sw, int ph,
                         int pw, int dh, int dw, int act, int out_f32, int tile, void* stream);

DTF_API int dtf_conv_fwd(const void* X, const void* Wt, void* Y, const float* bias, float* stats, int* stat_rows,
                         int N, int H, int W, int C, int K, int R, int S, int P, int Q, int sh, int sw, int ph,
                         int pw, int dh, int dw, int act, int out_f32, int tile, void* stream) {
  return conv_fwd_impl(X, Wt, Y, bias, stats, stat_rows, N, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw, act,
                       out_f32, tile, stream);
}

DTF_API int dtf_bn_finalize(float* part, int T, const float* gamma, const float* beta, float* running_mean,
                            float* running_var, long M, int C, float momentum, float eps, float* scale,
                            float* shift, float* mean_out, float* invstd_out, void* stream);  // norm.hip

// Conv forward + training BatchNorm statistics AND their finalize: the conv launch writes per-tile partial rows of
// sum / sum of squares, dtf_bn_finalize reduces them in a fixed order and writes scale/shift/mean/invstd and the
// running statistics. (An in-launch finalize by the last-arriving block measured slower and was removed in round 5:
// profiles/r4_negative_results.txt.) *fused (optional) is always 0: the API keeps the slot.
DTF_API int dtf_conv_fwd_bn(const void* X, const void* Wt, void* Y, float* stats, int N, int H, int W, int C, int K,
                            int R, int S, int P, int Q, int sh, int sw, int ph, int pw, int dh, int dw, int tile,
                            const float* gamma, const float* beta, float* rmean, float* rvar, float momentum,
                            float eps, float* scale, float* shift, float* mean, float* invstd, int* fused,
                            void* stream) {
  int rows = 0;
  int rc = conv_fwd_impl(X, Wt, Y, nullptr, stats, &rows, N, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw, 0, 0,
                         tile, stream);
  if (rc) return rc;
  rc = dtf_bn_finalize(stats, rows, gamma, beta, rmean, rvar, (long)N * P * Q, K, momentum, eps, scale, shift, mean,
                       invstd, stream);
  if (fused) *fused = 0;
  return rc;
}

static int conv_fwd_impl(const void* X, const void* Wt, void* Y, const float* bias, float* stats, int* stat_rows,
                         int N, int H, int W, int C, int K, int R, int S, int P, int Q, int sh, int sw, int ph,
                         int pw, int dh, int dw, int act, int out_f32, int tile, void* stream) {
  if ((C & 7) || (K & 3)) return -1;
  if (stats && !bias && !act && !out_f32 && tile < 0 && sh == 1 && sw == 1 && ph == 0 &&
      pw == 0 && dh == 1 && dw == 1) {
    // the space-to-depth ResNet stem (C 16, K 64, 4x4): its own kernel (stem.hip); the finalize runs after
    int rows = 0;
    const int rc = dtf_stem_fwd(X, Wt, Y, stats, &rows, N, H, W, C, K, R, S, P, Q, stream);
    if (rc != -1) {
      if (stat_rows) *stat_rows = rows;
      return rc;
    }
  }
  const bool pointwise = R == 1 && S == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0;
  if (pointwise && stats && !bias && !act && !out_f32 && (tile < 0 || tile == 30)) {
    // channel-expanding 1x1 layers: the persistent register-resident-filter kernel (pwconv.hip); the BN finalize
    // then runs as its own launch over its <= 256 partial rows
    const int rows = pwconv_try(X, Wt, Y, stats, (long)N * P * Q, C, K, (hipStream_t)stream);
    if (rows > 0) {
      if (stat_rows) *stat_rows = rows;
      return (int)hipGetLastError();
    }
  }
  GemmArgs a{};
  a.g = make_geom(N, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw);
  a.g_rowrep = rowrep(a.g.R, a.g.S);
  a.A = (const bf16_t*)X; a.B = (const bf16_t*)Wt; a.C = Y; a.bias = bias; a.stats = stats;
  a.M = N * P * Q; a.N = K; a.K = R * S * C;
  a.lda = C; a.ldb = (long)R * S * C; a.ldc = K;
  a.batch = 1; a.splitk = 1; a.kchunk = (a.K + BK - 1) / BK * BK;
  a.alpha = 1.f; a.beta = 0.f; a.act = act; a.out_f32 = out_f32;
  const int am = pointwise ? OP_KCONTIG : tap_uniform(C, R * S, (long)N * H * W * C) ? OP_IM2COL_T : OP_IM2COL;
  // tap-uniform convolutions with >= 256 output channels (ResNet-50 3x3, stages 3-4): the 4-wave 256-row kernel with
  // the implicit-GEMM loader and the BN-statistics epilogue (gemm_w4.h W4Gather), tile width by pick_w4. Per layer
  // at batch 1024 (profiles/r5_conv3x3_w4.txt): stage 3 287 / 253 us vs 324 / 299 on conv256, stage 4 219 / 215 vs
  // 255 / 251; stage 2 (128 channels, 256x128 tiles) 412 / 340 vs 375 / 297 on the 128x64 LDS-DMA tile: not taken.
  // (1x1 layers stay off it: strided projections 393-605 vs 350-508 us, the 2048-channel expansion 179 vs 150,
  // the reducing c1 layers a tie — profiles/r5_conv3x3_w4.txt)
  if (am == OP_IM2COL_T && R * S > 1 && tile < 0 && K >= 256 && !bias && !act && !out_f32) {
    const int bn = pick_w4(a.M, a.N, 1);
    if (bn && gemm_w4_try(a, am, OP_KCONTIG, (hipStream_t)stream, bn) == 0) {
      if (stat_rows) *stat_rows = a.tiles_m;
      return (int)hipGetLastError();
    }
  }
  if (!try_conv256(a, am, OP_KCONTIG, tile, (hipStream_t)stream)) {
    if (tile < 0) tile = pick_glds_tile(a, am, OP_KCONTIG);
    dispatch(a, am, OP_KCONTIG, tile, (hipStream_t)stream);
  }
  if (stat_rows) *stat_rows = a.tiles_m;
  return (int)hipGetLastError();
}

// NHWC conv data-gradient: dX[N,H,W,C] = dY[N,P,Q,K] (*) Wt where Wt is the filter
// re-laid out as [C][R][S][K] (see dtf_filter_to_crsk).
// Compact filter taps for one strided-dgrad phase: dst[c][j][jw][k] = src[c][rh + sh*j][rw + sw*jw][k]
__global__ void tap_gather_kernel(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst, int C, int R, int S,
                                  int K, int rh, int rw, int sh, int sw, int nkh, int nkw) {
  const long k8 = K / 8, total = (long)C * nkh * nkw * k8;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    long t = i;
    const int kc = (int)(t % k8); t /= k8;
    const int jw = (int)(t % nkw); t /= nkw;
    const int j = (int)(t % nkh);
    const int c = (int)(t / nkh);
    const long so = (((long)c * R + rh + sh * j) * S + rw + sw * jw) * K + kc * 8;
    *reinterpret_cast<uint4*>(dst + i * 8) = *reinterpret_cast<const uint4*>(src + so);
  }
}

// NHWC conv data-gradient: dX[N][H][W][C] = sum over taps of dY gathered at the taps' output pixels x W.
// Wcrsk: filter as [C][R][S][K]. Stride > 1 (dilation 1) is decomposed into sh*sw phases by output-pixel
// parity: every phase is a stride-1 dgrad over its own pixel sub-grid using only the taps that reach it
// (compact filter gathered into ws), stored through the epilogue's row remap. This removes the
// (1 - 1/(sh*sw)) of MFMA work a direct strided gather would spend on structural zeros.
//
// Optional fused BatchNorm-backward statistics of dX (bnx != nullptr; dX is the gradient of a BN(+ReLU) output
// whose BN input is bnx [N,H,W,C] with 1-bit ReLU mask bnmask and batch mean bnmean): partial rows
// [rows][2C] of sum(dz), sum(dz*(x-mean)) go to bnpart (capacity ceil(N*H*W/64) + sh*sw rows: a strided dgrad
// writes one set per phase launch); *bnrows = rows.
static int conv_dgrad_impl(const void* dY, const void* Wcrsk, void* dX, int N, int H, int W, int C, int K, int R,
                           int S, int P, int Q, int sh, int sw, int ph, int pw, int dh, int dw, int out_f32,
                           float beta, int tile, void* ws, long ws_bf16, const void* bnx, const void* bnmask,
                           const float* bnmean, float* bnpart, int* bnrows, const void* betamask,
                           const void* bsrc2, void* stream, const void* bnrx = nullptr, const void* bnrw = nullptr);

namespace dtf {
int pwconv_dgrad_try(const void* dY, const void* Wck, void* dX, float beta, const void* betamask, const void* bnx,
                     const void* bnmask, const float* bnmean, float* part, long M, int Kc, int N, const void* bsrc2,
                     int H, int W, hipStream_t st, const void* bnrx, const void* bnrw);
}
// DTF_PW_DGRAD=0 (or dtf_set_pw_dgrad(0)) keeps the pointwise data gradients on the general GEMM tiles (A/B switch)
static int g_pw_dgrad = -1;
static bool pwdgrad_enabled() {
  if (g_pw_dgrad < 0) {
    const char* e = getenv("DTF_PW_DGRAD");
    g_pw_dgrad = !(e && e[0] == '0');
  }
  return g_pw_dgrad != 0;
}
DTF_API int dtf_set_pw_dgrad(int on) {
  g_pw_dgrad = on ? 1 : 0;
  return 0;
}
namespace dtf {
int pw_wgrad_try(const void* X, const void* dY, float* dW, long P, int C, int K, int accumulate, float* ws,
                 long ws_elems, hipStream_t st, bool split_out);
}
namespace dtf {
int c3_wgrad_try(const void* X, const void* dY, float* dW, int N, int H, int W, int accumulate, float* ws,
                 long ws_elems, hipStream_t st);
}
// DTF_C3_WGRAD=0 (or dtf_set_c3_wgrad(0)) keeps the 64-channel 3x3 weight gradients on the general tiles
static int g_c3_wgrad = -1;
static bool c3wgrad_enabled() {
  if (g_c3_wgrad < 0) {
    const char* e = getenv("DTF_C3_WGRAD");
    g_c3_wgrad = !(e && e[0] == '0');
  }
  return g_c3_wgrad != 0;
}
DTF_API int dtf_set_c3_wgrad(int on) {
  g_c3_wgrad = on ? 1 : 0;
  return 0;
}
// DTF_PW_WGRAD=0 (or dtf_set_pw_wgrad(0)) keeps the 1x1 weight gradients on the general tiles (A/B switch)
static int g_pw_wgrad = -1;
static bool pwwgrad_enabled() {
  if (g_pw_wgrad < 0) {
    const char* e = getenv("DTF_PW_WGRAD");
    g_pw_wgrad = e ? atoi(e) : 1;
  }
  return g_pw_wgrad != 0;
}
// 0 off, 1 single-tile filters, 2 also the two-tile ones
DTF_API int dtf_set_pw_wgrad(int on) {
  g_pw_wgrad = on;
  return 0;
}

DTF_API int dtf_conv_dgrad(const void* dY, const void* Wcrsk, void* dX, int N, int H, int W, int C, int K, int R,
                           int S, int P, int Q, int sh, int sw, int ph, int pw, int dh, int dw, int out_f32,
                           float beta, int tile, void* ws, long ws_bf16, const void* bnx, const void* bnmask,
                           const float* bnmean, float* bnpart, int* bnrows, const void* betamask,
                           void* stream) {
  return conv_dgrad_impl(dY, Wcrsk, dX, N, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw, out_f32, beta, tile, ws,
                         ws_bf16, bnx, bnmask, bnmean, bnpart, bnrows, betamask, nullptr, stream);
}

// dtf_conv_dgrad of a stride-1 pointwise conv whose result also adds bsrc2: the compact [N, H/2, W/2, C] data
// gradient of a stride-2 1x1 projection shortcut of the same input, at the even pixels (the shortcut's full-size
// gradient, 3/4 zeros, is never written or read). H and W even.
// The general bf16 data gradient of the ConvBN path: optional beta accumulate (+ deferred ReLU mask betamask), the
// compact stride-2 shortcut gradient bsrc2 (pointwise stride-1 convs, H and W even), and the BN-backward statistics
// of dX (bnx/bnmask/bnmean -> bnpart/bnrows).
// bnrx / bnrw: the BN input is not stored but is bf16(bnrx bnrw^T) (a 64-channel-input 1x1 conv's output, pwconv.hip
// RX): only the persistent pointwise route recomputes it; any other route returns -12 with nothing launched (the
// caller then materialises it and passes bnx).
DTF_API int dtf_conv_dgrad_x(const void* dY, const void* Wcrsk, void* dX, int N, int H, int W, int C, int K, int R,
                             int S, int P, int Q, int sh, int sw, int ph, int pw, int dh, int dw, float beta, void* ws,
                             long ws_bf16, const void* bnx, const void* bnmask, const float* bnmean, float* bnpart,
                             int* bnrows, const void* betamask, const void* bsrc2, const void* bnrx, const void* bnrw,
                             void* stream) {
  if (bsrc2) {
    if ((H & 1) || (W & 1) || R != 1 || S != 1 || sh != 1 || sw != 1 || ph != 0 || pw != 0) return -11;
    return conv_dgrad_impl(dY, Wcrsk, dX, N, H, W, C, K, 1, 1, H, W, 1, 1, 0, 0, 1, 1, 0, 1.f, -1, ws, ws_bf16, bnx,
                           bnmask, bnmean, bnpart, bnrows, nullptr, bsrc2, stream, bnrx, bnrw);
  }
  return conv_dgrad_impl(dY, Wcrsk, dX, N, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw, 0, beta, -1, ws, ws_bf16,
                         bnx, bnmask, bnmean, bnpart, bnrows, betamask, nullptr, stream, bnrx, bnrw);
}

DTF_API int dtf_conv_dgrad_addsub2(const void* dY, const void* Wcrsk, void* dX, const void* bsrc2, int N, int H, int W,
                                   int C, int K, int tile, void* ws, long ws_bf16, const void* bnx,
                                   const void* bnmask, const float* bnmean, float* bnpart, int* bnrows,
                                   void* stream) {
  if ((H & 1) || (W & 1) || !bsrc2) return -11;
  return conv_dgrad_impl(dY, Wcrsk, dX, N, H, W, C, K, 1, 1, H, W, 1, 1, 0, 0, 1, 1, 0, 1.f, tile, ws, ws_bf16, bnx,
                         bnmask, bnmean, bnpart, bnrows, nullptr, bsrc2, stream);
}

static int conv_dgrad_impl(const void* dY, const void* Wcrsk, void* dX, int N, int H, int W, int C, int K, int R,
                           int S, int P, int Q, int sh, int sw, int ph, int pw, int dh, int dw, int out_f32,
                           float beta, int tile, void* ws, long ws_bf16, const void* bnx, const void* bnmask,
                           const float* bnmean, float* bnpart, int* bnrows, const void* betamask,
                           const void* bsrc2, void* stream, const void* bnrx, const void* bnrw) {
  if ((C & 3) || (K & 7)) return -1;
  if (bnrx && (bnx || !bnrw || !bnpart || !bnmean || !bnrows)) return -9;
  if (bnx && (out_f32 || (C & 7) || !bnpart || !bnmean || !bnrows)) return -9;
  if (betamask && (out_f32 || beta == 0.f || (C & 7) || sh > 1 || sw > 1)) return -10;
  hipStream_t st = (hipStream_t)stream;
  int prow = 0;  // BN partial rows written so far (strided dgrad: one set per phase)
  auto bn_args = [&](GemmArgs& a) {
    a.betamask = (const uint8_t*)betamask;
    if (bsrc2) {
      a.bsrc = (const bf16_t*)bsrc2;
      a.dBhw = make_fastdiv((uint32_t)(H * W));
      a.dBw = make_fastdiv((uint32_t)W);
      a.bH2 = H / 2;
      a.bW2 = W / 2;
    }
    if (!bnx) return;
    a.stats = bnpart + (long)prow * 2 * C;
    a.bnx = (const bf16_t*)bnx;
    a.bnmask = (const uint8_t*)bnmask;
    a.bnmean = bnmean;
  };
  const bool phased = (sh > 1 || sw > 1) && dh == 1 && dw == 1 && ws != nullptr &&
                      ws_bf16 >= (long)C * R * S * K && !(C & 7);
  if (bnrx && phased) return -12;
  if (!phased) {
    GemmArgs a{};
    a.g = make_geom(N, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw);
    a.g_rowrep = rowrep(a.g.R, a.g.S);
    a.A = (const bf16_t*)dY; a.B = (const bf16_t*)Wcrsk; a.C = dX;
    a.M = N * H * W; a.N = C; a.K = R * S * K;
    a.lda = K; a.ldb = (long)R * S * K; a.ldc = C;
    a.batch = 1; a.splitk = 1; a.kchunk = (a.K + BK - 1) / BK * BK;
    a.alpha = 1.f; a.beta = beta; a.act = 0; a.out_f32 = out_f32;
    bn_args(a);
    bool pointwise = R == 1 && S == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0;
    const int am = pointwise ? OP_KCONTIG
                   : (sh == 1 && sw == 1 && tap_uniform(K, R * S, (long)N * P * Q * K)) ? OP_DGRAD_T : OP_DGRAD;
    int t = tile;
    // channel-reducing pointwise data gradients (ResNet-50 bottleneck c1: dY width 64..256 -> 4x the channels): the
    // persistent pointwise kernel (filter in registers, beta accumulate + BN-backward partials in its store pass)
    if (pointwise && t < 0 && !out_f32 && pwdgrad_enabled()) {
      const int rows = pwconv_dgrad_try(dY, Wcrsk, dX, beta, betamask, bnx, bnmask, bnmean,
                                        (bnx || bnrx) ? bnpart : nullptr, a.M, K, C, bsrc2, H, W, st, bnrx, bnrw);
      if (rows > 0) {
        if (bnrows) *bnrows = (bnx || bnrx) ? rows : 0;
        return (int)hipGetLastError();
      }
    }
    if (bnrx) return -12;  // (nothing launched: the caller materialises the BN input)
    // stride-1 3x3 data gradients into >= 256 channels (ResNet-50 stages 3-4): the 4-wave kernel with the dY gather
    // loader and the BN-backward statistics epilogue (profiles/r5_conv3x3_w4.txt)
    if (am == OP_DGRAD_T && R * S > 1 && t < 0 && C >= 256 && !out_f32 && beta == 0.f && !betamask && !bsrc2) {
      const int bn = pick_w4(a.M, a.N, 1);
      if (bn && gemm_w4_try(a, am, OP_KCONTIG, st, bn) == 0) {
        if (bnrows) *bnrows = bnx ? a.tiles_m : 0;
        return (int)hipGetLastError();
      }
    }
    if (!try_conv256(a, am, OP_KCONTIG, t, st))
      dispatch(a, am, OP_KCONTIG, t < 0 ? pick_glds_tile(a, am, OP_KCONTIG) : t, st);
    if (bnrows) *bnrows = bnx ? a.tiles_m : 0;
    return (int)hipGetLastError();
  }
  // phases without taps produce zeros: clear dX once unless accumulating
  bool empty_phase = false;
  for (int h0 = 0; h0 < sh; ++h0)
    for (int w0 = 0; w0 < sw; ++w0) {
      const int rh = (h0 + ph) % sh, rw = (w0 + pw) % sw;
      if (rh >= R || rw >= S) empty_phase = true;
    }
  if (empty_phase && beta == 0.f)
    (void)hipMemsetAsync(dX, 0, (size_t)N * H * W * C * (out_f32 ? 4 : 2), st);
  bf16_t* wsb = (bf16_t*)ws;
  long used = 0;
  for (int h0 = 0; h0 < sh; ++h0) {
    for (int w0 = 0; w0 < sw; ++w0) {
      const int Hs = (H - h0 + sh - 1) / sh, Ws = (W - w0 + sw - 1) / sw;
      const int rh = (h0 + ph) % sh, rw = (w0 + pw) % sw;
      if (Hs <= 0 || Ws <= 0 || rh >= R || rw >= S) continue;
      const int nkh = (R - rh + sh - 1) / sh, nkw = (S - rw + sw - 1) / sw;
      const int ch = (h0 + ph - rh) / sh, cw = (w0 + pw - rw) / sw;
      const long taps = (long)C * nkh * nkw * K;
      bf16_t* Bp = wsb + used;
      used += taps;
      const long t8 = taps / 8;
      hipLaunchKernelGGL(tap_gather_kernel, dim3((unsigned)std::min<long>((t8 + 255) / 256, 2048)), dim3(256), 0,
                         st, (const bf16_t*)Wcrsk, Bp, C, R, S, K, rh, rw, sh, sw, nkh, nkw);
      GemmArgs a{};
      a.g = make_geom(N, Hs, Ws, C, K, nkh, nkw, P, Q, 1, 1, ch, cw, 1, 1);
      a.g_rowrep = rowrep(a.g.R, a.g.S);
      a.A = (const bf16_t*)dY; a.B = Bp; a.C = dX;
      a.M = N * Hs * Ws; a.N = C; a.K = nkh * nkw * K;
      a.lda = K; a.ldb = (long)nkh * nkw * K; a.ldc = C;
      a.batch = 1; a.splitk = 1; a.kchunk = (a.K + BK - 1) / BK * BK;
      a.alpha = 1.f; a.beta = beta; a.act = 0; a.out_f32 = out_f32;
      a.crm = 1;
      a.dRm1 = make_fastdiv((uint32_t)(Hs * Ws)); a.dRm2 = make_fastdiv((uint32_t)Ws);
      a.rmH = H; a.rmW = W; a.rmsh = sh; a.rmsw = sw; a.rmh0 = h0; a.rmw0 = w0;
      bn_args(a);
      // a 1x1 tap set reading dY pixel-for-pixel is a plain GEMM over dY rows
      const bool pointwise = nkh == 1 && nkw == 1 && ch == 0 && cw == 0 && Hs == P && Ws == Q;
      const int am = pointwise ? OP_KCONTIG
                     : tap_uniform(K, nkh * nkw, (long)N * P * Q * K) ? OP_DGRAD_T : OP_DGRAD;
      // (the phase launches stay on the 128-row LDS-DMA tiles: conv256 on the 4-tap phase measured slower, stride-2
      // stage-3/4 layers 433 / 384 us vs 368 / 323 at batch 1024, profiles/r5_conv3x3_w4.txt)
      int t = tile;
      if (t >= 0 && try_conv256(a, am, OP_KCONTIG, t, st)) {
      } else {
        dispatch(a, am, OP_KCONTIG, t < 0 ? pick_glds_tile(a, am, OP_KCONTIG) : t, st);
      }
      prow += a.tiles_m;
    }
  }
  if (bnrows) *bnrows = bnx ? prow : 0;
  return (int)hipGetLastError();
}

// NHWC conv weight-gradient: dW[K][R][S][C] (f32, accumulated over split-K slabs)
//   = sum_{n,p,q} dY[n,p,q,k] * X[n, p*sh-ph+r*dh, q*sw-pw+s*dw, c]
DTF_API int dtf_conv_wgrad(const void* X, const void* dY, float* dW, int N, int H, int W, int C, int K, int R,
                           int S, int P, int Q, int sh, int sw, int ph, int pw, int dh, int dw, int accumulate,
                           int splitk, int tile, float* ws, long ws_elems, void* stream) {
  if ((C & 7) || (K & 7)) return -1;
  const int splitk_req = splitk;
  // the space-to-depth stem filter (4x4 x 16 channels -> 64): the register-staged 64-row tile beats the swapped
  // LDS-DMA default (tools/bench_stem.py: 251 vs 289 us at batch 256; round 1: 289 vs 309)
  if (tile < 0 && C == 16 && R == 4 && S == 4 && K == 64) tile = 3;
  hipStream_t st = (hipStream_t)stream;
  GemmArgs a{};
  a.g = make_geom(N, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw);
  a.g_rowrep = rowrep(a.g.R, a.g.S);
  a.A = (const bf16_t*)dY; a.B = (const bf16_t*)X;
  a.M = K; a.N = R * S * C; a.K = N * P * Q;
  a.lda = K; a.ldb = C; a.ldc = (long)R * S * C;
  a.batch = 1;
  a.alpha = 1.f; a.beta = 0.f; a.act = 0; a.out_f32 = 1;
  const long mn = (long)a.M * a.N;
  if (splitk <= 0) splitk = choose_splitk(a.M, a.N, a.K, 128, 128, 1);
  if (ws == nullptr || ws_elems < mn * 2) splitk = 1;
  else if ((long)splitk * mn > ws_elems) splitk = (int)(ws_elems / mn);
  if (splitk < 1) splitk = 1;
  a.splitk = splitk;
  a.kchunk = ((a.K + splitk - 1) / splitk + BK - 1) / BK * BK;
  bool pointwise = R == 1 && S == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0;
  // small 1x1 filters over many pixels (ResNet-50 stages 1-2): the persistent kernel, whole filter tile per block
  if (pointwise && tile < 0 && splitk_req <= 0 && pwwgrad_enabled() &&
      pw_wgrad_try(X, dY, dW, (long)N * H * W, C, K, accumulate, ws, ws_elems, st, g_pw_wgrad == 2) == 0)
    return 0;
  // 64 -> 64 channel 3x3 / stride 1 / pad 1 (ResNet-50 stage 1): the persistent kernel (c3wgrad.hip)
  if (tile < 0 && splitk_req <= 0 && C == 64 && K == 64 && R == 3 && S == 3 && sh == 1 && sw == 1 && ph == 1 &&
      pw == 1 && dh == 1 && dw == 1 && P == H && Q == W && c3wgrad_enabled() &&
      c3_wgrad_try(X, dY, dW, N, H, W, accumulate, ws, ws_elems, st) == 0)
    return 0;
  const bool small = (long)N * H * W * C * 2 < (1l << 31) && (long)N * P * Q * K * 2 < (1l << 31);
  // spatial filters: LDS-DMA staged 128x128 (measured best for every ResNet-50 3x3 filter); 1x1 filters keep
  // the register-staged kernels (tools/conv_roofline.py --only wgrad --tiles)
  const bool use_glds = small && (tile >= 7 || (tile < 0 && R * S > 1));
  // row-mapped / LDS-DMA loaders: one pixel decode per lane per K-tile row (spatial filters), buffer loads
  const bool rowmap = small && (use_glds || !pointwise);
  // Kout <= 64 spatial filters (ResNet's 56x56 stage and stem): a 128-row tile over Kout would be half empty;
  // compute dW^T [R*S*C][Kout] with the operands swapped on 128x64 tiles and transpose it into dW
  constexpr bool swap_on = true;
  // conv256: dW^T [R*S*C][Kout] = X^T . dY on the 256-row pipelined kernel (M = filter taps x channels, the long
  // dimension; N = Kout), split-K over the pixels into f32 slabs, reduced and transposed into dW
  constexpr bool c256w = false;  // (default-on measured slower than gemm_core.h on every ResNet-50 filter)
  const bool c256_forced = tile >= 11 && tile <= 14;
  if (small && ws != nullptr && (c256_forced || (tile < 0 && c256w && conv256_on())) &&
      (pointwise || (C % 8 == 0 && (dh == 1 && dw == 1)))) {
    GemmArgs b = a;
    b.A = (const bf16_t*)X; b.B = (const bf16_t*)dY;
    b.M = R * S * C; b.N = K;
    b.lda = C; b.ldb = K; b.ldc = K;
    const int cfg = c256_forced ? tile - 11 : (K <= 64 ? 2 : K >= 256 ? 1 : 0);
    const int bn = cfg == 1 ? 256 : cfg == 2 ? 64 : 128;
    const long mnT = (long)b.M * b.N;
    const long tiles = (long)cdiv(b.M, 256) * cdiv(b.N, bn);
    // ~2 rounds of 1-block/CU tiles, >= 16 K-tiles (1024 pixels) per split
    long sk = std::max<long>(1, (512 + tiles - 1) / tiles);
    sk = std::min<long>(sk, std::max<long>(1, (long)b.K / 1024));
    if ((sk + 1) * mnT > ws_elems) sk = ws_elems / mnT - 1;
    if (sk >= 1) {
      b.splitk = (int)sk;
      b.kchunk = (int)(((b.K + sk - 1) / sk + BK - 1) / BK * BK);
      b.C = ws;
      b.slab = mnT;
      b.beta = 0.f;
      b.atomic_out = 0;
      if (conv256_try(b, pointwise ? OP_KOUTER : OP_WGRADX_R, OP_KOUTER_R, cfg, st, true) == 0) {
        float* dwt = ws + (long)b.splitk * mnT;
        dtf_sum_rows(ws, mnT, b.splitk, mnT, dwt, 0, st);
        hipLaunchKernelGGL(transpose_acc_kernel, dim3(cdiv(b.N, 32), cdiv(b.M, 32)), dim3(256), 0, st, dwt, dW,
                           b.M, b.N, accumulate);
        return (int)hipGetLastError();
      }
    }
  }
  if (c256_forced) tile = -1;
  // 1x1 filters of >= 4 256x128 tiles: the plain TN GEMM dW = dY^T . X over the pixels on the 4-wave kernel (K-outer
  // operands through ds_read_b64_tr_b16), split-K into f32 slabs by plan_w4_split_long (the pixel count is the long
  // K), reduced in a fixed order into dW (smaller filters keep the 128-row tiles: one tile over millions of pixels
  // cannot fill the chip without more slab traffic than it saves)
  // (ResNet-50 b1024: 13,285 / 13,213 vs 13,236 / 13,154 img/s with the 128-row tiles, interleaved; stage-3/4 filters
  // 40-42 vs 46-49 us at b256: profiles/r5_wgrad_w4.txt)
  if (pointwise && tile < 0 && ws != nullptr && K >= 128 && C >= 128 && (long)K * C >= 4 * 256 * 128) {
    int bn = 0;
    const int s = plan_w4_split_long(a.M, a.N, a.K, 1, bn);
    if (bn && s >= 1 && (s == 1 || (long)s * mn <= ws_elems)) {
      GemmArgs b = a;
      b.splitk = s;
      b.kchunk = ((b.K + s - 1) / s + BK - 1) / BK * BK;
      if (s > 1) {
        b.C = ws;
        b.slab = mn;
        b.beta = 0.f;
      } else {
        b.C = dW;
        b.beta = accumulate ? 1.f : 0.f;
      }
      if (tile256_try(b, OP_KOUTER, OP_KOUTER, st, bn) == 0) {
        if (s > 1) {
          count_launch(LC_SPLITK);
          dtf_sum_rows(ws, mn, s, mn, dW, accumulate, st);
        }
        return (int)hipGetLastError();
      }
    }
  }
  if (swap_on && use_glds && tile < 0 && K <= 64 && R * S > 1 && ws != nullptr) {
    GemmArgs b = a;
    b.A = (const bf16_t*)X; b.B = (const bf16_t*)dY;
    b.M = R * S * C; b.N = K;
    b.lda = C; b.ldb = K; b.ldc = K;
    const long mnT = (long)b.M * b.N;
    int sk = choose_splitk(b.M, b.N, b.K, 128, 64, 1);
    if ((long)(sk + 1) * mnT > ws_elems) sk = (int)(ws_elems / mnT) - 1;
    if (sk >= 1) {
      b.splitk = sk;
      b.kchunk = ((b.K + sk - 1) / sk + BK - 1) / BK * BK;
      b.C = ws;
      b.slab = mnT;
      b.beta = 0.f;
      dispatch(b, OP_WGRADX_R, OP_KOUTER_R, 8, st);
      float* dwt = ws + (long)sk * mnT;
      dtf_sum_rows(ws, mnT, sk, mnT, dwt, 0, st);
      hipLaunchKernelGGL(transpose_acc_kernel, dim3(cdiv(b.N, 32), cdiv(b.M, 32)), dim3(256), 0, st, dwt, dW, b.M,
                         b.N, accumulate);
      return (int)hipGetLastError();
    }
  }
  if (tile < 0 && use_glds) tile = 7;
  if (tile < 0) {  // measured on ResNet-50's filters (tools/conv_roofline.py --only wgrad --tiles)
    if (a.M <= 64) tile = pointwise && a.N >= 256 ? 4 : 3;  // Kout = 64: no half-empty 128-row tiles
    else if (R * S > 1) tile = 0;                  // spatial filters: 128x128
  }
  auto run = [&]() {
    dispatch(a, rowmap ? OP_KOUTER_R : OP_KOUTER, rowmap ? OP_WGRADX_R : pointwise ? OP_KOUTER : OP_WGRADX, tile, st);
  };
  if (splitk == 1) {
    a.C = dW;
    a.beta = accumulate ? 1.f : 0.f;
    run();
    return (int)hipGetLastError();
  }
  a.C = ws;
  a.slab = mn;
  run();
  dtf_sum_rows(ws, mn, splitk, mn, dW, accumulate, st);
  return (int)hipGetLastError();
}
