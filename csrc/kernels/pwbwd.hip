// Fused backward of a channel-REDUCING 1x1 stride-1 convolution (ResNet-50 stage-1 bottleneck c3 and stride-1
// projection: K_out = 256 output channels from C_in = 64): ONE pass over dY computes both
//   dX[p][c]  = sum_k dY[p][k] W[k][c]          (+ the BatchNorm-backward partial rows of dX, MODE 3 style), and
//   dW[k][c] += sum_p dY[p][k] X[p][c]          (whole filter in the block's accumulators, one f32 partial per block).
// The separate kernels read dY — the 4x-wide tensor, 4 of the 5 activation widths either of them reads — twice (the
// dgrad on the main stream, the wgrad on the side stream: 1.64 GB each per layer at batch 1024). Here each 64-pixel
// dY tile arrives once by LDS-DMA as a K-outer image that serves both products: the weight gradient reads it
// transposed (ds_read_b64_tr_b16, frag_kouter's addressing), the data gradient row-wise (16-B reads at the same
// swizzled chunks) against the filter held in registers. X (the layer input, 64 channels) rides in the same ring.
// The dX tile is staged through LDS and stored as 16-B row chunks with the BN partials of the stored values.
// pw_bwd_bn_kernel (below) goes further: dY itself is never stored — it is the BatchNorm(+ReLU) backward of the conv
// output y, computed per tile from dout, y and the ReLU bits (stage 1 and stage 2 shapes); optionally y is not stored
// either and is recomputed from the X tile (YR), and the same pass takes a projection shortcut's BN-backward sums (SC).
// Measured effects: profiles/r6_fused_1x1_backward.txt.
// Reference op: the Conv2D gradients of the model trainer/task.py:62-71 builds.
#include "gemm_core.h"

namespace dtf {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));

struct PbArgs {
  const bf16_t* dY;   // [P][K]
  const bf16_t* X;    // [P][C]
  const bf16_t* Wck;  // [C][K] (the conv filter as [C][1][1][K])
  bf16_t* dX;         // [P][C]
  const bf16_t* bnx;  // optional BN-backward partials of dX: BN input [P][C], its ReLU bits, batch mean
  const uint8_t* bnmask;
  const float* bnmean;
  float* part;        // [slots][2C]
  float* ws;          // [slots][K][C] weight-gradient partials
  int P, tiles_p, slots;
};

template <int R>
__device__ __forceinline__ v8bf tr_frag(const char* lds, int cb, int kk, int lane) {
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

// row fragment of the same K-outer image: pixel row pr + (lane & 15), channels 32 s + 8 (lane >> 4) .. +7
template <int R>
__device__ __forceinline__ v8bf row_frag(const char* lds, int pr, int s, int lane) {
  const int row = pr + (lane & 15);
  const int c16 = 4 * s + (lane >> 4);
  const int pc = c16 ^ (kouter_swz<R>(row) << 1);
  const uint32_t addr = (uint32_t)(uintptr_t)LDS_PTR(char, lds + row * (R * 2) + pc * 16);
  v4i r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(addr));
  return __builtin_bit_cast(v8bf, r);
}

template <int R>
struct KoDma {  // LDS-DMA of a [64 pixel][R] slice into the K-outer image (pwwgrad.hip WgOperand)
  static constexpr int L = R / 32;
  __amdgpu_buffer_rsrc_t rsrc;
  int kr[L], coff[L];
  __device__ __forceinline__ void init(const bf16_t* p, long rows) {
    const int t = threadIdx.x;
    rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)(rows * R * 2), 0x00020000);
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int pb = i * 4096 + t * 16;
      kr[i] = pb / (R * 2);
      coff[i] = ((((pb % (R * 2)) >> 4) ^ (kouter_swz<R>(kr[i]) << 1)) * 16);
    }
  }
  __device__ __forceinline__ void issue(int p0, int P, char* lds) {
    const int wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int p = p0 + kr[i];
      const uint32_t off = p < P ? (uint32_t)(p * (R * 2) + coff[i]) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsrc, (__attribute__((address_space(3))) void*)(lds + i * 4096 + wave * 1024), 16, off, 0, 0, 0);
    }
  }
};

template <int K, int C>
__global__ void __launch_bounds__(256, 1) pw_bwd_kernel(PbArgs a) {
  static_assert(K == 256 && C == 64, "the stage-1 shape: 4 waves x 64 filter rows, 4 waves x 16 dX columns");
  constexpr int IMG_Y = 64 * K * 2, IMG_X = 64 * C * 2, IMG = IMG_Y + IMG_X, NBUF = 3;
  constexpr int LD = K / 32 + C / 32;     // DMA instructions per thread per tile
  constexpr int SROW = C + 8;             // staged dX row (bf16), 16-B pad
  constexpr int CH = C / 8;               // 16-B chunks per dX row
  constexpr int ST = 64 * CH / 256;       // dX chunks per thread per tile
  __shared__ __attribute__((aligned(16))) char smem[NBUF * IMG + 64 * SROW * 2];
  char* stg = smem + NBUF * IMG;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int slot = blockIdx.x;

  // the wave's dgrad filter slice: W[c = 16 wave + (lane & 15)][k = 32 s + 8 (lane >> 4) .. +7]
  v8bf fw[K / 32];
#pragma unroll
  for (int s = 0; s < K / 32; ++s)
    fw[s] = *reinterpret_cast<const v8bf*>(a.Wck + (long)(16 * wave + (lane & 15)) * K + 32 * s + 8 * (lane >> 4));
  // consume them here, before any DMA is in flight: otherwise the compiler places their vmcnt waits at the first
  // MFMA inside the tile loop, where every iteration would then drain the prefetch
#pragma unroll
  for (int s = 0; s < K / 32; ++s) asm volatile("" ::"v"(fw[s]));

  KoDma<K> dmy;
  KoDma<C> dmx;
  dmy.init(a.dY, a.P);
  dmx.init(a.X, a.P);
  auto issue = [&](int tile, int buf) {
    char* img = smem + buf * IMG;
    dmy.issue(tile * 64, a.P, img);
    dmx.issue(tile * 64, a.P, img + IMG_Y);
  };
  const int step = a.slots;
  const int n_mine = slot < a.tiles_p ? (a.tiles_p - slot + step - 1) / step : 0;
  if (n_mine > 0) issue(slot, 0);
  if (n_mine > 1) issue(slot + step, 1);

  // BN partials of dX: this thread's 8-channel chunk is fixed (256 % CH == 0)
  const int ch = t % CH, nch = ch * 8;
  const __amdgpu_buffer_rsrc_t dxr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.dX, (short)0, (int)((long)a.P * C * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t xbr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.bnx, (short)0, a.bnmean ? (int)((long)a.P * C * 2) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t xmr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.bnmask, (short)0, a.bnmask ? (int)((long)a.P * C / 8) : 0, 0x00020000);
  const uint32_t xm_or = a.bnmask ? 0u : 0xFFu;
  float mu[8], bs[8], bq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    bs[j] = bq[j] = 0.f;
    mu[j] = a.bnmean ? a.bnmean[nch + j] : 0.f;
  }

  v4f aw[4][4];  // weight gradient: wave rows k = 64 wave + 16 j, columns c = 16 i (acc[i][j]: lane 4 c of one k)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) aw[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};

  for (int it = 0; it < n_mine; ++it) {
    // tile `it` landed. Issued after it: tile it+1's DMA (a dummy one past the last tile; none when n_mine == 1 at
    // it 0) and, from iteration 1 on, tile it-1's ST stores
    if (it == 0) {
      if (n_mine > 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LD) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LD + ST) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const int tile = slot + it * step;
    // this tile's BN inputs and mask bytes, in flight under the MFMAs (issued before tile it+2's DMA)
    uint4 xv[ST];
    uint32_t xmb[ST];
#pragma unroll
    for (int k = 0; k < ST; ++k) {
      const int p = tile * 64 + ((t + 256 * k) / CH);
      const uint32_t e = (uint32_t)p * C + nch;
      const bool ok = p < a.P;
      xv[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xbr, ok ? e * 2u : 0x80000000u, 0, 0));
      xmb[k] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(xmr, ok ? e >> 3 : 0x80000000u, 0, 0);
    }
    // (issued unconditionally — past the last tile every row is out of range and the ring buffer no tile uses gets
    // zeros — so the compiler's wait counts for the loads above stay the same on every iteration)
    issue(it + 2 < n_mine ? slot + (it + 2) * step : a.tiles_p, (it + 2) % NBUF);
    const char* img = smem + (it % NBUF) * IMG;

    // ---- weight gradient: D[c][k] += X^T dY over this tile's 64 pixels
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      v8bf fx[4], fy[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fx[i] = tr_frag<C>(img + IMG_Y, 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fy[j] = tr_frag<K>(img, 64 * wave + 16 * j, kk, lane);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(fx[i]));
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(fy[j]));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) aw[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fx[i], fy[j], aw[i][j], 0, 0, 0);
    }

    // ---- data gradient: dX[p][16 wave ..] = dY[p][:] W[:][16 wave ..] (lane: pixel row, 4 consecutive c)
    v4f ad[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) ad[i] = (v4f){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < K / 32; ++s) {
      v8bf fa[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = row_frag<K>(img, 16 * i, s, lane);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(fa[i]));
#pragma unroll
      for (int i = 0; i < 4; ++i) ad[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[s], fa[i], ad[i], 0, 0, 0);
    }
    // stage the bf16 dX tile (inline-asm LDS stores: see pwconv.hip stage_write)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int pl = 16 * i + (lane & 15), cl = 16 * wave + 4 * (lane >> 4);
      uint2 o;
      o.x = pack2bf(ad[i][0], ad[i][1]);
      o.y = pack2bf(ad[i][2], ad[i][3]);
      const uint32_t addr = (uint32_t)(uintptr_t)LDS_PTR(char, stg + (pl * SROW + cl) * 2);
      asm volatile("ds_write_b64 %0, %1" ::"v"(addr), "v"(o) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // the tile is staged
    // the BN loads are in: everything but tile it+2's DMA (issued after them) has completed
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LD) : "memory");
#pragma unroll
    for (int k = 0; k < ST; ++k) {
      const int pl = (t + 256 * k) / CH;
      const int p = tile * 64 + pl;
      uint4 val;
      {
        const uint32_t addr = (uint32_t)(uintptr_t)LDS_PTR(char, stg + (pl * SROW + nch) * 2);
        v4i r;
        asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(addr) : "memory");
        val = __builtin_bit_cast(uint4, r);
      }
      const uint32_t off = p < a.P ? ((uint32_t)p * C + nch) * 2u : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, val), dxr, off, 0, 0);
      const uint32_t vw[4] = {val.x, val.y, val.z, val.w}, xw[4] = {xv[k].x, xv[k].y, xv[k].z, xv[k].w};
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int r = 2 * q + h;
          const float dv = __uint_as_float(h ? (vw[q] & 0xffff0000u) : (vw[q] << 16));
          const float xx = __uint_as_float(h ? (xw[q] & 0xffff0000u) : (xw[q] << 16));
          const float dz = (((xmb[k] | xm_or) >> r) & 1u) ? dv : 0.f;
          bs[r] += dz;
          bq[r] = fmaf(dz, xx - mu[r], bq[r]);
        }
    }
  }

  // ---- weight-gradient partial of this block: lane holds c = 16 i + 4 (lane >> 4) + r of k = 64 wave + 16 j + lane&15
  float* slab = a.ws + (long)slot * K * C;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 64 * wave + 16 * j + (lane & 15);
      const int c = 16 * i + 4 * (lane >> 4);
      *reinterpret_cast<float4*>(slab + (long)k * C + c) = make_float4(aw[i][j][0], aw[i][j][1], aw[i][j][2], aw[i][j][3]);
    }
  if (!a.bnmean) return;
  // ---- one BN partial row per block: the 256 / CH threads of each chunk folded through LDS in a fixed order
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the dummy DMA past the last tile has landed too
  __syncthreads();  // every tile's reads of the ring are done
  float* red = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[t * 16 + j] = bs[j];
    red[t * 16 + 8 + j] = bq[j];
  }
  __syncthreads();
  if (t < C) {
    const int c8 = t >> 3, j = t & 7;
    float sv = 0.f, qv = 0.f;
    for (int u = c8; u < 256; u += CH) {
      sv += red[u * 16 + j];
      qv += red[u * 16 + 8 + j];
    }
    float* prow = a.part + (long)slot * 2 * C;
    prow[t] = sv;
    prow[C + t] = qv;
  }
}

// ---- the same with the BatchNorm(+ReLU) backward of the conv's output folded in: dY = a dz + b y + c per channel
// (dz = dout where the ReLU bit is set, else 0; y the conv output; a, b, c from bn_bwd_finalize) is computed per
// tile from dout / y / the mask bits in registers — bn_bwd_apply_row's arithmetic, bitwise the same bf16 dY — and
// written into the K-outer image by this kernel, so the standalone apply pass (read dout + y, write dY) and this
// kernel's read of dY disappear. The next tile's dout / y / mask chunks are loaded into registers while this tile
// is multiplied; dY images are double-buffered, X keeps its 3-deep LDS-DMA ring.
struct PbnArgs {
  PbArgs b;
  const bf16_t* dout;   // [P][K] gradient of the BN(+ReLU) output
  const bf16_t* y;      // [P][K] BN input (the conv output)
  const uint8_t* ymask; // [P][K] ReLU bits (nullptr: no ReLU)
  const float* coef;    // [3][K]
  // SC: the BatchNorm-backward reduction of a projection shortcut whose (deferred) BN output was added as this
  // layer's residual: its incoming gradient is the same masked dz, its BN input ysc [P][K] with batch mean msc;
  // one partial row per block [slots][2K] (sum dz | sum dz (ysc - msc)) — bn_bwd_apply_kernel<true>'s sums
  const bf16_t* ysc;
  const float* msc;
  float* psc;
  // YR: y is not stored — recompute it per tile as bf16(X W^T) from the X tile already in LDS and wy [K][C] (the
  // layer's forward filter), the forward pwconv's MFMA sequence (bitwise its stored values)
  const bf16_t* wy;
};

// <K, C, BMP, CB>: BMP pixels per tile; each block owns CB of the C columns (C / CB blocks per pixel slot, on one XCD
// and in step, so the second one's dout / y reads hit L2): dX[:, its CB] and dW[:, its CB]. Waves split dW by K/4
// rows and dX by 16 columns.
template <int K, int C, int BMP, int CB, bool SC = false, bool YR = false>
__global__ void __launch_bounds__(256, 1) pw_bwd_bn_kernel(PbnArgs A) {
  static_assert(CB == 64 && BMP % 32 == 0 && BMP <= 64 && C % CB == 0, "geometry");
  static_assert(!SC || C == CB, "the shortcut sums are taken by the only block of a pixel slot");
  static_assert(!YR || (C == CB && BMP == 64 && K == 256), "y recompute: the stage-1 shape (one block per slot)");
  constexpr int NH = C / CB;                   // blocks per pixel slot
  constexpr int FK = K / 4 / 16;               // dW row fragments per wave
  constexpr int FP = BMP / 16;                 // dX pixel fragments
  constexpr int NKK = BMP / 32;                // 32-pixel MFMA k-substeps per tile
  constexpr int IMG_Y = BMP * K * 2, IMG_X = BMP * CB * 2;
  constexpr int LDX = IMG_X / 4096;            // X DMA instructions per thread per tile
  constexpr int U = BMP * (K / 8) / 256;       // dY chunks per thread per tile
  constexpr int RPT = 256 / (K / 8);           // rows covered by one pass of the 256 threads
  constexpr int LR = (3 + (SC ? 1 : 0) - (YR ? 1 : 0)) * U;  // register loads per thread per tile (dout, y, mask, ysc)
  constexpr int YROW = K + 8;                  // YR: staged y row (bf16), 16-B pad
  constexpr int SROW = CB + 8, CH = CB / 8, ST = BMP * CH / 256;
  static_assert(LDX >= 1 && ST >= 1 && U >= 1 && RPT >= 1, "geometry");
  __shared__ __attribute__((aligned(16))) char smem[2 * IMG_Y + 3 * IMG_X + BMP * SROW * 2 + (YR ? BMP * YROW * 2 : 0)];
  char* ximg = smem + 2 * IMG_Y;
  char* stg = ximg + 3 * IMG_X;
  char* ystg = stg + BMP * SROW * 2;
  const PbArgs& a = A.b;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  // block -> (pixel slot, column block h): the NH blocks of a slot are blockIdx b, b+8, ... (one XCD)
  const int b = blockIdx.x, xcd = b & 7, j8 = b >> 3;
  const int h = j8 % NH, slot = xcd + 8 * (j8 / NH);
  const int c0 = h * CB;

  v8bf fw[K / 32];  // W[c = c0 + 16 wave + (lane & 15)][k = 32 s + 8 (lane >> 4) .. +7]
#pragma unroll
  for (int s = 0; s < K / 32; ++s)
    fw[s] = *reinterpret_cast<const v8bf*>(a.Wck + (long)(c0 + 16 * wave + (lane & 15)) * K + 32 * s +
                                           8 * (lane >> 4));
  const int cy = t % (K / 8), ry = t / (K / 8);  // this thread's dY chunk (fixed) and first row (rows ry + RPT u)
  float ka[8], kb[8], kc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ka[j] = A.coef[cy * 8 + j];
    kb[j] = A.coef[K + cy * 8 + j];
    kc[j] = A.coef[2 * K + cy * 8 + j];
  }
  // YR: the wave's forward-filter slice wy[k = 64 wave + 16 j + (lane & 15)][c = 32 kk + 8 (lane >> 4) .. +7]
  v8bf wyf[YR ? 4 : 1][2];
  if constexpr (YR) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        wyf[j][kk] = *reinterpret_cast<const v8bf*>(A.wy + (long)(64 * wave + 16 * j + (lane & 15)) * CB + 32 * kk +
                                                     8 * (lane >> 4));
#pragma unroll
    for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(wyf[j][0]), "v"(wyf[j][1]));
  }
  // consume these loads before any DMA is in flight (else their waits land inside the tile loop)
#pragma unroll
  for (int s = 0; s < K / 32; ++s) asm volatile("" ::"v"(fw[s]));
#pragma unroll
  for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(ka[j]), "v"(kb[j]), "v"(kc[j]));

  const __amdgpu_buffer_rsrc_t dr =
      __builtin_amdgcn_make_buffer_rsrc((void*)A.dout, (short)0, (int)((long)a.P * K * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t yr =
      __builtin_amdgcn_make_buffer_rsrc((void*)A.y, (short)0, (int)((long)a.P * K * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t mr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)A.ymask, (short)0, A.ymask ? (int)((long)a.P * K / 8) : 0, 0x00020000);
  const uint32_t ym_or = A.ymask ? 0u : 0xFFu;
  uint4 dv[U], yv[U], sv_[SC ? U : 1];
  uint32_t mb[U];
  const __amdgpu_buffer_rsrc_t scr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)A.ysc, (short)0, SC ? (int)((long)a.P * K * 2) : 0, 0x00020000);
  float ssc[8], qsc[8], msc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ssc[j] = qsc[j] = 0.f;
    msc[j] = SC ? A.msc[cy * 8 + j] : 0.f;
  }
  auto load_tile = [&](int tile) {  // past the last tile (tile == tiles_p) every row is out of range: zeros
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = tile * BMP + ry + RPT * u;
      const uint32_t e = (uint32_t)p * K + cy * 8;
      const bool ok = p < a.P;
      dv[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(dr, ok ? e * 2u : 0x80000000u, 0, 0));
      if constexpr (!YR)
        yv[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(yr, ok ? e * 2u : 0x80000000u, 0, 0));
      mb[u] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(mr, ok ? e >> 3 : 0x80000000u, 0, 0);
      if constexpr (SC)
        sv_[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(scr, ok ? e * 2u : 0x80000000u, 0, 0));
    }
  };
  auto transform = [&](int tile, char* img) {  // dY = a dz + b y + c -> bf16 -> the K-outer image
    if constexpr (YR) {  // this tile's y chunks from the LDS stage
      v4i yr4[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t addr = (uint32_t)(uintptr_t)LDS_PTR(char, ystg + ((ry + RPT * u) * YROW + cy * 8) * 2);
        asm volatile("ds_read_b128 %0, %1" : "=v"(yr4[u]) : "v"(addr));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int u = 0; u < U; ++u) {
        asm volatile("" : "+v"(yr4[u]));
        yv[u] = __builtin_bit_cast(uint4, yr4[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = ry + RPT * u;
      const bool ok = tile * BMP + row < a.P;
      const uint32_t dw_[4] = {dv[u].x, dv[u].y, dv[u].z, dv[u].w}, yw[4] = {yv[u].x, yv[u].y, yv[u].z, yv[u].w};
      const uint32_t bits = mb[u] | ym_or;
      float o[8];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int j = 2 * q + hh;
          float d = __uint_as_float(hh ? (dw_[q] & 0xffff0000u) : (dw_[q] << 16));
          const float yy = __uint_as_float(hh ? (yw[q] & 0xffff0000u) : (yw[q] << 16));
          if (!((bits >> j) & 1u)) d = 0.f;
          o[j] = ok ? fmaf(ka[j], d, fmaf(kb[j], yy, kc[j])) : 0.f;
          if constexpr (SC) {  // (rows past P: d is 0)
            const uint32_t sw = hh ? (sv_[u][q] & 0xffff0000u) : (sv_[u][q] << 16);
            ssc[j] += d;
            qsc[j] = fmaf(d, __uint_as_float(sw) - msc[j], qsc[j]);
          }
        }
      const v4i w4 = {(int)pack2bf(o[0], o[1]), (int)pack2bf(o[2], o[3]), (int)pack2bf(o[4], o[5]),
                      (int)pack2bf(o[6], o[7])};
      const int pc = cy ^ (kouter_swz<K>(row) << 1);
      const uint32_t addr = (uint32_t)(uintptr_t)LDS_PTR(char, img + row * (K * 2) + pc * 16);
      asm volatile("ds_write_b128 %0, %1" ::"v"(addr), "v"(w4) : "memory");
    }
  };

  // X: the [BMP][CB] column block of rows with stride C, by LDS-DMA into a K-outer image (pwwgrad.hip's mapping)
  const __amdgpu_buffer_rsrc_t xsr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.X, (short)0, (int)((long)a.P * C * 2), 0x00020000);
  int xkr[LDX], xco[LDX];
#pragma unroll
  for (int i = 0; i < LDX; ++i) {
    const int pb = i * 4096 + t * 16;
    xkr[i] = pb / (CB * 2);
    xco[i] = (c0 + ((((pb % (CB * 2)) >> 4) ^ (kouter_swz<CB>(xkr[i]) << 1)) * 8)) * 2;
  }
  auto x_issue = [&](int tile, char* img) {
#pragma unroll
    for (int i = 0; i < LDX; ++i) {
      const int p = tile * BMP + xkr[i];
      const uint32_t off = p < a.P ? (uint32_t)(p * (C * 2) + xco[i]) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          xsr, (__attribute__((address_space(3))) void*)(img + i * 4096 + wave * 1024), 16, off, 0, 0, 0);
    }
  };

  const int step = a.slots;
  const int n_mine = slot < a.tiles_p ? (a.tiles_p - slot + step - 1) / step : 0;
  auto tile_of = [&](int i) { return i < n_mine ? slot + i * step : a.tiles_p; };
  // prologue, in this order: X tile 0, registers of tile 0, X tile 1
  x_issue(tile_of(0), ximg);
  load_tile(tile_of(0));
  x_issue(tile_of(1), ximg + IMG_X);

  const int ch = t % CH, nch = c0 + ch * 8;
  const __amdgpu_buffer_rsrc_t dxr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.dX, (short)0, (int)((long)a.P * C * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t xbr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.bnx, (short)0, a.bnmean ? (int)((long)a.P * C * 2) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t xmr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.bnmask, (short)0, a.bnmask ? (int)((long)a.P * C / 8) : 0, 0x00020000);
  const uint32_t xm_or = a.bnmask ? 0u : 0xFFu;
  float mu[8], bs[8], bq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    bs[j] = bq[j] = 0.f;
    mu[j] = a.bnmean ? a.bnmean[nch + j] : 0.f;
  }
  v4f aw[4][FK];  // dW: rows k = (K/4) wave + 16 j, columns c0 + 16 i (lane: 4 consecutive c of one k)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < FK; ++j) aw[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};

  for (int it = 0; it < n_mine; ++it) {
    // this tile's registers and X image are in. Issued after them: X of tile it+1 (LDX) and, from iteration 1 on,
    // the ST dX stores of tile it-1
    if (it == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LDX) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LDX + ST) : "memory");
    const int tile = slot + it * step;
    char* yimg = smem + (it & 1) * IMG_Y;
    const char* xim = ximg + (it % 3) * IMG_X;
    if constexpr (YR) {
      // every wave's X share landed; every wave is done with the previous tile's y stage
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      // (in two halves of 32 pixels: half the accumulators)
#pragma unroll
      for (int hp = 0; hp < 2; ++hp) {
        v4f ay[2][4];  // y[p = 32 hp + 16 i + (lane & 15)][k = 64 wave + 16 j + 4 (lane >> 4) + r]
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) ay[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          v8bf xa[2];
#pragma unroll
          for (int i = 0; i < 2; ++i) xa[i] = row_frag<CB>(xim, 32 * hp + 16 * i, kk, lane);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
          for (int i = 0; i < 2; ++i) asm volatile("" : "+v"(xa[i]));
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              ay[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wyf[j][kk], xa[i], ay[i][j], 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            uint2 o;
            o.x = pack2bf(ay[i][j][0], ay[i][j][1]);
            o.y = pack2bf(ay[i][j][2], ay[i][j][3]);
            const int pl = 32 * hp + 16 * i + (lane & 15), kl = 64 * wave + 16 * j + 4 * (lane >> 4);
            const uint32_t addr = (uint32_t)(uintptr_t)LDS_PTR(char, ystg + (pl * YROW + kl) * 2);
            asm volatile("ds_write_b64 %0, %1" ::"v"(addr), "v"(o) : "memory");
          }
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // y staged
    }
    transform(tile, yimg);
    // every wave's dY share is written, every wave's X share landed; every wave is done with the dY image and the X
    // buffer that this iteration's loads below refill
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    uint4 xv[ST];
    uint32_t xmb[ST];
#pragma unroll
    for (int k = 0; k < ST; ++k) {
      const int p = tile * BMP + ((t + 256 * k) / CH);
      const uint32_t e = (uint32_t)p * C + nch;
      const bool ok = p < a.P;
      xv[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xbr, ok ? e * 2u : 0x80000000u, 0, 0));
      xmb[k] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(xmr, ok ? e >> 3 : 0x80000000u, 0, 0);
    }
    load_tile(tile_of(it + 1));
    x_issue(tile_of(it + 2), ximg + ((it + 2) % 3) * IMG_X);

    // ---- dW[k][c] += sum over the tile's pixels of dY[p][k] X[p][c]
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      v8bf fx[4], fy[FK];
#pragma unroll
      for (int i = 0; i < 4; ++i) fx[i] = tr_frag<CB>(xim, 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < FK; ++j) fy[j] = tr_frag<K>(yimg, (K / 4) * wave + 16 * j, kk, lane);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(fx[i]));
#pragma unroll
      for (int j = 0; j < FK; ++j) asm volatile("" : "+v"(fy[j]));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < FK; ++j) aw[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fx[i], fy[j], aw[i][j], 0, 0, 0);
    }
    // ---- dX[p][c0 + 16 wave ..] = dY[p][:] W[:][..]
    v4f ad[FP];
#pragma unroll
    for (int i = 0; i < FP; ++i) ad[i] = (v4f){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < K / 32; ++s) {
      v8bf fa[FP];
#pragma unroll
      for (int i = 0; i < FP; ++i) fa[i] = row_frag<K>(yimg, 16 * i, s, lane);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < FP; ++i) asm volatile("" : "+v"(fa[i]));
#pragma unroll
      for (int i = 0; i < FP; ++i) ad[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[s], fa[i], ad[i], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < FP; ++i) {
      const int pl = 16 * i + (lane & 15), cl = 16 * wave + 4 * (lane >> 4);
      uint2 o;
      o.x = pack2bf(ad[i][0], ad[i][1]);
      o.y = pack2bf(ad[i][2], ad[i][3]);
      const uint32_t addr = (uint32_t)(uintptr_t)LDS_PTR(char, stg + (pl * SROW + cl) * 2);
      asm volatile("ds_write_b64 %0, %1" ::"v"(addr), "v"(o) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // the tile is staged
    // the BN loads are in: issued after them, the next tile's registers (LR) and X image (LDX)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LR + LDX) : "memory");
#pragma unroll
    for (int k = 0; k < ST; ++k) {
      const int pl = (t + 256 * k) / CH;
      const int p = tile * BMP + pl;
      uint4 val;
      {
        const uint32_t addr = (uint32_t)(uintptr_t)LDS_PTR(char, stg + (pl * SROW + ch * 8) * 2);
        v4i r;
        asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(addr) : "memory");
        val = __builtin_bit_cast(uint4, r);
      }
      const bool ok = p < a.P;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, val), dxr,
                                             ok ? ((uint32_t)p * C + nch) * 2u : 0x80000000u, 0, 0);
      const uint32_t bits = ok ? (xmb[k] | xm_or) : 0u;
      const uint32_t vw[4] = {val.x, val.y, val.z, val.w}, xw[4] = {xv[k].x, xv[k].y, xv[k].z, xv[k].w};
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int r = 2 * q + hh;
          const float dvv = __uint_as_float(hh ? (vw[q] & 0xffff0000u) : (vw[q] << 16));
          const float xx = __uint_as_float(hh ? (xw[q] & 0xffff0000u) : (xw[q] << 16));
          const float dz = ((bits >> r) & 1u) ? dvv : 0.f;
          bs[r] += dz;
          bq[r] = fmaf(dz, xx - mu[r], bq[r]);
        }
    }
  }

  float* slab = a.ws + (long)slot * K * C;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < FK; ++j) {
      const int k = (K / 4) * wave + 16 * j + (lane & 15);
      const int c = c0 + 16 * i + 4 * (lane >> 4);
      *reinterpret_cast<float4*>(slab + (long)k * C + c) = make_float4(aw[i][j][0], aw[i][j][1], aw[i][j][2], aw[i][j][3]);
    }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the dummy loads / DMA past the last tile have landed too
  if constexpr (SC) {  // the shortcut's partial row: the RPT threads of each dY chunk folded in a fixed order
    __syncthreads();
    float* red2 = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red2[t * 16 + j] = ssc[j];
      red2[t * 16 + 8 + j] = qsc[j];
    }
    __syncthreads();
    for (int c = t; c < K; c += 256) {
      const int c8 = c >> 3, j = c & 7;
      float sv = 0.f, qv = 0.f;
      for (int u = c8; u < 256; u += K / 8) {
        sv += red2[u * 16 + j];
        qv += red2[u * 16 + 8 + j];
      }
      float* prow = A.psc + (long)slot * 2 * K;
      prow[c] = sv;
      prow[K + c] = qv;
    }
  }
  if (!a.bnmean) return;
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[t * 16 + j] = bs[j];
    red[t * 16 + 8 + j] = bq[j];
  }
  __syncthreads();
  if (t < CB) {
    const int c8 = t >> 3, j = t & 7;
    float sv = 0.f, qv = 0.f;
    for (int u = c8; u < 256; u += CH) {
      sv += red[u * 16 + j];
      qv += red[u * 16 + 8 + j];
    }
    float* prow = a.part + (long)slot * 2 * C;
    prow[c0 + t] = sv;
    prow[C + c0 + t] = qv;
  }
}

}  // namespace
}  // namespace dtf

// Fused data + weight gradient of a 1x1 stride-1 conv with K_out = 256, C_in = 64 over P pixels (see the top):
// dX (bf16 [P][C]); dW (f32 [K][C]) = or += (accumulate) the weight gradient; with bnmean, the BatchNorm-backward
// partial rows of dX (sum dz | sum dz (bnx - mean), dz = dX * bnmask bit) into part, *rows = their count.
// ws: >= 256 * K * C floats. Returns 0, or -1 when the shape is not handled (nothing launched).
DTF_API int dtf_pw_conv_bwd(const void* dY, const void* X, const void* Wck, void* dX, float* dW, int accumulate,
                            const void* bnx, const void* bnmask, const float* bnmean, float* part, int* rows,
                            float* ws, long ws_elems, long P, int K, int C, void* stream) {
  using namespace dtf;
  hipStream_t st = (hipStream_t)stream;
  if (K != 256 || C != 64) return -1;
  if (((uintptr_t)dY & 15) || ((uintptr_t)X & 15) || ((uintptr_t)Wck & 15) || ((uintptr_t)dX & 15) ||
      ((uintptr_t)bnx & 15) || !ws || !dW)
    return -1;
  if (bnmean && (!bnx || !part)) return -1;
  if (P * K * 2 >= (1l << 31) || P < 64 * 256) return -1;
  PbArgs a{};
  a.dY = (const bf16_t*)dY; a.X = (const bf16_t*)X; a.Wck = (const bf16_t*)Wck; a.dX = (bf16_t*)dX;
  a.bnx = (const bf16_t*)bnx; a.bnmask = (const uint8_t*)bnmask; a.bnmean = bnmean; a.part = part; a.ws = ws;
  a.P = (int)P;
  a.tiles_p = (int)((P + 63) / 64);
  a.slots = 256;
  if ((long)a.slots * K * C > ws_elems) return -1;
  hipLaunchKernelGGL((pw_bwd_kernel<256, 64>), dim3(a.slots), dim3(256), 0, st, a);
  if (hipGetLastError() != hipSuccess) return -1;
  dtf_sum_rows(ws, (long)K * C, a.slots, (long)K * C, dW, accumulate, st);
  if (rows) *rows = bnmean ? a.slots : 0;
  return (int)hipGetLastError();
}

// dtf_pw_conv_bwd with the conv output's BatchNorm(+ReLU) backward applied on the fly (see pw_bwd_bn_kernel):
// dY = a dz + b y + c from dout, y, the ReLU bits ymask (nullptr: none) and coef [3][K] (bn_bwd_finalize's
// coefficients, dtf_bn_bwd_coef); dY itself is never stored.
// ysc / msc / psc (stage-1 shape only): the projection shortcut's BN-backward partial rows (see PbnArgs), *rsc rows.
// wy (stage-1 shape only, y == nullptr): recompute y from X and the forward filter wy [K][C] instead of reading it.
DTF_API int dtf_pw_conv_bwd_bn(const void* dout, const void* y, const void* ymask, const float* coef, const void* X,
                               const void* Wck, void* dX, float* dW, int accumulate, const void* bnx,
                               const void* bnmask, const float* bnmean, float* part, int* rows, float* ws,
                               long ws_elems, long P, int K, int C, const void* ysc, const float* msc, float* psc,
                               int* rsc, const void* wy, void* stream) {
  using namespace dtf;
  hipStream_t st = (hipStream_t)stream;
  // stage 1 (256 -> 64): one block per 64-pixel slot; stage 2 (512 -> 128): two column blocks per 32-pixel slot
  const bool s1 = K == 256 && C == 64, s2 = K == 512 && C == 128;
  if (!(s1 || s2) || !coef) return -1;
  if (((uintptr_t)dout & 15) || ((uintptr_t)y & 15) || ((uintptr_t)X & 15) || ((uintptr_t)Wck & 15) ||
      ((uintptr_t)dX & 15) || ((uintptr_t)bnx & 15) || !ws || !dW)
    return -1;
  if (bnmean && (!bnx || !part)) return -1;
  const bool sc = ysc != nullptr;
  if (sc && (!s1 || !msc || !psc || ((uintptr_t)ysc & 15))) return -1;
  const int bmp = s1 ? 64 : 32, nh = C / 64;
  PbnArgs A{};
  PbArgs& a = A.b;
  a.X = (const bf16_t*)X; a.Wck = (const bf16_t*)Wck; a.dX = (bf16_t*)dX;
  a.bnx = (const bf16_t*)bnx; a.bnmask = (const uint8_t*)bnmask; a.bnmean = bnmean; a.part = part; a.ws = ws;
  a.P = (int)P;
  a.tiles_p = (int)((P + bmp - 1) / bmp);
  a.slots = 256 / nh;
  if (P * K * 2 >= (1l << 31) || a.tiles_p < a.slots) return -1;
  A.dout = (const bf16_t*)dout; A.y = (const bf16_t*)y; A.ymask = (const uint8_t*)ymask; A.coef = coef;
  if ((long)a.slots * K * C > ws_elems) return -1;
  A.ysc = (const bf16_t*)ysc; A.msc = msc; A.psc = psc;
  A.wy = (const bf16_t*)wy;
  if (wy && (!s1 || y || ((uintptr_t)wy & 15))) return -1;
  if (!wy && !y) return -1;
  if (s1 && wy && sc) hipLaunchKernelGGL((pw_bwd_bn_kernel<256, 64, 64, 64, true, true>), dim3(256), dim3(256), 0, st, A);
  else if (s1 && wy) hipLaunchKernelGGL((pw_bwd_bn_kernel<256, 64, 64, 64, false, true>), dim3(256), dim3(256), 0, st, A);
  else if (s1 && sc) hipLaunchKernelGGL((pw_bwd_bn_kernel<256, 64, 64, 64, true>), dim3(256), dim3(256), 0, st, A);
  else if (s1) hipLaunchKernelGGL((pw_bwd_bn_kernel<256, 64, 64, 64>), dim3(256), dim3(256), 0, st, A);
  else hipLaunchKernelGGL((pw_bwd_bn_kernel<512, 128, 32, 64>), dim3(256), dim3(256), 0, st, A);
  if (hipGetLastError() != hipSuccess) return -1;
  dtf_sum_rows(ws, (long)K * C, a.slots, (long)K * C, dW, accumulate, st);
  if (rows) *rows = bnmean ? a.slots : 0;
  if (rsc) *rsc = sc ? a.slots : 0;
  return (int)hipGetLastError();
}
