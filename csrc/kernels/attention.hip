// Fused multi-head attention for gfx950: FlashAttention-2-style forward (online softmax,
// never materialising the [S, S] score matrix), and a two-kernel backward (dK/dV by key blocks, dQ by query
// blocks: no atomics, deterministic). Head dim 64, bf16 in/out, f32 accumulation on
// v_mfma_f32_16x16x32_bf16.
//
// Orientation trick: scores are computed TRANSPOSED (S^T = K Q^T, keys on MFMA rows, queries on the
// 16-lane column index), so each lane owns one query column and its softmax statistics stay in the lane
// that also owns that query's output accumulators (O^T = V^T P^T). The P fragment that feeds the second
// MFMA is assembled from the lane's own score registers; the matching V^T fragment is read with
// ds_read_b64_tr_b16 with its k-rows permuted to the same slot order (slot 4h+q <-> row 16h+4G+q).
// Q, K, V, O and the gradients are addressed with (batch, seq, head) strides, so the kernels read the
// packed QKV projection output [B, S, 3, H, 64] and write O as [B, S, H, 64] with no head transposes.
//
// Dropout on P: one 64-bit counter hash per (b*H+h, q, k/4) block gives four 16-bit uniforms, one per key
// of the block; an element is kept when its 16-bit value < thr = round(keep * 65536) and scaled by
// 65536/thr (the exact inverse of the realised keep probability). The forward and dQ kernels own 4
// consecutive keys of one query per lane (one hash per 4 elements); the dK/dV kernel owns 4 queries of
// one key and gathers the bits across its lane quad. Masking work is skipped on tiles that are entirely
// below the causal diagonal.
#include "common.h"

namespace {

constexpr int HD = 64;  // head dim
constexpr float LOG2E = 1.4426950408889634f;

struct AttnArgs {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  bf16_t* o;
  const bf16_t* dout;
  bf16_t* dq;
  bf16_t* dk;
  bf16_t* dv;
  float* lse;          // [B*H][Sq], log2 domain
  float* dvec;         // [B*H][Sq], rowsum(dO * O)
  const float* kmask;  // optional additive key mask [B][Sk] (natural-log units)
  long qsb, qss, qsh;  // strides (elements) of q and dq: batch, sequence, head
  long ksb, kss, ksh;  // strides of k/v and dk/dv
  long osb, oss, osh;  // strides of o / dout
  int B, H, Sq, Sk;
  float scale;
  uint32_t thr;     // keep threshold on 16-bit uniforms (65536 = no dropout)
  float inv_keep;   // 65536 / thr
  uint32_t seed;
  const unsigned long long* seedctr;  // optional device step counter (per-step masks under hipGraph replay)
  int nkq;          // (Sk + 3) / 4 hash blocks per query row
  int causal;
  bf16_t* ds;       // optional dS^T scratch [B*H][dsld / 64 query tiles][Sk][64] (the dS backward path)
  int dsld;         // Sq rounded up to 64
};

// XCD-aware block order: the hardware deals workgroups to the 8 XCDs round-robin by linear id, so the few blocks
// of one (batch, head) — which all read the same K/V (or Q/dO, or K) tiles — would land on different XCDs and each
// fetch those tiles into its own L2. The linear id is remapped bijectively so that every XCD owns one contiguous range
// of (head, block) pairs: a head's blocks share one L2 and its operand tiles leave HBM once.
__device__ __forceinline__ int xcd_linear() {
  const int total = (int)(gridDim.x * gridDim.y);
  const int L = (int)(blockIdx.x + gridDim.x * blockIdx.y);
  const int xcd = L & 7, qq = total >> 3, rr = total & 7;
  return (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (L >> 3);
}
__device__ __forceinline__ int attn_bx() { return xcd_linear() % (int)gridDim.x; }
__device__ __forceinline__ int attn_by() { return xcd_linear() / (int)gridDim.x; }

__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
__device__ __forceinline__ uint32_t drop_salt(const AttnArgs& a, int bh) {
  uint32_t s = a.seed;
  if (a.seedctr) {
    const unsigned long long c = *a.seedctr * 0xD1B54A32D192ED03ull;
    s ^= (uint32_t)(c ^ (c >> 32));
  }
  return fmix32(s ^ ((uint32_t)bh * 0x9E3779B9u));
}
// 4 x 16-bit uniforms for keys 4 kq .. 4 kq + 3 of query q: the counter's full fmix32, and a second word from it by
// one xor-shift-multiply round (its low half mixes both halves of the first word, its high half every bit of it)
__device__ __forceinline__ uint2 drop_bits(const AttnArgs& a, uint32_t salt, int q, int kq) {
  const uint32_t x = fmix32(((uint32_t)q * (uint32_t)a.nkq + (uint32_t)kq) ^ salt);
  return make_uint2(x, (x ^ (x >> 16)) * 0x45D9F3Bu);
}
// keep test of field j (compile-time) against thr (< 65536 whenever dropout is on): the high field of a word is
// compared whole against thr << 16, the low one after a shift — one or two VALU ops, no field extraction
template <int J>
__device__ __forceinline__ bool keep_j(uint2 b, uint32_t thr) {
  const uint32_t w = J < 2 ? b.x : b.y;
  return (J & 1) ? w < (thr << 16) : (w << 16) < (thr << 16);
}
// lanes 4 g .. 4 g + 3 (a DPP quad) all take lane 4 g + r's value: a VALU move, no LDS round trip
template <int R>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, R * 0x55, 0xF, 0xF, false);
}
__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

// ---- [64 rows][64 cols] bf16 LDS tile, 128 B rows, 16-B chunk XOR swizzle ----
__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

struct TileRegs {
  uint4 r[2];
};
__device__ __forceinline__ void tile_load(TileRegs& t, const bf16_t* base, long rs, int row0, int nrows) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int idx = threadIdx.x + 256 * u, row = idx >> 3, c = idx & 7;
    if (row0 + row < nrows)
      t.r[u] = *reinterpret_cast<const uint4*>(base + (long)(row0 + row) * rs + c * 8);
    else
      t.r[u] = make_uint4(0, 0, 0, 0);
  }
}
__device__ __forceinline__ void tile_store(const TileRegs& t, char* lds) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int idx = threadIdx.x + 256 * u, row = idx >> 3, c = idx & 7;
    *reinterpret_cast<uint4*>(lds + swz(row, c)) = t.r[u];
  }
}
// additive key-mask value (log2 units) of key `key`: -inf past the end
__device__ __forceinline__ float key_bias(const AttnArgs& a, int b, int key) {
  if (key >= a.Sk) return -INFINITY;
  return a.kmask ? a.kmask[(long)b * a.Sk + key] * LOG2E : 0.f;
}
// row fragment: lane (G, i) gets row rb + i, columns 32 kk + 8 G .. + 7
__device__ __forceinline__ v8bf frag_row(const char* lds, int rb, int kk, int lane) {
  return *reinterpret_cast<const v8bf*>(lds + swz(rb + (lane & 15), 4 * kk + (lane >> 4)));
}
// transposed fragment: lane (G, i) gets column cb + i at rows rb + 16 h + 4 G + q  (slot j = 4 h + q)
__device__ __forceinline__ v8bf frag_tr(const char* lds, int rb, int cb, int lane) {
  const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  v4s r[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = rb + 16 * h + 4 * G + q, g = (cb >> 2) + p;
    r[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, lds + swz(row, g >> 1) + (g & 1) * 8));
  }
  v8s both = __builtin_shufflevector(r[0], r[1], 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(v8bf, both);
}
// global 16-B fragment of a row (zeros when out of range)
__device__ __forceinline__ v8bf frag_global(const bf16_t* rowp, bool ok) {
  uint4 u = ok ? *reinterpret_cast<const uint4*>(rowp) : make_uint4(0, 0, 0, 0);
  return __builtin_bit_cast(v8bf, u);
}
// pack the lane's slot values: slots 0..3 from tile h=0 regs, 4..7 from tile h=1 regs
__device__ __forceinline__ v8bf pack_slots(const v4f& t0, const v4f& t1) {
  uint4 u;
  u.x = pack2bf(t0[0], t0[1]);
  u.y = pack2bf(t0[2], t0[3]);
  u.z = pack2bf(t1[0], t1[1]);
  u.w = pack2bf(t1[2], t1[3]);
  return __builtin_bit_cast(v8bf, u);
}
__device__ __forceinline__ v4f mfma(v8bf a, v8bf b, v4f c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void store4(bf16_t* p, const v4f& v, float s) {
  uint2 u;
  u.x = pack2bf(v[0] * s, v[1] * s);
  u.y = pack2bf(v[2] * s, v[3] * s);
  *reinterpret_cast<uint2*>(p) = u;
}

// ------------------------------------------------------------------------------------------------ forward
// block: 4 waves x (16 QT) queries; grid (cdiv(Sq, 64 QT), B*H)
// Tiles whose 64 keys all carry a zero additive mask (no padding, no -inf past the end) take a fast softmax: the
// max runs on the raw scores and p = exp2(s * c - m) is ONE fma + exp per score (no per-element mask add or
// subtract). smask[64] holds that flag (written by wave 0, which stages the mask).
__device__ __forceinline__ void stage_mask(float* smask, float mreg) {
  if (threadIdx.x < 64) {
    smask[threadIdx.x] = mreg;
    const bool z = __all(mreg == 0.f);
    if (threadIdx.x == 0) smask[64] = z ? 1.f : 0.f;
  }
}

template <int QT, bool DROP>
__device__ __forceinline__ void attn_fwd_body(const AttnArgs& a, const int qblk, char* sk, char* sv, float* smask) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, G = lane >> 4, i = lane & 15;
  const int bh = attn_by(), b = bh / a.H, h = bh % a.H;
  const int BM = 64 * QT;
  const int q0 = qblk * BM + w * 16 * QT;
  const bf16_t* Q = a.q + b * a.qsb + h * a.qsh;
  const bf16_t* K = a.k + b * a.ksb + h * a.ksh;
  const bf16_t* V = a.v + b * a.ksb + h * a.ksh;
  const int off = a.Sk - a.Sq;
  const float c = a.scale * LOG2E;
  constexpr bool drop = DROP;
  const uint32_t salt = drop_salt(a, bh);

  v8bf qf[QT][2];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    const int qi = q0 + 16 * qt + i;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) qf[qt][kk] = frag_global(Q + (long)qi * a.qss + 32 * kk + 8 * G, qi < a.Sq);
  }
  v4f o[4][QT];
  float m[QT], l[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    m[qt] = -INFINITY;
    l[qt] = 0.f;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt][qt] = v4f{0.f, 0.f, 0.f, 0.f};
  }
  int kend = a.Sk;
  if (a.causal) kend = min(a.Sk, qblk * BM + BM + off);
  const int ntiles = (kend + 63) / 64;
  TileRegs tk, tv;
  float mreg = 0.f;
  if (ntiles > 0) {
    tile_load(tk, K, a.kss, 0, a.Sk);
    tile_load(tv, V, a.kss, 0, a.Sk);
    if (threadIdx.x < 64) mreg = key_bias(a, b, threadIdx.x);
  }
  for (int t = 0; t < ntiles; ++t) {
    __syncthreads();
    tile_store(tk, sk);
    tile_store(tv, sv);
    stage_mask(smask, mreg);
    __syncthreads();
    const int k0 = t * 64;
    if (t + 1 < ntiles) {
      tile_load(tk, K, a.kss, k0 + 64, a.Sk);
      tile_load(tv, V, a.kss, k0 + 64, a.Sk);
      if (threadIdx.x < 64) mreg = key_bias(a, b, k0 + 64 + threadIdx.x);
    }
    v4f s[4][QT];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      const v8bf k0f = frag_row(sk, 16 * kt, 0, lane), k1f = frag_row(sk, 16 * kt, 1, lane);
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        v4f acc = {0.f, 0.f, 0.f, 0.f};
        acc = mfma(k0f, qf[qt][0], acc);
        s[kt][qt] = mfma(k1f, qf[qt][1], acc);
      }
    }
    const bool diag = a.causal && (k0 + 63 > q0 + off);  // wave-uniform
    if (!diag && smask[64] != 0.f) {
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        const int qi = q0 + 16 * qt + i;
        float mx = s[0][qt][0];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[kt][qt][r]);
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float mnew = fmaxf(m[qt], mx * c);  // (c > 0) finite: every key of the tile is valid
        const float alpha = ex2(m[qt] - mnew);
        m[qt] = mnew;
        float ls = 0.f;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
          uint2 bits = make_uint2(0, 0);
          if (drop) bits = drop_bits(a, salt, qi, (k0 >> 2) + 4 * kt + G);
          float p[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            p[r] = ex2(fmaf(s[kt][qt][r], c, -mnew));
            ls += p[r];
          }
          // dropped probabilities are zeroed here; the 1/keep scale is applied once, to the output row
          if (drop) {
            p[0] = keep_j<0>(bits, a.thr) ? p[0] : 0.f;
            p[1] = keep_j<1>(bits, a.thr) ? p[1] : 0.f;
            p[2] = keep_j<2>(bits, a.thr) ? p[2] : 0.f;
            p[3] = keep_j<3>(bits, a.thr) ? p[3] : 0.f;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) s[kt][qt][r] = p[r];
        }
        l[qt] = l[qt] * alpha + ls;
        if (__any(alpha != 1.f)) {  // the running max moved for some query of the wave
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) o[dt][qt] *= alpha;
        }
      }
    } else {
    float km[4][4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) km[kt][r] = smask[16 * kt + 4 * G + r];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      const int qi = q0 + 16 * qt + i;
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float x = fmaf(s[kt][qt][r], c, km[kt][r]);
          if (diag && k0 + 16 * kt + 4 * G + r > qi + off) x = -INFINITY;
          s[kt][qt][r] = x;
          mx = fmaxf(mx, x);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mnew = fmaxf(m[qt], mx);
      const float ms = mnew == -INFINITY ? 0.f : mnew;
      const float alpha = ex2(m[qt] - ms);
      m[qt] = mnew;
      float ls = 0.f;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        uint2 bits = make_uint2(0, 0);
        if (drop) bits = drop_bits(a, salt, qi, (k0 >> 2) + 4 * kt + G);
        float p[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          p[r] = ex2(s[kt][qt][r] - ms);
          ls += p[r];
        }
        if (drop) {
          p[0] = keep_j<0>(bits, a.thr) ? p[0] : 0.f;
          p[1] = keep_j<1>(bits, a.thr) ? p[1] : 0.f;
          p[2] = keep_j<2>(bits, a.thr) ? p[2] : 0.f;
          p[3] = keep_j<3>(bits, a.thr) ? p[3] : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) s[kt][qt][r] = p[r];
      }
      l[qt] = l[qt] * alpha + ls;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt][qt] *= alpha;
    }
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      v8bf pf[QT];
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) pf[qt] = pack_slots(s[2 * kk][qt], s[2 * kk + 1][qt]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const v8bf vf = frag_tr(sv, 32 * kk, 16 * dt, lane);
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) o[dt][qt] = mfma(vf, pf[qt], o[dt][qt]);
      }
    }
  }
  bf16_t* O = a.o + b * a.osb + h * a.osh;
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    float L = l[qt] + __shfl_xor(l[qt], 16, 64);
    L += __shfl_xor(L, 32, 64);
    const float inv = L > 0.f ? (drop ? a.inv_keep : 1.f) / L : 0.f;
    const int qi = q0 + 16 * qt + i;
    if (qi < a.Sq) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) store4(O + (long)qi * a.oss + 16 * dt + 4 * G, o[dt][qt], inv);
      if (G == 0) a.lse[(long)bh * a.Sq + qi] = L > 0.f ? m[qt] + log2f(L) : INFINITY;
    }
  }
}

// Causal launches pair the logical block x with nblk - 1 - x in one workgroup (heavy block first), so every
// workgroup walks the same number of tiles; otherwise block x is logical block nblk - 1 - x.
__device__ __forceinline__ int pair_block(int causal, int nblk, int pass) {
  const int x = attn_bx();
  if (!causal) return pass == 0 ? nblk - 1 - x : -1;
  const int heavy = nblk - 1 - x, light = x;
  return pass == 0 ? heavy : (light < heavy ? light : -1);
}
__host__ __forceinline__ unsigned pair_grid(int causal, int nblk) {
  return (unsigned)(causal ? (nblk + 1) / 2 : nblk);
}

template <int QT, bool DROP>
__global__ void __launch_bounds__(256, 2) attn_fwd_kernel(AttnArgs a, int nblk) {
  __shared__ __attribute__((aligned(16))) char sk[64 * 128];
  __shared__ __attribute__((aligned(16))) char sv[64 * 128];
  __shared__ float smask[65];
  for (int pass = 0; pass < 2; ++pass) {
    const int blk = pair_block(a.causal, nblk, pass);
    if (blk < 0) break;
    if (pass) __syncthreads();  // the previous block's last tile is no longer read
    attn_fwd_body<QT, DROP>(a, blk, sk, sv, smask);
  }
}

// ------------------------------------------------------------------------------------------------ backward
// D[q] = sum_d dO[q][d] * O[q][d]: 8 lanes per (bh, q) row, 16 B each, rows visited in memory order (heads
// innermost for the packed [B, S, H, 64] layout) so a wave reads 8 consecutive 128-B rows
// (32-bit row decode: the host guarantees B * H * Sq < 2^31; 64-bit divisions by the runtime H and Sq cost ~4x the
// whole pass on GPT-2-medium b32)
__global__ void __launch_bounds__(256) attn_dvec_kernel(AttnArgs a) {
  const int n = a.B * a.H * a.Sq;
  const int sub = threadIdx.x & 7;
  const bool hfast = a.osh == HD;
  const int step = (int)((gridDim.x * blockDim.x) >> 3);
  const uint32_t H = (uint32_t)a.H, Sq = (uint32_t)a.Sq;
  for (int r = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 3); r < n; r += step) {
    int b, h, q;
    if (hfast) {
      const uint32_t t = (uint32_t)r / H;
      h = (int)((uint32_t)r - t * H);
      const uint32_t t2 = t / Sq;
      q = (int)(t - t2 * Sq);
      b = (int)t2;
    } else {
      const uint32_t t = (uint32_t)r / Sq;
      q = (int)((uint32_t)r - t * Sq);
      const uint32_t t2 = t / H;
      h = (int)(t - t2 * H);
      b = (int)t2;
    }
    const long base = b * a.osb + h * a.osh + (long)q * a.oss + sub * 8;
    float x[8], y[8];
    load8(a.o + base, x);
    load8(a.dout + base, y);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s = fmaf(x[j], y[j], s);
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 4, 64);
    if (sub == 0) a.dvec[((long)b * a.H + h) * a.Sq + q] = s;
  }
}

// dK, dV: block = 4 waves x (16 KT) keys, loop over 64-query tiles; grid (cdiv(Sk, 64 KT), B*H).
// Query subtiles are processed in pairs (one 32-query MFMA k-step) so only 2 x KT score tiles are live.
// DS: also store dS^T (the values the dK MFMAs use) for the dQ GEMM of the dS backward path
template <int KT, bool DS>
__device__ __forceinline__ void attn_dkdv_body(const AttnArgs& a, const int kblk, char* sq, char* sdo, float* slse,
                                               float* sdv) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, G = lane >> 4, i = lane & 15;
  const int bh = attn_by(), b = bh / a.H, h = bh % a.H;
  const int BN = 64 * KT;
  const int k0w = kblk * BN + w * 16 * KT;
  const long hb = b * a.qsb + h * a.qsh, kb = b * a.ksb + h * a.ksh, ob = b * a.osb + h * a.osh;
  const bf16_t* Q = a.q + hb;
  const bf16_t* K = a.k + kb;
  const bf16_t* V = a.v + kb;
  const bf16_t* dO = a.dout + ob;
  const int off = a.Sk - a.Sq;
  const float c = a.scale * LOG2E;
  const bool drop = a.thr < 65536u;
  const uint32_t salt = drop_salt(a, bh);
  const int quad = lane & ~3, fld = i & 3;

  v8bf kf[KT][2], vf[KT][2];
  float km[KT];
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
    const int key = k0w + 16 * kt + i;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      kf[kt][kk] = frag_global(K + (long)key * a.kss + 32 * kk + 8 * G, key < a.Sk);
      vf[kt][kk] = frag_global(V + (long)key * a.kss + 32 * kk + 8 * G, key < a.Sk);
    }
    km[kt] = key_bias(a, b, key);
  }
  v4f dk[4][KT], dv[4][KT];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      dk[dt][kt] = v4f{0.f, 0.f, 0.f, 0.f};
      dv[dt][kt] = v4f{0.f, 0.f, 0.f, 0.f};
    }
  int qstart = 0;
  if (a.causal) qstart = max(0, (kblk * BN - off) / 64 * 64);
  const int ntiles = qstart >= a.Sq ? 0 : (a.Sq - qstart + 63) / 64;
  TileRegs tq, td;
  float lreg = 0.f, dreg = 0.f;
  auto load_vec = [&](int q0) {
    if (threadIdx.x < 64) {
      const int qi = q0 + threadIdx.x;
      lreg = qi < a.Sq ? a.lse[(long)bh * a.Sq + qi] : INFINITY;
      dreg = qi < a.Sq ? a.dvec[(long)bh * a.Sq + qi] : 0.f;
    }
  };
  if (ntiles > 0) {
    tile_load(tq, Q, a.qss, qstart, a.Sq);
    tile_load(td, dO, a.oss, qstart, a.Sq);
    load_vec(qstart);
  }
  for (int t = 0; t < ntiles; ++t) {
    const int q0 = qstart + t * 64;
    __syncthreads();
    tile_store(tq, sq);
    tile_store(td, sdo);
    if (threadIdx.x < 64) {
      slse[threadIdx.x] = lreg;
      sdv[threadIdx.x] = dreg;
    }
    __syncthreads();
    if (t + 1 < ntiles) {
      tile_load(tq, Q, a.qss, q0 + 64, a.Sq);
      tile_load(td, dO, a.oss, q0 + 64, a.Sq);
      load_vec(q0 + 64);
    }
    const bool diag = a.causal && (k0w + 16 * KT - 1 > q0 + off);  // wave-uniform
#pragma unroll
    for (int kq = 0; kq < 2; ++kq) {
      v4f P[2][KT], dS[2][KT];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int qs = 2 * kq + hh;
        const v8bf q0f = frag_row(sq, 16 * qs, 0, lane), q1f = frag_row(sq, 16 * qs, 1, lane);
        const v8bf d0f = frag_row(sdo, 16 * qs, 0, lane), d1f = frag_row(sdo, 16 * qs, 1, lane);
#pragma unroll
        for (int kt = 0; kt < KT; ++kt) {
          v4f s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
          s = mfma(q0f, kf[kt][0], s);
          s = mfma(q1f, kf[kt][1], s);
          dp = mfma(d0f, vf[kt][0], dp);
          dp = mfma(d1f, vf[kt][1], dp);
          const int key = k0w + 16 * kt + i;
          uint2 mine = make_uint2(0, 0);
          if (drop) mine = drop_bits(a, salt, q0 + 16 * qs + 4 * G + fld, key >> 2);
          // query row r's bits live in the quad lane whose field index is r (DPP quad broadcast); this lane's key is
          // field fld of that word: the word by fld >> 1, the half by fld & 1 (lane constants)
          uint32_t wsel[4] = {0u, 0u, 0u, 0u};
          if (drop) {
            const uint32_t b0x = quad_bcast<0>(mine.x), b0y = quad_bcast<0>(mine.y);
            const uint32_t b1x = quad_bcast<1>(mine.x), b1y = quad_bcast<1>(mine.y);
            const uint32_t b2x = quad_bcast<2>(mine.x), b2y = quad_bcast<2>(mine.y);
            const uint32_t b3x = quad_bcast<3>(mine.x), b3y = quad_bcast<3>(mine.y);
            wsel[0] = fld < 2 ? b0x : b0y;
            wsel[1] = fld < 2 ? b1x : b1y;
            wsel[2] = fld < 2 ? b2x : b2y;
            wsel[3] = fld < 2 ? b3x : b3y;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int ql = 16 * qs + 4 * G + r, qi = q0 + ql;
            float x = fmaf(s[r], c, km[kt]);
            if (diag && key > qi + off) x = -INFINITY;
            const float p = ex2(x - slse[ql]);
            float pd = p, dpv = dp[r];
            if (drop) {
              const bool z = ((fld & 1) ? wsel[r] : (wsel[r] << 16)) < (a.thr << 16);
              pd = z ? p : 0.f;  // (the 1/keep scale of dV is applied once, at its store)
              dpv = z ? dpv * a.inv_keep : 0.f;
            }
            P[hh][kt][r] = pd;
            dS[hh][kt][r] = p * (dpv - sdv[ql]);
          }
        }
      }
      v8bf pf[KT], sf[KT];
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        pf[kt] = pack_slots(P[0][kt], P[1][kt]);
        sf[kt] = pack_slots(dS[0][kt], dS[1][kt]);
        if constexpr (DS) {
          // dS^T for the dQ GEMM (attn_dq_ds_kernel): the lane's key row, queries 32 kq + 4 G .. + 3 and + 16
          const int key = k0w + 16 * kt + i;
          if (key < a.Sk) {
            const uint4 u = __builtin_bit_cast(uint4, sf[kt]);
            // (query-tile-major: the 64 queries of tile q0 / 64 for every key are one contiguous 128-B row)
            bf16_t* row = a.ds + (((long)bh * (a.dsld >> 6) + (q0 >> 6)) * a.Sk + key) * 64 + 32 * kq + 4 * G;
            *reinterpret_cast<uint2*>(row) = make_uint2(u.x, u.y);
            *reinterpret_cast<uint2*>(row + 16) = make_uint2(u.z, u.w);
          }
        }
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const v8bf dof = frag_tr(sdo, 32 * kq, 16 * dt, lane);
        const v8bf qtf = frag_tr(sq, 32 * kq, 16 * dt, lane);
#pragma unroll
        for (int kt = 0; kt < KT; ++kt) {
          dv[dt][kt] = mfma(dof, pf[kt], dv[dt][kt]);
          dk[dt][kt] = mfma(qtf, sf[kt], dk[dt][kt]);
        }
      }
    }
  }
  bf16_t* dK = a.dk + kb;
  bf16_t* dV = a.dv + kb;
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
    const int key = k0w + 16 * kt + i;
    if (key < a.Sk) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        store4(dK + (long)key * a.kss + 16 * dt + 4 * G, dk[dt][kt], a.scale);
        store4(dV + (long)key * a.kss + 16 * dt + 4 * G, dv[dt][kt], drop ? a.inv_keep : 1.f);
      }
    }
  }
}

// key block kblk walks the query tiles from its diagonal on (causal): heavy = small kblk
template <int KT, bool DS>
__global__ void __launch_bounds__(256, 2) attn_bwd_dkdv_kernel(AttnArgs a, int nblk) {
  __shared__ __attribute__((aligned(16))) char sq[64 * 128];
  __shared__ __attribute__((aligned(16))) char sdo[64 * 128];
  __shared__ float slse[64], sdv[64];
  for (int pass = 0; pass < 2; ++pass) {
    int blk = pair_block(a.causal, nblk, pass);
    if (blk < 0) break;
    blk = nblk - 1 - blk;  // (pair_block orders by descending index; here the heavy blocks are the low ones)
    if (pass) __syncthreads();
    attn_dkdv_body<KT, DS>(a, blk, sq, sdo, slse, sdv);
  }
}

// dQ: block = 4 waves x (16 QT) queries, loop over 64-key tiles; grid (cdiv(Sq, 64 QT), B*H)
template <int QT>
__device__ __forceinline__ void attn_dq_body(const AttnArgs& a, const int qblk, char* sk, char* sv, float* smask) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, G = lane >> 4, i = lane & 15;
  const int bh = attn_by(), b = bh / a.H, h = bh % a.H;
  const int BM = 64 * QT;
  const int q0 = qblk * BM + w * 16 * QT;
  const long hb = b * a.qsb + h * a.qsh, kb = b * a.ksb + h * a.ksh, ob = b * a.osb + h * a.osh;
  const bf16_t* Q = a.q + hb;
  const bf16_t* K = a.k + kb;
  const bf16_t* V = a.v + kb;
  const bf16_t* dO = a.dout + ob;
  const int off = a.Sk - a.Sq;
  const float c = a.scale * LOG2E;
  const bool drop = a.thr < 65536u;
  const uint32_t salt = drop_salt(a, bh);

  v8bf qf[QT][2], df[QT][2];
  float lse[QT], dd[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    const int qi = q0 + 16 * qt + i;
    const bool ok = qi < a.Sq;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      qf[qt][kk] = frag_global(Q + (long)qi * a.qss + 32 * kk + 8 * G, ok);
      df[qt][kk] = frag_global(dO + (long)qi * a.oss + 32 * kk + 8 * G, ok);
    }
    lse[qt] = ok ? a.lse[(long)bh * a.Sq + qi] : INFINITY;
    // D[q] = rowsum(dO * O): the lane's 16 dims, then the 4 lane groups of the row
    float d = 0.f;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const v8bf of = frag_global(a.o + ob + (long)qi * a.oss + 32 * kk + 8 * G, ok);
#pragma unroll
      for (int j = 0; j < 8; ++j) d = fmaf((float)df[qt][kk][j], (float)of[j], d);
    }
    d += __shfl_xor(d, 16, 64);
    d += __shfl_xor(d, 32, 64);
    dd[qt] = d;
    if (ok && G == 0) a.dvec[(long)bh * a.Sq + qi] = d;  // for the dK/dV kernel, launched after this one
  }
  v4f dq[4][QT];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) dq[dt][qt] = v4f{0.f, 0.f, 0.f, 0.f};
  int kend = a.Sk;
  if (a.causal) kend = min(a.Sk, qblk * BM + BM + off);
  const int ntiles = (kend + 63) / 64;
  TileRegs tk, tv;
  float mreg = 0.f;
  if (ntiles > 0) {
    tile_load(tk, K, a.kss, 0, a.Sk);
    tile_load(tv, V, a.kss, 0, a.Sk);
    if (threadIdx.x < 64) mreg = key_bias(a, b, threadIdx.x);
  }
  for (int t = 0; t < ntiles; ++t) {
    __syncthreads();
    tile_store(tk, sk);
    tile_store(tv, sv);
    if (threadIdx.x < 64) smask[threadIdx.x] = mreg;
    __syncthreads();
    const int k0 = t * 64;
    if (t + 1 < ntiles) {
      tile_load(tk, K, a.kss, k0 + 64, a.Sk);
      tile_load(tv, V, a.kss, k0 + 64, a.Sk);
      if (threadIdx.x < 64) mreg = key_bias(a, b, k0 + 64 + threadIdx.x);
    }
    const bool diag = a.causal && (k0 + 63 > q0 + off);
    v4f dS[4][QT];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      const v8bf k0f = frag_row(sk, 16 * kt, 0, lane), k1f = frag_row(sk, 16 * kt, 1, lane);
      const v8bf v0f = frag_row(sv, 16 * kt, 0, lane), v1f = frag_row(sv, 16 * kt, 1, lane);
      float km[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) km[r] = smask[16 * kt + 4 * G + r];
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        v4f s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
        s = mfma(k0f, qf[qt][0], s);
        s = mfma(k1f, qf[qt][1], s);
        dp = mfma(v0f, df[qt][0], dp);
        dp = mfma(v1f, df[qt][1], dp);
        const int qi = q0 + 16 * qt + i;
        uint2 bits = make_uint2(0, 0);
        if (drop) bits = drop_bits(a, salt, qi, (k0 >> 2) + 4 * kt + G);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float x = fmaf(s[r], c, km[r]);
          if (diag && k0 + 16 * kt + 4 * G + r > qi + off) x = -INFINITY;
          const float p = ex2(x - lse[qt]);
          float dpv = dp[r];
          if (drop) {
            const bool kp = r == 0 ? keep_j<0>(bits, a.thr) : r == 1 ? keep_j<1>(bits, a.thr)
                            : r == 2 ? keep_j<2>(bits, a.thr) : keep_j<3>(bits, a.thr);
            dpv = kp ? dpv * a.inv_keep : 0.f;
          }
          dS[kt][qt][r] = p * (dpv - dd[qt]);
        }
      }
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      v8bf sf[QT];
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) sf[qt] = pack_slots(dS[2 * kk][qt], dS[2 * kk + 1][qt]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const v8bf ktf = frag_tr(sk, 32 * kk, 16 * dt, lane);
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) dq[dt][qt] = mfma(ktf, sf[qt], dq[dt][qt]);
      }
    }
  }
  bf16_t* dQ = a.dq + hb;
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    const int qi = q0 + 16 * qt + i;
    if (qi < a.Sq) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) store4(dQ + (long)qi * a.qss + 16 * dt + 4 * G, dq[dt][qt], a.scale);
    }
  }
}

// MINW: register budget (waves per SIMD). 2 (<= 256 VGPRs) measured faster on the non-causal BERT shape
// (bwd 287 -> 247 us with dropout), 1 on the causal GPT-2 shape (208 vs 230 us).
template <int QT, int MINW>
__global__ void __launch_bounds__(256, MINW) attn_bwd_dq_kernel(AttnArgs a, int nblk) {
  __shared__ __attribute__((aligned(16))) char sk[64 * 128];
  __shared__ __attribute__((aligned(16))) char sv[64 * 128];
  __shared__ float smask[64];
  for (int pass = 0; pass < 2; ++pass) {
    const int blk = pair_block(a.causal, nblk, pass);
    if (blk < 0) break;
    if (pass) __syncthreads();
    attn_dq_body<QT>(a, blk, sk, sv, smask);
  }
}

// dQ = scale * dS K from the dS^T scratch the dK/dV kernel wrote (a memory-bound GEMM: no score recompute, no
// exponentials, no dropout hashes). Block: 4 waves x 16 queries of one query tile over 64-key tiles; the tile's dS^T
// strip is contiguous (64 keys x 128 B per K-tile). LDS-DMA staged through a 3-stage ring (two tiles in flight under
// the MFMAs, counted vmcnt waits: register-staged loads made the compiler drain the queue every tile), one barrier
// per tile; causal: only the key tiles up to the diagonal (exactly the tiles the dK/dV kernel wrote).
__global__ void __launch_bounds__(256) attn_dq_ds_kernel(AttnArgs a, int nqt) {
  constexpr int NS = 3, TB = 64 * 128;  // ring stages; bytes of one [64][64] bf16 tile
  __shared__ __attribute__((aligned(16))) char smem[NS * 2 * TB];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, G = lane >> 4, i = lane & 15;
  const int bh = attn_by(), b = bh / a.H, h = bh % a.H;
  const int qt = nqt - 1 - attn_bx();  // heavy (late) query tiles first under causal masking
  const int q0 = qt * 64;
  const int off = a.Sk - a.Sq;
  int kend = a.Sk;
  if (a.causal) kend = min(a.Sk, q0 + 64 + off);
  const int ntiles = kend > 0 ? (kend + 63) / 64 : 0;
  const bf16_t* D = a.ds + ((long)bh * (a.dsld >> 6) + qt) * a.Sk * 64;
  const bf16_t* K = a.k + b * a.ksb + h * a.ksh;
  // LDS-DMA: a wave instruction fills 1 KiB = 8 rows of a tile lane-linearly; each lane fetches the logical 16-B
  // chunk that the swz() XOR swizzle puts at its physical slot; rows past Sk read zeros (range check)
  const __amdgpu_buffer_rsrc_t rd =
      __builtin_amdgcn_make_buffer_rsrc((void*)D, (short)0, (int)((long)a.Sk * 128), 0x00020000);
  const __amdgpu_buffer_rsrc_t rk =
      __builtin_amdgcn_make_buffer_rsrc((void*)K, (short)0, (int)(((long)(a.Sk - 1) * a.kss + 64) * 2), 0x00020000);
  int rrow[2], lch[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int row = 32 * u + 8 * w + (lane >> 3);  // physical byte offset (4 u + w) KiB + 16 lane
    rrow[u] = row;
    lch[u] = (lane & 7) ^ ((row >> 1) & 7);
  }
  auto issue = [&](int t, int slot) {
    char* sd = smem + slot * 2 * TB;
    char* sk = sd + TB;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int key = t * 64 + rrow[u];
      const bool ok = key < a.Sk;
      const uint32_t od = ok ? (uint32_t)((key * 64 + lch[u] * 8) * 2) : 0x80000000u;
      const uint32_t okk = ok ? (uint32_t)(((long)key * a.kss + lch[u] * 8) * 2) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rd, (__attribute__((address_space(3))) void*)(sd + u * 4096 + w * 1024),
                                               16, od, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (__attribute__((address_space(3))) void*)(sk + u * 4096 + w * 1024),
                                               16, okk, 0, 0, 0);
    }
  };
  v4f acc[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) acc[dt] = v4f{0.f, 0.f, 0.f, 0.f};
  // every step issues exactly one tile (4 DMA instructions per thread, past the end: zeros), so vmcnt(4) after the
  // issue of tile t + 1 means tile t has landed
  issue(0, 0);
  issue(1, 1);
  int slot = 0;
  for (int t = 0; t < ntiles; ++t) {
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    __syncthreads();  // tile t landed for every wave; every wave is done with the slot of tile t - 1
    issue(t + 2, slot == 0 ? 2 : slot - 1);
    const char* cd = smem + slot * 2 * TB;
    const char* ck = cd + TB;
    v8bf sf[2], kf[2][4];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      sf[kk] = frag_tr(cd, 32 * kk, 16 * w, lane);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) kf[kk][dt] = frag_tr(ck, 32 * kk, 16 * dt, lane);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) acc[dt] = mfma(kf[kk][dt], sf[kk], acc[dt]);
    slot = slot == 2 ? 0 : slot + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA into LDS outstanding when the block retires
  const int qi = q0 + 16 * w + i;
  if (qi < a.Sq) {
    bf16_t* dQ = a.dq + b * a.qsb + h * a.qsh + (long)qi * a.qss;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) store4(dQ + 16 * dt + 4 * G, acc[dt], a.scale);
  }
}

AttnArgs make_args(const void* q, const void* k, const void* v, const long* qstr, const long* kstr, const void* o,
                   const void* dout, const long* ostr, int B, int H, int Sq, int Sk, float scale, float dropout,
                   unsigned long long seed, int causal, const float* kmask,
                   const unsigned long long* seedctr) {
  AttnArgs a{};
  a.q = (const bf16_t*)q;
  a.k = (const bf16_t*)k;
  a.v = (const bf16_t*)v;
  a.o = (bf16_t*)o;
  a.dout = (const bf16_t*)dout;
  a.qsb = qstr[0];
  a.qss = qstr[1];
  a.qsh = qstr[2];
  a.ksb = kstr[0];
  a.kss = kstr[1];
  a.ksh = kstr[2];
  a.osb = ostr[0];
  a.oss = ostr[1];
  a.osh = ostr[2];
  a.B = B;
  a.H = H;
  a.Sq = Sq;
  a.Sk = Sk;
  a.scale = scale;
  long thr = lrintf((1.f - dropout) * 65536.f);
  thr = thr < 1 ? 1 : (thr > 65536 ? 65536 : thr);
  a.thr = (uint32_t)thr;
  a.inv_keep = 65536.f / (float)thr;
  a.seed = (uint32_t)(seed ^ (seed >> 32));
  a.seedctr = dropout > 0.f ? seedctr : nullptr;
  a.nkq = (Sk + 3) / 4;
  a.causal = causal;
  a.kmask = kmask;
  return a;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }



}  // namespace

// q/k/v: bf16 with strides {batch, seq, head} (elements; head dim 64 contiguous): qstr for q (and dq), kstr for
// k/v (and dk/dv), ostr for o / dout. lse: f32 [B*H][Sq]. kmask: optional f32 [B][Sk] additive (0 keep, large
// negative drop). dropout: probability of zeroing an attention weight (training).
DTF_API int dtf_attn_fwd(const void* q, const void* k, const void* v, const long* qstr, const long* kstr, void* o,
                         const long* ostr, float* lse, const float* kmask, int B, int H, int Sq, int Sk, int D,
                         float scale, float dropout, unsigned long long seed, int causal, const void* seedctr,
                         void* stream) {
  if (D != HD || !aligned16(q) || !aligned16(k) || !aligned16(v) || !aligned16(o)) return -1;
  if ((qstr[0] | qstr[1] | qstr[2] | kstr[0] | kstr[1] | kstr[2] | ostr[0] | ostr[1] | ostr[2]) & 7) return -1;
  if (dropout < 0.f || dropout >= 1.f) return -1;
  AttnArgs a = make_args(q, k, v, qstr, kstr, o, nullptr, ostr, B, H, Sq, Sk, scale, dropout, seed, causal, kmask,
                         (const unsigned long long*)seedctr);
  a.lse = lse;
  const int nqb = (Sq + 127) / 128;
  dim3 grid(pair_grid(causal, nqb), (unsigned)(B * H));
  if (a.thr < 65536u) hipLaunchKernelGGL((attn_fwd_kernel<2, true>), grid, dim3(256), 0, (hipStream_t)stream, a, nqb);
  else hipLaunchKernelGGL((attn_fwd_kernel<2, false>), grid, dim3(256), 0, (hipStream_t)stream, a, nqb);
  return (int)hipGetLastError();
}

// dvec: f32 [B*H][Sq] scratch (rowsum(dO * O), written by the dQ kernel, read by the dK/dV kernel).
DTF_API int dtf_attn_bwd(const void* q, const void* k, const void* v, const long* qstr, const long* kstr,
                         const void* o, const void* dout, const long* ostr, const float* lse, float* dvec, void* dq,
                         void* dk, void* dv, const float* kmask, int B, int H, int Sq, int Sk, int D, float scale,
                         float dropout, unsigned long long seed, int causal, const void* seedctr, void* stream) {
  if (D != HD || !aligned16(q) || !aligned16(k) || !aligned16(v) || !aligned16(o) || !aligned16(dout) ||
      !aligned16(dq) || !aligned16(dk) || !aligned16(dv))
    return -1;
  if ((qstr[0] | qstr[1] | qstr[2] | kstr[0] | kstr[1] | kstr[2] | ostr[0] | ostr[1] | ostr[2]) & 7) return -1;
  if (dropout < 0.f || dropout >= 1.f) return -1;
  hipStream_t st = (hipStream_t)stream;
  AttnArgs a = make_args(q, k, v, qstr, kstr, o, dout, ostr, B, H, Sq, Sk, scale, dropout, seed, causal, kmask,
                         (const unsigned long long*)seedctr);
  a.lse = const_cast<float*>(lse);
  a.dvec = dvec;
  a.dq = (bf16_t*)dq;
  a.dk = (bf16_t*)dk;
  a.dv = (bf16_t*)dv;
  const int nkb = (Sk + 127) / 128, nqb = (Sq + 127) / 128;
  // dQ first: it forms D = rowsum(dO * O) per query (dvec) that the dK/dV kernel reads
  if (causal)
    hipLaunchKernelGGL((attn_bwd_dq_kernel<2, 1>), dim3(pair_grid(causal, nqb), (unsigned)(B * H)), dim3(256), 0, st,
                       a, nqb);
  else
    hipLaunchKernelGGL((attn_bwd_dq_kernel<2, 2>), dim3(pair_grid(causal, nqb), (unsigned)(B * H)), dim3(256), 0, st,
                       a, nqb);
  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<2, false>), dim3(pair_grid(causal, nkb), (unsigned)(B * H)), dim3(256), 0,
                     st, a, nkb);
  return (int)hipGetLastError();
}

// dtf_attn_bwd through a dS^T scratch (ds: bf16, >= B*H*round_up(Sq, 64)*Sk elements): D = rowsum(dO * O) by a
// small pass, the dK/dV kernel also stores dS^T (the values its dK MFMAs use), and dQ = scale * dS K is a
// memory-bound GEMM over the stored tiles instead of a second kernel that recomputes the scores, the
// probabilities and dP (3 of the 5 backward MFMA products). Same results as dtf_attn_bwd up to the f32 order of
// the dQ sums.
DTF_API int dtf_attn_bwd_ds(const void* q, const void* k, const void* v, const long* qstr, const long* kstr,
                            const void* o, const void* dout, const long* ostr, const float* lse, float* dvec, void* dq,
                            void* dk, void* dv, const float* kmask, int B, int H, int Sq, int Sk, int D, float scale,
                            float dropout, unsigned long long seed, int causal, const void* seedctr, void* ds,
                            void* stream) {
  if (D != HD || !aligned16(q) || !aligned16(k) || !aligned16(v) || !aligned16(o) || !aligned16(dout) ||
      !aligned16(dq) || !aligned16(dk) || !aligned16(dv) || !aligned16(ds))
    return -1;
  if ((qstr[0] | qstr[1] | qstr[2] | kstr[0] | kstr[1] | kstr[2] | ostr[0] | ostr[1] | ostr[2]) & 7) return -1;
  if (dropout < 0.f || dropout >= 1.f) return -1;
  hipStream_t st = (hipStream_t)stream;
  AttnArgs a = make_args(q, k, v, qstr, kstr, o, dout, ostr, B, H, Sq, Sk, scale, dropout, seed, causal, kmask,
                         (const unsigned long long*)seedctr);
  a.lse = const_cast<float*>(lse);
  a.dvec = dvec;
  a.dq = (bf16_t*)dq;
  a.dk = (bf16_t*)dk;
  a.dv = (bf16_t*)dv;
  a.ds = (bf16_t*)ds;
  a.dsld = (Sq + 63) / 64 * 64;
  if ((long)B * H * Sq >= (1l << 31)) return -1;
  const long blocks = ((long)B * H * Sq + 31) / 32;  // 32 rows per block
  hipLaunchKernelGGL(attn_dvec_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256), 0, st, a);
  const int nkb = (Sk + 127) / 128, nqt = (Sq + 63) / 64;
  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<2, true>), dim3(pair_grid(causal, nkb), (unsigned)(B * H)), dim3(256), 0,
                     st, a, nkb);
  hipLaunchKernelGGL(attn_dq_ds_kernel, dim3((unsigned)nqt, (unsigned)(B * H)), dim3(256), 0, st, a, nqt);
  return (int)hipGetLastError();
}
