// The dropout mask of the elementwise dropout kernels (elementwise.hip) and of the LayerNorm backward that applies a
// following dropout's backward in its store pass (norm.hip): one definition, so both regenerate the same bits.
#pragma once
#include <cmath>

#include "common.h"

namespace {

__device__ __forceinline__ uint64_t step_seed(uint64_t seed, const uint64_t* ctr) {
  return ctr ? seed ^ (*ctr * 0xD1B54A32D192ED03ull) : seed;
}

// Dropout mask of an 8-element chunk: two 64-bit counter hashes give eight 16-bit uniforms; element j is kept
// when its uniform is below thr = round(keep * 65536), and kept values are scaled by 65536 / thr (the exact
// inverse of the realised keep probability). 4x fewer hashes than one per element.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint32_t keep_bits8(uint64_t seed, long chunk, uint32_t thr) {
  const uint64_t h0 = mix64(seed + 0x9E3779B97F4A7C15ull * (uint64_t)(2 * chunk + 1));
  const uint64_t h1 = mix64(seed + 0x9E3779B97F4A7C15ull * (uint64_t)(2 * chunk + 2));
  uint32_t bits = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    bits |= (uint32_t)(((h0 >> (16 * j)) & 0xFFFFu) < thr) << j;
    bits |= (uint32_t)(((h1 >> (16 * j)) & 0xFFFFu) < thr) << (4 + j);
  }
  return bits;
}

}  // namespace

static inline uint32_t keep_threshold(float keep) {  // 16-bit keep threshold of the dropout kernels (>= 1)
  long t = lrintf(keep * 65536.f);
  return (uint32_t)(t < 1 ? 1 : (t > 65536 ? 65536 : t));
}
