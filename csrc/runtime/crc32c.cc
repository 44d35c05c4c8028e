// CRC32C (Castagnoli) for checkpoint / TFRecord integrity: SSE4.2 crc32 instruction when the
// host has it, slicing-by-8 tables otherwise.
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>

#include "runtime.h"

#if defined(__x86_64__)
#include <cpuid.h>
#include <nmmintrin.h>
#endif

namespace dtfrt {

static uint32_t table[8][256];
static bool have_sse42 = false;

static void init_tables() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82f63b78u : (c >> 1);
    table[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i)
    for (int t = 1; t < 8; ++t) table[t][i] = (table[t - 1][i] >> 8) ^ table[0][table[t - 1][i] & 0xff];
#if defined(__x86_64__)
  unsigned a, b, c, d;
  if (__get_cpuid(1, &a, &b, &c, &d)) have_sse42 = (c & bit_SSE4_2) != 0;
#endif
}

static std::once_flag once;

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) static uint32_t crc_hw(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t c = crc;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return c32;
}
#endif

uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n) {
  std::call_once(once, init_tables);
  const uint8_t* p = (const uint8_t*)data;
  uint32_t c = ~crc;
#if defined(__x86_64__)
  if (have_sse42) return ~crc_hw(c, p, n);
#endif
  while (n >= 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= c;
    c = table[7][lo & 0xff] ^ table[6][(lo >> 8) & 0xff] ^ table[5][(lo >> 16) & 0xff] ^ table[4][lo >> 24] ^
        table[3][hi & 0xff] ^ table[2][(hi >> 8) & 0xff] ^ table[1][(hi >> 16) & 0xff] ^ table[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = (c >> 8) ^ table[0][(c ^ *p++) & 0xff];
  return ~c;
}

static thread_local std::string last_err;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  last_err = buf;
}

}  // namespace dtfrt

DTF_RT const char* dtfrt_last_error() { return dtfrt::last_err.c_str(); }

DTF_RT uint32_t dtfrt_crc32c(const void* data, size_t n, uint32_t init) { return dtfrt::crc32c_extend(init, data, n); }
DTF_RT uint32_t dtfrt_crc_mask(uint32_t c) { return dtfrt::crc_mask(c); }
