// Host-side native runtime of distributed_tensorflow_amd (C ABI, loaded with ctypes).
//
// Replaces the TF C++ runtime pieces the reference relies on:
//   T10 Saver / tensor-bundle checkpoints  -> tensor_bundle.cc
//   T12 EventsWriter / TFRecord framing    -> event_writer.cc
//   T3/T13 gRPC server, FIFOQueue done-signal, Supervisor readiness -> kv_store.cc
//   T4 Send/Recv of parameters and gradients for PS training -> ps_transport.cc
#pragma once
#include <stddef.h>
#include <stdint.h>

#define DTF_RT extern "C" __attribute__((visibility("default")))

namespace dtfrt {
uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n);
inline uint32_t crc32c(const void* data, size_t n) { return crc32c_extend(0, data, n); }
// TF / LevelDB masked CRC: rotate right by 15 and add a constant.
inline uint32_t crc_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }
inline uint32_t crc_unmask(uint32_t m) {
  uint32_t rot = m - 0xa282ead8u;
  return ((rot >> 17) | (rot << 15));
}
void set_error(const char* fmt, ...);
}  // namespace dtfrt

DTF_RT const char* dtfrt_last_error();
