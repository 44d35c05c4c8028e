// Native self-test of the host runtime, built with sanitizers by tools/sanitize_runtime.sh
// (AddressSanitizer + UndefinedBehaviorSanitizer, and ThreadSanitizer for the threaded services).
// SURVEY §5 "Race detection / sanitizers": exercises every C entry point the Python layer uses, with
// concurrent clients on the KV store and the PS transport and multi-process-free shm reduction.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "runtime.h"

DTF_RT uint32_t dtfrt_crc32c(const void* data, size_t n, uint32_t init);
DTF_RT void* dtfrt_bundle_writer_open(const char* prefix, int num_shards);
DTF_RT int dtfrt_bundle_add(void* h, const char* name, int dtype, int ndims, const int64_t* dims, const void* data,
                            int64_t nbytes, int shard);
DTF_RT int dtfrt_bundle_finish(void* h);
DTF_RT void* dtfrt_bundle_reader_open(const char* prefix);
DTF_RT int dtfrt_bundle_num_tensors(void* h);
DTF_RT int dtfrt_bundle_info(void* h, const char* name, int* dtype, int* ndims, int64_t* dims, int64_t* nbytes);
DTF_RT int dtfrt_bundle_read(void* h, const char* name, void* dst, int64_t nbytes);
DTF_RT void dtfrt_bundle_reader_close(void* h);
DTF_RT void* dtfrt_events_open(const char* path);
DTF_RT int dtfrt_events_scalar(void* h, const char* tag, float value, int64_t step, double wall);
DTF_RT void dtfrt_tfrecord_writer_close(void* h);
DTF_RT void* dtfrt_tfrecord_reader_open(const char* path);
DTF_RT int dtfrt_tfrecord_next(void* h, const char** data, uint64_t* n);
DTF_RT void dtfrt_tfrecord_reader_close(void* h);
DTF_RT void* dtfrt_kv_server_start(const char* host, int port, int* bound);
DTF_RT void dtfrt_kv_server_stop(void* h);
DTF_RT void* dtfrt_kv_connect(const char* host, int port, int timeout_ms);
DTF_RT void dtfrt_kv_close(void* h);
DTF_RT int dtfrt_kv_set(void* h, const char* key, const void* val, uint64_t n);
DTF_RT int dtfrt_kv_get(void* h, const char* key, int64_t timeout_ms, uint64_t* n);
DTF_RT const char* dtfrt_kv_result(void* h);
DTF_RT int64_t dtfrt_kv_add(void* h, const char* key, int64_t delta);
DTF_RT int dtfrt_kv_wait_ge(void* h, const char* key, int64_t target, int64_t timeout_ms, int64_t* cur);
DTF_RT void* dtfrt_ps_server_start(const char* host, int port, int* bound);
DTF_RT int dtfrt_ps_register(void* h, int var_id, void* host, uint64_t nbytes);
DTF_RT int dtfrt_ps_lock(void* h, int var_id);
DTF_RT int dtfrt_ps_unlock(void* h, int var_id, int bump_version);
DTF_RT int dtfrt_ps_next_push(void* h, int timeout_ms, int* var_id, uint64_t* off, uint64_t* n, void** data);
DTF_RT int dtfrt_ps_push_done(void* h, int token, int status);
DTF_RT void dtfrt_ps_server_stop(void* h);
DTF_RT void* dtfrt_ps_connect(const char* host, int port, int timeout_ms);
DTF_RT int dtfrt_ps_pull(void* h, int var, uint64_t off, void* dst, uint64_t n, uint64_t* version);
DTF_RT int dtfrt_ps_push(void* h, int var, uint64_t off, const void* src, uint64_t n, uint64_t* version);
DTF_RT void dtfrt_ps_close(void* h);
DTF_RT void* dtfrt_shm_open(const char* name, int rank, int world, uint64_t max_bytes);
DTF_RT int dtfrt_shm_allreduce_f32(void* hp, void* data, uint64_t n);
DTF_RT void dtfrt_shm_close(void* hp, int unlink_it);

static int failures = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      fprintf(stderr, "CHECK failed %s:%d: %s (%s)\n", __FILE__, __LINE__, #c, dtfrt_last_error()); \
      ++failures;                                                       \
    }                                                                   \
  } while (0)

static void test_crc() {
  CHECK(dtfrt_crc32c("123456789", 9, 0) == 0xE3069283u);
  std::vector<char> big(1 << 20);
  for (size_t i = 0; i < big.size(); ++i) big[i] = (char)(i * 131);
  uint32_t whole = dtfrt_crc32c(big.data(), big.size(), 0);
  uint32_t part = dtfrt_crc32c(big.data() + 7, big.size() - 7, dtfrt_crc32c(big.data(), 7, 0));
  CHECK(whole == part);
}

static void test_bundle(const std::string& dir) {
  std::string prefix = dir + "/ckpt";
  void* w = dtfrt_bundle_writer_open(prefix.c_str(), 2);
  CHECK(w != nullptr);
  std::vector<float> a(1000), b(7);
  for (int i = 0; i < 1000; ++i) a[i] = i * 0.5f;
  for (int i = 0; i < 7; ++i) b[i] = -i;
  int64_t da[2] = {10, 100}, db[1] = {7};
  CHECK(dtfrt_bundle_add(w, "layer/kernel", 1, 2, da, a.data(), (int64_t)a.size() * 4, 0) == 0);
  CHECK(dtfrt_bundle_add(w, "layer/bias", 1, 1, db, b.data(), (int64_t)b.size() * 4, 1) == 0);
  CHECK(dtfrt_bundle_finish(w) == 0);
  void* r = dtfrt_bundle_reader_open(prefix.c_str());
  CHECK(r != nullptr);
  if (!r) return;
  CHECK(dtfrt_bundle_num_tensors(r) == 2);
  int dt = 0, nd = 0;
  int64_t dims[8], nb = 0;
  CHECK(dtfrt_bundle_info(r, "layer/kernel", &dt, &nd, dims, &nb) == 0 && nd == 2 && dims[1] == 100 && nb == 4000);
  std::vector<float> back(1000);
  CHECK(dtfrt_bundle_read(r, "layer/kernel", back.data(), 4000) == 0 && back[999] == 499.5f);
  CHECK(dtfrt_bundle_read(r, "missing", back.data(), 4) != 0);
  dtfrt_bundle_reader_close(r);
}

static void test_events(const std::string& dir) {
  std::string path = dir + "/events.out.tfevents.selftest";
  void* h = dtfrt_events_open(path.c_str());
  CHECK(h != nullptr);
  for (int i = 0; i < 50; ++i) CHECK(dtfrt_events_scalar(h, "loss", 1.f / (i + 1), i, 1000.0 + i) == 0);
  dtfrt_tfrecord_writer_close(h);
  void* rd = dtfrt_tfrecord_reader_open(path.c_str());
  CHECK(rd != nullptr);
  if (!rd) return;
  const char* data;
  uint64_t n;
  int count = 0;
  while (dtfrt_tfrecord_next(rd, &data, &n) > 0) ++count;  // 1 = record, 0 = EOF, < 0 = corrupt
  CHECK(count == 51);  // file_version event + 50 scalars
  dtfrt_tfrecord_reader_close(rd);
}

static void test_kv() {
  int port = 0;
  void* srv = dtfrt_kv_server_start("127.0.0.1", 0, &port);
  CHECK(srv != nullptr);
  if (!srv) return;
  const int T = 8, N = 200;
  std::vector<std::thread> th;
  std::atomic<int> ok{0};
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      void* c = dtfrt_kv_connect("127.0.0.1", port, 5000);
      if (!c) return;
      for (int i = 0; i < N; ++i) dtfrt_kv_add(c, "ctr", 1);
      std::string k = "key" + std::to_string(t);
      dtfrt_kv_set(c, k.c_str(), k.data(), k.size());
      int64_t cur = 0;
      if (dtfrt_kv_wait_ge(c, "ctr", (int64_t)T * N, 10000, &cur) == 0) ok++;
      dtfrt_kv_close(c);
    });
  for (auto& x : th) x.join();
  CHECK(ok.load() == T);
  void* c = dtfrt_kv_connect("127.0.0.1", port, 5000);
  CHECK(dtfrt_kv_add(c, "ctr", 0) == (int64_t)T * N);
  uint64_t n = 0;
  CHECK(dtfrt_kv_get(c, "key3", 1000, &n) == 0 && n == 4 && memcmp(dtfrt_kv_result(c), "key3", 4) == 0);
  CHECK(dtfrt_kv_get(c, "nokey", 50, &n) == 1);  // timeout
  dtfrt_kv_close(c);
  dtfrt_kv_server_stop(srv);
}

static void test_ps() {
  int port = 0;
  void* srv = dtfrt_ps_server_start("127.0.0.1", 0, &port);
  CHECK(srv != nullptr);
  if (!srv) return;
  std::vector<float> mirror(4096, 1.f);
  CHECK(dtfrt_ps_register(srv, 0, mirror.data(), mirror.size() * 4) == 0);
  std::atomic<bool> stop{false};
  std::atomic<int> applied{0};
  std::thread server([&] {  // the PS apply loop
    while (!stop.load()) {
      int var;
      uint64_t off, n;
      void* data;
      int tok = dtfrt_ps_next_push(srv, 20, &var, &off, &n, &data);
      if (tok == 0) continue;
      dtfrt_ps_lock(srv, 0);
      const float* g = (const float*)data;
      for (uint64_t i = 0; i < n / 4; ++i) mirror[i] -= 0.001f * g[i];
      dtfrt_ps_unlock(srv, 0, 1);
      applied++;
      dtfrt_ps_push_done(srv, tok, 0);
    }
  });
  const int W = 4, STEPS = 25;
  std::vector<std::thread> ws;
  for (int w = 0; w < W; ++w)
    ws.emplace_back([&] {
      void* c = dtfrt_ps_connect("127.0.0.1", port, 5000);
      if (!c) return;
      std::vector<float> p(4096), g(4096, 1.f);
      uint64_t ver;
      for (int s = 0; s < STEPS; ++s) {
        dtfrt_ps_pull(c, 0, 0, p.data(), p.size() * 4, &ver);
        dtfrt_ps_push(c, 0, 0, g.data(), g.size() * 4, &ver);
      }
      dtfrt_ps_close(c);
    });
  for (auto& x : ws) x.join();
  stop = true;
  server.join();
  CHECK(applied.load() == W * STEPS);
  CHECK(mirror[17] < 1.f - 0.001f * W * STEPS + 1e-3f && mirror[17] > 1.f - 0.001f * W * STEPS - 1e-3f);
  dtfrt_ps_server_stop(srv);
}

static void test_shm() {
  // world 3 in threads of one process (the same code path the CPU Mirrored replicas use across processes)
  const int W = 3;
  const uint64_t N = 10000;
  std::string name = "selftest_" + std::to_string(getpid());
  std::vector<std::vector<float>> bufs(W, std::vector<float>(N));
  void* h0 = dtfrt_shm_open(name.c_str(), 0, W, N * 4);  // rank 0 creates the segment first
  CHECK(h0 != nullptr);
  if (!h0) return;
  std::vector<void*> hs(W, nullptr);
  hs[0] = h0;
  for (int r = 1; r < W; ++r) hs[r] = dtfrt_shm_open(name.c_str(), r, W, N * 4);
  std::vector<std::thread> th;
  for (int r = 0; r < W; ++r)
    th.emplace_back([&, r] {
      for (uint64_t i = 0; i < N; ++i) bufs[r][i] = (float)(r + 1) * (float)(i % 7);
      dtfrt_shm_allreduce_f32(hs[r], bufs[r].data(), N);
    });
  for (auto& x : th) x.join();
  for (int r = 0; r < W; ++r) CHECK(bufs[r][13] == 6.f * (13 % 7));
  for (int r = W - 1; r >= 0; --r) dtfrt_shm_close(hs[r], r == 0);
}

int main(int argc, char** argv) {
  std::string dir = argc > 1 ? argv[1] : "/tmp";
  test_crc();
  test_bundle(dir);
  test_events(dir);
  test_kv();
  test_ps();
  test_shm();
  if (failures) {
    fprintf(stderr, "selftest: %d failures\n", failures);
    return 1;
  }
  printf("selftest ok\n");
  return 0;
}
