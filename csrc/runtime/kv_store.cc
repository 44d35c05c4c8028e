// Cluster control plane: a TCP key-value store with blocking reads, atomic counters and
// wait-for-count, hosted by one task of a TF_CONFIG cluster (the chief or PS 0).
//
// It replaces the TF runtime services the reference leans on for coordination
// (SURVEY §2.2 T3/T11/T13):
//   * cluster bootstrap / readiness (Supervisor's wait-for-chief, reference trainer/task.py:215-226)
//     -> SET "ready" by the chief, GET (blocking) by the others;
//   * the auto-stop-PS FIFOQueue done-signal (reference auto_stop_ps/task.py:127-150,270-272)
//     -> ADD "done" + WAITGE "done" >= num_trainers (exactly one counter, no queue race);
//   * RCCL unique-id exchange, barriers, global_step counters and heartbeats.
// Protocol: request  [u8 op][u32 klen][key][u64 vlen][val]
//           response [i32 status][u64 len][bytes]
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "net.h"
#include "runtime.h"

using namespace dtfrt;

namespace {

enum Op : uint8_t { SET = 1, GET = 2, ADD = 3, CHECK = 4, DEL = 5, WAITGE = 6, PING = 7, KEYS = 8 };

struct Server {
  int lfd = -1;
  int port = 0;
  std::atomic<bool> stop{false};
  std::thread acceptor;
  std::mutex mu;
  std::condition_variable cv;
  std::map<std::string, std::string> kv;
  std::vector<std::thread> workers;
  std::vector<int> fds;
};

int64_t as_int(const std::string& s) {
  int64_t v = 0;
  if (s.size() == 8) memcpy(&v, s.data(), 8);
  return v;
}
std::string from_int(int64_t v) { return std::string((const char*)&v, 8); }

bool reply(int fd, int32_t st, const std::string& b) {
  uint64_t n = b.size();
  char hdr[12];
  memcpy(hdr, &st, 4);
  memcpy(hdr + 4, &n, 8);
  return send_all(fd, hdr, 12) && (n == 0 || send_all(fd, b.data(), n));
}

void serve(Server* s, int fd) {
  for (;;) {
    uint8_t op;
    uint32_t kl;
    uint64_t vl;
    if (!recv_all(fd, &op, 1) || !recv_all(fd, &kl, 4)) break;
    std::string key(kl, '\0');
    if (kl && !recv_all(fd, &key[0], kl)) break;
    if (!recv_all(fd, &vl, 8)) break;
    std::string val(vl, '\0');
    if (vl && !recv_all(fd, &val[0], vl)) break;
    bool ok = true;
    switch (op) {
      case SET: {
        {
          std::lock_guard<std::mutex> g(s->mu);
          s->kv[key] = val;
        }
        s->cv.notify_all();
        ok = reply(fd, 0, "");
        break;
      }
      case GET: {  // val: i64 timeout ms (<0: forever)
        int64_t to = as_int(val);
        std::unique_lock<std::mutex> g(s->mu);
        auto pred = [&] { return s->kv.count(key) > 0 || s->stop; };
        bool found = to < 0 ? (s->cv.wait(g, pred), s->kv.count(key) > 0)
                            : s->cv.wait_for(g, std::chrono::milliseconds(to), pred) && s->kv.count(key) > 0;
        std::string v = found ? s->kv[key] : "";
        g.unlock();
        ok = reply(fd, found ? 0 : 1, v);
        break;
      }
      case ADD: {
        int64_t nv;
        {
          std::lock_guard<std::mutex> g(s->mu);
          nv = as_int(s->kv[key]) + as_int(val);
          s->kv[key] = from_int(nv);
        }
        s->cv.notify_all();
        ok = reply(fd, 0, from_int(nv));
        break;
      }
      case CHECK: {
        std::lock_guard<std::mutex> g(s->mu);
        ok = reply(fd, s->kv.count(key) ? 0 : 1, "");
        break;
      }
      case DEL: {
        {
          std::lock_guard<std::mutex> g(s->mu);
          s->kv.erase(key);
        }
        ok = reply(fd, 0, "");
        break;
      }
      case WAITGE: {  // val: [i64 target][i64 timeout ms]
        int64_t target = 0, to = -1;
        if (val.size() >= 16) {
          memcpy(&target, val.data(), 8);
          memcpy(&to, val.data() + 8, 8);
        }
        std::unique_lock<std::mutex> g(s->mu);
        auto pred = [&] { return as_int(s->kv[key]) >= target || s->stop; };
        bool r = to < 0 ? (s->cv.wait(g, pred), true) : s->cv.wait_for(g, std::chrono::milliseconds(to), pred);
        int64_t cur = as_int(s->kv[key]);
        g.unlock();
        ok = reply(fd, (r && cur >= target) ? 0 : 1, from_int(cur));
        break;
      }
      case PING:
        ok = reply(fd, 0, "pong");
        break;
      case KEYS: {  // keys with prefix `key`, '\n'-separated
        std::string out;
        {
          std::lock_guard<std::mutex> g(s->mu);
          for (auto it = s->kv.lower_bound(key); it != s->kv.end() && it->first.compare(0, key.size(), key) == 0;
               ++it)
            out += it->first + "\n";
        }
        ok = reply(fd, 0, out);
        break;
      }
      default:
        ok = reply(fd, -1, "bad op");
    }
    if (!ok) break;
  }
  ::close(fd);
}

struct Client {
  int fd = -1;
  std::mutex mu;
  std::string last;
};

int request(Client* c, uint8_t op, const char* key, size_t kl, const void* val, uint64_t vl, std::string& out) {
  std::lock_guard<std::mutex> g(c->mu);
  uint32_t k = (uint32_t)kl;
  if (!send_all(c->fd, &op, 1) || !send_all(c->fd, &k, 4) || (kl && !send_all(c->fd, key, kl)) ||
      !send_all(c->fd, &vl, 8) || (vl && !send_all(c->fd, val, vl))) {
    set_error("kv: send failed");
    return -100;
  }
  char hdr[12];
  if (!recv_all(c->fd, hdr, 12)) {
    set_error("kv: connection lost");
    return -101;
  }
  int32_t st;
  uint64_t n;
  memcpy(&st, hdr, 4);
  memcpy(&n, hdr + 4, 8);
  out.resize(n);
  if (n && !recv_all(c->fd, &out[0], n)) {
    set_error("kv: connection lost");
    return -101;
  }
  return st;
}

}  // namespace

// Start a KV server on host:port (port 0 = ephemeral). Returns a handle; *bound receives the port.
DTF_RT void* dtfrt_kv_server_start(const char* host, int port, int* bound) {
  int fd = listen_on(host, port);
  if (fd < 0) {
    set_error("kv: cannot listen on %s:%d (%s)", host ? host : "", port, strerror(errno));
    return nullptr;
  }
  auto* s = new Server;
  s->lfd = fd;
  s->port = bound_port(fd);
  if (bound) *bound = s->port;
  s->acceptor = std::thread([s] {
    while (!s->stop) {
      int c = ::accept(s->lfd, nullptr, nullptr);
      if (c < 0) {
        if (s->stop) break;
        continue;
      }
      tune(c);
      std::lock_guard<std::mutex> g(s->mu);
      s->fds.push_back(c);
      s->workers.emplace_back(serve, s, c);
    }
  });
  return s;
}

DTF_RT void dtfrt_kv_server_stop(void* h) {
  auto* s = (Server*)h;
  s->stop = true;
  s->cv.notify_all();
  ::shutdown(s->lfd, SHUT_RDWR);
  ::close(s->lfd);
  if (s->acceptor.joinable()) s->acceptor.join();
  {
    std::lock_guard<std::mutex> g(s->mu);
    for (int fd : s->fds) ::shutdown(fd, SHUT_RDWR);
  }
  for (auto& t : s->workers)
    if (t.joinable()) t.join();
  delete s;
}

DTF_RT void* dtfrt_kv_connect(const char* host, int port, int timeout_ms) {
  int fd = connect_to(host, port, timeout_ms);
  if (fd < 0) {
    set_error("kv: cannot connect to %s:%d", host, port);
    return nullptr;
  }
  auto* c = new Client;
  c->fd = fd;
  return c;
}

DTF_RT void dtfrt_kv_close(void* h) {
  auto* c = (Client*)h;
  ::close(c->fd);
  delete c;
}

DTF_RT int dtfrt_kv_set(void* h, const char* key, const void* val, uint64_t n) {
  std::string out;
  return request((Client*)h, SET, key, strlen(key), val, n, out);
}

// Blocking get; returns 0 and fills the client's buffer (read with dtfrt_kv_result), 1 on timeout.
DTF_RT int dtfrt_kv_get(void* h, const char* key, int64_t timeout_ms, uint64_t* n) {
  auto* c = (Client*)h;
  int st = request(c, GET, key, strlen(key), &timeout_ms, 8, c->last);
  *n = c->last.size();
  return st;
}

DTF_RT const char* dtfrt_kv_result(void* h) { return ((Client*)h)->last.data(); }

DTF_RT int64_t dtfrt_kv_add(void* h, const char* key, int64_t delta) {
  std::string out;
  int st = request((Client*)h, ADD, key, strlen(key), &delta, 8, out);
  if (st != 0) return INT64_MIN;
  return as_int(out);
}

DTF_RT int dtfrt_kv_check(void* h, const char* key) {
  std::string out;
  return request((Client*)h, CHECK, key, strlen(key), nullptr, 0, out);
}

DTF_RT int dtfrt_kv_del(void* h, const char* key) {
  std::string out;
  return request((Client*)h, DEL, key, strlen(key), nullptr, 0, out);
}

// Block until the counter at `key` >= target (0), or timeout (1). *cur receives the counter.
DTF_RT int dtfrt_kv_wait_ge(void* h, const char* key, int64_t target, int64_t timeout_ms, int64_t* cur) {
  int64_t v[2] = {target, timeout_ms};
  std::string out;
  int st = request((Client*)h, WAITGE, key, strlen(key), v, 16, out);
  if (cur) *cur = as_int(out);
  return st;
}

DTF_RT int dtfrt_kv_keys(void* h, const char* prefix, uint64_t* n) {
  auto* c = (Client*)h;
  int st = request(c, KEYS, prefix, strlen(prefix), nullptr, 0, c->last);
  *n = c->last.size();
  return st;
}
