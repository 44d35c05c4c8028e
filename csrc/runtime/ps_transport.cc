// Parameter-server data plane: variable pull / gradient push between worker and PS processes.
//
// The reference's between-graph PS training moves every parameter PS->worker and every gradient
// worker->PS on each step through TF's gRPC Send/Recv rendezvous (reference
// trainer/task.py:236). Here:
//   * the PS process registers host mirrors of its variable shards (PULL is served straight from
//     them by the connection threads — no Python on the pull path; a per-variable reader/writer
//     lock keeps a pull from seeing a half-written update);
//   * a PUSH lands in a per-connection buffer and is queued; the PS's training loop pops it
//     (dtfrt_ps_next_push), applies the fused optimizer kernel to the HBM-resident shard, refreshes
//     the mirror, and acks (dtfrt_ps_push_done) — asynchronous (Hogwild) semantics like the
//     reference's use_locking=False apply ops, but every update is applied whole.
// Frames: request [u8 op][u32 var][u64 off][u64 n][payload]; reply [i32 status][u64 version].
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

#include "net.h"
#include "runtime.h"

using namespace dtfrt;

namespace {

enum : uint8_t { PULL = 1, PUSH = 2, META = 3, BYE = 4 };

struct Var {
  char* host = nullptr;
  uint64_t nbytes = 0;
  std::shared_mutex lock;
  std::atomic<uint64_t> version{0};
};

struct Push {
  int token;
  int var;
  uint64_t off, n;
  std::vector<char> data;
  int worker_fd;
  bool done = false;
  std::mutex mu;
  std::condition_variable cv;
  int status = 0;
};

struct Server {
  int lfd = -1, port = 0;
  std::atomic<bool> stop{false};
  std::thread acceptor;
  std::mutex mu;
  std::map<int, std::unique_ptr<Var>> vars;
  std::vector<std::thread> conns;
  std::vector<int> fds;
  std::mutex qmu;
  std::condition_variable qcv;
  std::deque<std::shared_ptr<Push>> queue;
  std::map<int, std::shared_ptr<Push>> inflight;
  int next_token = 1;
  std::atomic<uint64_t> pulls{0}, pushes{0};
};

Var* find_var(Server* s, int id) {
  std::lock_guard<std::mutex> g(s->mu);
  auto it = s->vars.find(id);
  return it == s->vars.end() ? nullptr : it->second.get();
}

bool send_reply(int fd, int32_t st, uint64_t ver) {
  char b[12];
  memcpy(b, &st, 4);
  memcpy(b + 4, &ver, 8);
  return send_all(fd, b, 12);
}

void serve(Server* s, int fd) {
  for (;;) {
    char hdr[21];
    if (!recv_all(fd, hdr, 21)) break;
    uint8_t op = (uint8_t)hdr[0];
    uint32_t vid;
    uint64_t off, n;
    memcpy(&vid, hdr + 1, 4);
    memcpy(&off, hdr + 5, 8);
    memcpy(&n, hdr + 13, 8);
    if (op == BYE) break;
    Var* v = find_var(s, (int)vid);
    if (op == META) {
      send_reply(fd, v ? 0 : -1, v ? v->nbytes : 0);
      continue;
    }
    if (op == PULL) {
      if (!v || off + n > v->nbytes) {
        send_reply(fd, -1, 0);
        continue;
      }
      std::shared_lock<std::shared_mutex> g(v->lock);
      uint64_t ver = v->version.load();
      if (!send_reply(fd, 0, ver) || !send_all(fd, v->host + off, n)) break;
      s->pulls++;
      continue;
    }
    if (op == PUSH) {
      auto p = std::make_shared<Push>();
      p->var = (int)vid;
      p->off = off;
      p->n = n;
      p->data.resize(n);
      if (n && !recv_all(fd, p->data.data(), n)) break;
      if (!v || off + n > v->nbytes) {
        send_reply(fd, -1, 0);
        continue;
      }
      {
        std::lock_guard<std::mutex> g(s->qmu);
        p->token = s->next_token++;
        s->queue.push_back(p);
        s->inflight[p->token] = p;
      }
      s->qcv.notify_one();
      std::unique_lock<std::mutex> g(p->mu);
      p->cv.wait(g, [&] { return p->done || s->stop.load(); });
      s->pushes++;
      if (!send_reply(fd, p->status, v->version.load())) break;
      continue;
    }
    send_reply(fd, -2, 0);
  }
  ::close(fd);
}

struct Client {
  int fd = -1;
  std::mutex mu;
};

}  // namespace

DTF_RT void* dtfrt_ps_server_start(const char* host, int port, int* bound) {
  int fd = listen_on(host, port);
  if (fd < 0) {
    set_error("ps: cannot listen on %s:%d (%s)", host ? host : "", port, strerror(errno));
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
      s->conns.emplace_back(serve, s, c);
    }
  });
  return s;
}

// Register (or re-register) a variable's host mirror.
DTF_RT int dtfrt_ps_register(void* h, int var_id, void* host, uint64_t nbytes) {
  auto* s = (Server*)h;
  std::lock_guard<std::mutex> g(s->mu);
  auto& v = s->vars[var_id];
  if (!v) v.reset(new Var);
  v->host = (char*)host;
  v->nbytes = nbytes;
  return 0;
}

// Writer side of the mirror lock: hold it while refreshing a mirror after an update.
DTF_RT int dtfrt_ps_lock(void* h, int var_id) {
  Var* v = find_var((Server*)h, var_id);
  if (!v) return -1;
  v->lock.lock();
  return 0;
}
DTF_RT int dtfrt_ps_unlock(void* h, int var_id, int bump_version) {
  Var* v = find_var((Server*)h, var_id);
  if (!v) return -1;
  if (bump_version) v->version++;
  v->lock.unlock();
  return 0;
}

// Pop the next queued gradient push (wait up to timeout_ms). Returns token > 0, 0 on timeout.
DTF_RT int dtfrt_ps_next_push(void* h, int timeout_ms, int* var_id, uint64_t* off, uint64_t* n, void** data) {
  auto* s = (Server*)h;
  std::unique_lock<std::mutex> g(s->qmu);
  if (!s->qcv.wait_for(g, std::chrono::milliseconds(timeout_ms), [&] { return !s->queue.empty() || s->stop; }))
    return 0;
  if (s->queue.empty()) return 0;
  auto p = s->queue.front();
  s->queue.pop_front();
  *var_id = p->var;
  *off = p->off;
  *n = p->n;
  *data = p->data.data();
  return p->token;
}

DTF_RT int dtfrt_ps_push_done(void* h, int token, int status) {
  auto* s = (Server*)h;
  std::shared_ptr<Push> p;
  {
    std::lock_guard<std::mutex> g(s->qmu);
    auto it = s->inflight.find(token);
    if (it == s->inflight.end()) return -1;
    p = it->second;
    s->inflight.erase(it);
  }
  {
    std::lock_guard<std::mutex> g(p->mu);
    p->done = true;
    p->status = status;
  }
  p->cv.notify_all();
  return 0;
}

DTF_RT void dtfrt_ps_stats(void* h, uint64_t* pulls, uint64_t* pushes) {
  auto* s = (Server*)h;
  *pulls = s->pulls;
  *pushes = s->pushes;
}

DTF_RT void dtfrt_ps_server_stop(void* h) {
  auto* s = (Server*)h;
  s->stop = true;
  s->qcv.notify_all();
  {
    std::lock_guard<std::mutex> g(s->qmu);
    for (auto& kv : s->inflight) {
      std::lock_guard<std::mutex> pg(kv.second->mu);
      kv.second->done = true;
      kv.second->status = -3;
      kv.second->cv.notify_all();
    }
  }
  ::shutdown(s->lfd, SHUT_RDWR);
  ::close(s->lfd);
  if (s->acceptor.joinable()) s->acceptor.join();
  {
    std::lock_guard<std::mutex> g(s->mu);
    for (int fd : s->fds) ::shutdown(fd, SHUT_RDWR);
  }
  for (auto& t : s->conns)
    if (t.joinable()) t.join();
  delete s;
}

DTF_RT void* dtfrt_ps_connect(const char* host, int port, int timeout_ms) {
  int fd = connect_to(host, port, timeout_ms);
  if (fd < 0) {
    set_error("ps: cannot connect to %s:%d", host, port);
    return nullptr;
  }
  auto* c = new Client;
  c->fd = fd;
  return c;
}

static int ps_req(Client* c, uint8_t op, int var, uint64_t off, uint64_t n, const void* payload, void* dst,
                  uint64_t* version) {
  std::lock_guard<std::mutex> g(c->mu);
  char hdr[21];
  hdr[0] = (char)op;
  uint32_t v = (uint32_t)var;
  memcpy(hdr + 1, &v, 4);
  memcpy(hdr + 5, &off, 8);
  memcpy(hdr + 13, &n, 8);
  if (!send_all(c->fd, hdr, 21)) return -100;
  if (op == PUSH && n && !send_all(c->fd, payload, n)) return -100;
  char rep[12];
  if (!recv_all(c->fd, rep, 12)) return -101;
  int32_t st;
  memcpy(&st, rep, 4);
  if (version) memcpy(version, rep + 4, 8);
  if (st == 0 && op == PULL && n && !recv_all(c->fd, dst, n)) return -101;
  return st;
}

DTF_RT int dtfrt_ps_pull(void* h, int var, uint64_t off, void* dst, uint64_t n, uint64_t* version) {
  int st = ps_req((Client*)h, PULL, var, off, n, nullptr, dst, version);
  if (st) set_error("ps pull var %d failed (%d)", var, st);
  return st;
}

DTF_RT int dtfrt_ps_push(void* h, int var, uint64_t off, const void* src, uint64_t n, uint64_t* version) {
  int st = ps_req((Client*)h, PUSH, var, off, n, src, nullptr, version);
  if (st) set_error("ps push var %d failed (%d)", var, st);
  return st;
}

DTF_RT int64_t dtfrt_ps_var_bytes(void* h, int var) {
  uint64_t n = 0;
  int st = ps_req((Client*)h, META, var, 0, 0, nullptr, nullptr, &n);
  return st ? -1 : (int64_t)n;
}

DTF_RT void dtfrt_ps_close(void* h) {
  auto* c = (Client*)h;
  char hdr[21] = {0};
  hdr[0] = (char)BYE;
  send_all(c->fd, hdr, 21);
  ::close(c->fd);
  delete c;
}
