// Minimal blocking TCP helpers shared by the KV store and the PS transport.
#pragma once
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <string>
#include <thread>

namespace dtfrt {

inline bool send_all(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n) {
    ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    c += k;
    n -= (size_t)k;
  }
  return true;
}

inline bool recv_all(int fd, void* p, size_t n) {
  char* c = (char*)p;
  while (n) {
    ssize_t k = ::recv(fd, c, n, 0);
    if (k == 0) return false;
    if (k < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    c += k;
    n -= (size_t)k;
  }
  return true;
}

inline void tune(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  int buf = 8 << 20;
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof buf);
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof buf);
}

inline int listen_on(const char* host, int port) {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) return -1;
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  a.sin_addr.s_addr = (host && *host && strcmp(host, "0.0.0.0") != 0) ? inet_addr(host) : INADDR_ANY;
  if (a.sin_addr.s_addr == INADDR_NONE) a.sin_addr.s_addr = INADDR_ANY;
  if (::bind(fd, (sockaddr*)&a, sizeof a) < 0 || ::listen(fd, 128) < 0) {
    ::close(fd);
    return -1;
  }
  return fd;
}

inline int bound_port(int fd) {
  sockaddr_in a{};
  socklen_t l = sizeof a;
  getsockname(fd, (sockaddr*)&a, &l);
  return ntohs(a.sin_port);
}

// Connect with retries until timeout_ms (servers of a cluster start in any order).
inline int connect_to(const char* host, int port, int timeout_ms) {
  auto t0 = std::chrono::steady_clock::now();
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  std::string ps = std::to_string(port);
  for (;;) {
    if (getaddrinfo(host, ps.c_str(), &hints, &res) == 0 && res) {
      int fd = ::socket(AF_INET, SOCK_STREAM, 0);
      if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
        freeaddrinfo(res);
        tune(fd);
        return fd;
      }
      if (fd >= 0) ::close(fd);
      freeaddrinfo(res);
      res = nullptr;
    }
    auto el = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
    if (el >= timeout_ms) return -1;
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
}

}  // namespace dtfrt
