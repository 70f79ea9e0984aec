// TCP bootstrap of a multi-node RCCL communicator: the node of rank 0 creates the ncclUniqueId and
// serves it to the other nodes, which connect to DSTACK_MASTER_NODE_IP (the same rendezvous the
// job's torchrun uses, one port above MASTER_PORT).  Header-only and RCCL-free, so the exchange is
// unit-tested on the CPU with a stub 128-byte id (native/tests/native_tests.cpp).
#pragma once
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <string>
#include <thread>

namespace dsa {

inline bool bs_send_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL);
    if (w <= 0) return false;
    c += w;
    n -= (size_t)w;
  }
  return true;
}

inline bool bs_recv_all(int fd, void* p, size_t n, int timeout_ms) {
  char* c = static_cast<char*>(p);
  while (n) {
    struct pollfd pf{fd, POLLIN, 0};
    if (::poll(&pf, 1, timeout_ms) <= 0) return false;
    ssize_t r = ::recv(fd, c, n, 0);
    if (r <= 0) return false;
    c += r;
    n -= (size_t)r;
  }
  return true;
}

// Node 0: listen on `port` and hand `id` (id_len bytes) to `peers` connecting nodes; each peer
// first sends its node rank (4 bytes) so a duplicate or out-of-range rank is refused.
// Returns "" on success, else an error.
inline std::string bootstrap_serve(int port, const void* id, size_t id_len, int peers, int timeout_ms,
                                   int* bound_port = nullptr) {
  int lfd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (lfd < 0) return "socket failed";
  int one = 1;
  setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  struct sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  a.sin_addr.s_addr = htonl(INADDR_ANY);
  if (::bind(lfd, (struct sockaddr*)&a, sizeof a) != 0 || ::listen(lfd, 64) != 0) {
    ::close(lfd);
    return "bind/listen on port " + std::to_string(port) + " failed";
  }
  if (bound_port) {
    socklen_t len = sizeof a;
    getsockname(lfd, (struct sockaddr*)&a, &len);
    *bound_port = ntohs(a.sin_port);
  }
  std::string err;
  std::string seen((size_t)peers + 1, '\0');
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  for (int served = 0; served < peers && err.empty();) {
    const int left = (int)std::chrono::duration_cast<std::chrono::milliseconds>(
                         deadline - std::chrono::steady_clock::now()).count();
    struct pollfd pf{lfd, POLLIN, 0};
    if (left <= 0 || ::poll(&pf, 1, left) <= 0) {
      err = "timed out waiting for " + std::to_string(peers - served) + " node(s)";
      break;
    }
    int c = ::accept(lfd, nullptr, nullptr);
    if (c < 0) continue;
    int32_t r = -1;
    if (bs_recv_all(c, &r, 4, 5000) && r >= 1 && r <= peers && !seen[(size_t)r]) {
      uint32_t n = (uint32_t)id_len;
      if (bs_send_all(c, &n, 4) && bs_send_all(c, id, id_len)) {
        seen[(size_t)r] = 1;
        ++served;
      }
    }
    ::close(c);
  }
  ::close(lfd);
  return err;
}

// Node r > 0: connect to host:port (retrying until timeout: node 0 may start later) and read the id.
inline std::string bootstrap_fetch(const std::string& host, int port, int node_rank, void* id, size_t id_len,
                                   int timeout_ms) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  while (std::chrono::steady_clock::now() < deadline) {
    struct addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) == 0 && res) {
      int fd = ::socket(res->ai_family, res->ai_socktype, 0);
      if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
        freeaddrinfo(res);
        int32_t r = node_rank;
        uint32_t n = 0;
        bool ok = bs_send_all(fd, &r, 4) && bs_recv_all(fd, &n, 4, 10000) && n == id_len &&
                  bs_recv_all(fd, id, id_len, 10000);
        ::close(fd);
        return ok ? "" : "bad bootstrap reply";
      }
      if (fd >= 0) ::close(fd);
      freeaddrinfo(res);
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
  }
  return "could not reach the master node " + host + ":" + std::to_string(port);
}

}  // namespace dsa
