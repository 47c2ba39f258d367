// Small POSIX TCP helpers shared by the native store and the host backend.
#pragma once

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

namespace tds_comm {

inline void put_u32(std::string& s, uint32_t v) { s.append(reinterpret_cast<const char*>(&v), 4); }

inline void send_all(int fd, const void* buf, size_t n) {
  const char* p = static_cast<const char*>(buf);
  while (n > 0) {
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(std::string("tds net: send failed: ") + std::strerror(errno));
    }
    p += w;
    n -= (size_t)w;
  }
}

enum class RecvStatus { kOk, kTimeout, kClosed };

// kTimeout: the socket's receive timeout (SO_RCVTIMEO) expired with the peer still connected;
// kClosed: EOF, reset or any other error -- the connection is gone.
inline RecvStatus recv_all_status(int fd, void* buf, size_t n) {
  char* p = static_cast<char*>(buf);
  while (n > 0) {
    ssize_t r = ::recv(fd, p, n, 0);
    if (r == 0) return RecvStatus::kClosed;
    if (r < 0) {
      if (errno == EINTR) continue;
      return (errno == EAGAIN || errno == EWOULDBLOCK) ? RecvStatus::kTimeout : RecvStatus::kClosed;
    }
    p += r;
    n -= (size_t)r;
  }
  return RecvStatus::kOk;
}

// false on EOF / timeout / error
inline bool recv_all_nothrow(int fd, void* buf, size_t n) { return recv_all_status(fd, buf, n) == RecvStatus::kOk; }

inline void recv_all(int fd, void* buf, size_t n) {
  if (!recv_all_nothrow(fd, buf, n)) throw std::runtime_error("tds net: connection closed or timed out");
}

inline std::string recv_str(int fd) {
  uint32_t n = 0;
  recv_all(fd, &n, 4);
  std::string s(n, '\0');
  if (n) recv_all(fd, &s[0], n);
  return s;
}

inline void set_rcv_timeout(int fd, int64_t ms) {
  timeval tv;
  tv.tv_sec = ms / 1000;
  tv.tv_usec = (ms % 1000) * 1000;
  ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
}

inline int listen_on(int port, int* actual_port, const char* bind_addr = nullptr) {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) throw std::runtime_error("tds net: socket() failed");
  int one = 1;
  ::setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  a.sin_addr.s_addr = bind_addr ? inet_addr(bind_addr) : htonl(INADDR_ANY);
  if (::bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) {
    ::close(fd);
    throw std::runtime_error("tds net: bind to port " + std::to_string(port) + " failed: " + std::strerror(errno));
  }
  if (::listen(fd, 1024) != 0) {
    ::close(fd);
    throw std::runtime_error("tds net: listen failed");
  }
  socklen_t len = sizeof(a);
  ::getsockname(fd, reinterpret_cast<sockaddr*>(&a), &len);
  if (actual_port) *actual_port = ntohs(a.sin_port);
  return fd;
}

// Connect with retries until timeout_ms (the server may not be up yet).
inline int connect_to(const std::string& host, int port, int64_t timeout_ms) {
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  std::string last;
  while (true) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (::getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) == 0 && res) {
      int fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
      if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
        ::freeaddrinfo(res);
        int one = 1;
        ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        return fd;
      }
      last = std::strerror(errno);
      if (fd >= 0) ::close(fd);
      ::freeaddrinfo(res);
    } else {
      last = "getaddrinfo failed for " + host;
    }
    if (std::chrono::steady_clock::now() > deadline)
      throw std::runtime_error("tds net: could not connect to " + host + ":" + std::to_string(port) + " (" + last +
                               ")");
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

}  // namespace tds_comm
