// Native TCP key-value store for rendezvous.
//
// Replaces the role c10d::TCPStore plays behind `init_process_group(init_method=
// "env://")` in the reference (allreduce_toy.py:44, mnist_distributed.py:50):
// rank 0 hosts a server thread, every rank connects as a client; the device
// (RCCL) and host backends exchange their communicator ids / peer addresses
// through it.  A Python `torch.distributed.Store` subclass
// (parallel/store.py) wraps this class so torch's own process groups can
// rendezvous through it too.
//
// Wire format (little endian):
//   request : u8 op | u32 klen | key | u32 vlen | value [| u32 v2len | value2]
//   response: u8 status (0 ok, 1 missing/false, 2 error) | u32 vlen | value
// GET and WAIT block on the server until the key exists; clients bound every
// call by their timeout (SO_RCVTIMEO) so a dead peer cannot hang a rank.
#include <ATen/ATen.h>
#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <torch/custom_class.h>
#include <torch/library.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "comm/net.h"

namespace tds_comm {

enum Op : uint8_t { SET = 1, GET = 2, ADD = 3, CHECK = 4, WAIT = 5, DEL = 6, NUMKEYS = 7, CAS = 8, PING = 9 };

// ------------------------------------------------------------------ server
class StoreServer {
 public:
  explicit StoreServer(int port) {
    listen_fd_ = listen_on(port, &port_);
    stop_pipe_[0] = stop_pipe_[1] = -1;
    if (::pipe(stop_pipe_) != 0) throw std::runtime_error("tds store: pipe failed");
    thread_ = std::thread([this] { loop(); });
  }
  ~StoreServer() {
    char c = 1;
    if (stop_pipe_[1] >= 0) (void)!::write(stop_pipe_[1], &c, 1);
    if (thread_.joinable()) thread_.join();
    for (auto& kv : clients_) ::close(kv.first);
    ::close(listen_fd_);
    ::close(stop_pipe_[0]);
    ::close(stop_pipe_[1]);
  }
  int port() const { return port_; }

 private:
  struct Waiter {
    int fd;
    uint8_t op;
  };
  int listen_fd_ = -1, port_ = 0;
  int stop_pipe_[2];
  std::thread thread_;
  std::unordered_map<int, bool> clients_;
  std::map<std::string, std::string> data_;
  std::map<std::string, std::vector<Waiter>> waiters_;

  static void reply(int fd, uint8_t status, const std::string& v) {
    std::string msg;
    msg.push_back((char)status);
    put_u32(msg, (uint32_t)v.size());
    msg += v;
    send_all(fd, msg.data(), msg.size());
  }

  void wake(const std::string& key) {
    auto it = waiters_.find(key);
    if (it == waiters_.end()) return;
    for (auto& w : it->second) {
      try {
        reply(w.fd, 0, w.op == GET ? data_[key] : std::string());
      } catch (...) {
      }
    }
    waiters_.erase(it);
  }

  bool handle(int fd) {
    uint8_t op;
    if (!recv_all_nothrow(fd, &op, 1)) return false;
    std::string key = recv_str(fd);
    std::string val = recv_str(fd);
    switch (op) {
      case SET:
        data_[key] = val;
        reply(fd, 0, "");
        wake(key);
        break;
      case GET:
      case WAIT: {
        auto it = data_.find(key);
        if (it != data_.end()) reply(fd, 0, op == GET ? it->second : std::string());
        else waiters_[key].push_back({fd, op});
        break;
      }
      case ADD: {
        int64_t delta = 0;
        std::memcpy(&delta, val.data(), std::min<size_t>(8, val.size()));
        int64_t cur = 0;
        auto it = data_.find(key);
        if (it != data_.end()) cur = std::stoll(it->second);
        cur += delta;
        data_[key] = std::to_string(cur);
        std::string out(8, '\0');
        std::memcpy(&out[0], &cur, 8);
        reply(fd, 0, out);
        wake(key);
        break;
      }
      case CHECK:
        reply(fd, data_.count(key) ? 0 : 1, "");
        break;
      case DEL:
        reply(fd, data_.erase(key) ? 0 : 1, "");
        break;
      case NUMKEYS: {
        int64_t n = (int64_t)data_.size();
        std::string out(8, '\0');
        std::memcpy(&out[0], &n, 8);
        reply(fd, 0, out);
        break;
      }
      case CAS: {
        std::string desired = recv_str(fd);
        auto it = data_.find(key);
        if (it == data_.end()) {
          if (val.empty()) {
            data_[key] = desired;
            reply(fd, 0, desired);
            wake(key);
          } else {
            reply(fd, 0, val);
          }
        } else if (it->second == val) {
          it->second = desired;
          reply(fd, 0, desired);
          wake(key);
        } else {
          reply(fd, 0, it->second);
        }
        break;
      }
      case PING:
        reply(fd, 0, "pong");
        break;
      default:
        reply(fd, 2, "bad op");
    }
    return true;
  }

  void drop(int fd) {
    for (auto it = waiters_.begin(); it != waiters_.end();) {
      auto& v = it->second;
      v.erase(std::remove_if(v.begin(), v.end(), [fd](const Waiter& w) { return w.fd == fd; }), v.end());
      it = v.empty() ? waiters_.erase(it) : std::next(it);
    }
    clients_.erase(fd);
    ::close(fd);
  }

  void loop() {
    while (true) {
      std::vector<pollfd> fds;
      fds.push_back({stop_pipe_[0], POLLIN, 0});
      fds.push_back({listen_fd_, POLLIN, 0});
      for (auto& kv : clients_) fds.push_back({kv.first, POLLIN, 0});
      int r = ::poll(fds.data(), fds.size(), 1000);
      if (r < 0) {
        if (errno == EINTR) continue;
        break;
      }
      if (fds[0].revents) break;
      if (fds[1].revents & POLLIN) {
        int c = ::accept(listen_fd_, nullptr, nullptr);
        if (c >= 0) {
          int one = 1;
          ::setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
          clients_[c] = true;
        }
      }
      for (size_t i = 2; i < fds.size(); ++i) {
        if (!fds[i].revents) continue;
        bool ok = false;
        if (fds[i].revents & POLLIN) {
          try {
            ok = handle(fds[i].fd);
          } catch (...) {
            ok = false;
          }
        }
        if (!ok) drop(fds[i].fd);
      }
    }
  }
};

// ------------------------------------------------------------------ client (torch custom class)
class TCPStore : public torch::CustomClassHolder {
 public:
  TCPStore(std::string host, int64_t port, int64_t world_size, bool is_server, int64_t timeout_ms)
      : host_(std::move(host)), world_(world_size), timeout_ms_(timeout_ms) {
    if (is_server) {
      server_ = std::make_unique<StoreServer>((int)port);
      port_ = server_->port();
    } else {
      port_ = (int)port;
    }
    fd_ = connect_to(host_, port_, timeout_ms_);
    set_rcv_timeout(fd_, timeout_ms_);
  }
  ~TCPStore() override {
    if (fd_ >= 0) ::close(fd_);
  }

  void set(const std::string& key, const at::Tensor& value) { call(SET, key, bytes_of(value)); }
  at::Tensor get(const std::string& key) { return to_tensor(call(GET, key, "")); }
  int64_t add(const std::string& key, int64_t delta) {
    std::string v(8, '\0');
    std::memcpy(&v[0], &delta, 8);
    std::string r = call(ADD, key, v);
    int64_t out = 0;
    std::memcpy(&out, r.data(), 8);
    return out;
  }
  bool check(const std::string& key) { return call_status(CHECK, key, "") == 0; }
  void wait(const std::string& key, int64_t timeout_ms) {
    std::lock_guard<std::mutex> g(mu_);
    request(WAIT, key, "", nullptr, timeout_ms > 0 ? timeout_ms : timeout_ms_);
    response(nullptr);  // (a timed-out WAIT replaces the connection there, once)
  }
  bool delete_key(const std::string& key) { return call_status(DEL, key, "") == 0; }
  int64_t num_keys() {
    std::string r = call(NUMKEYS, "", "");
    int64_t n = 0;
    std::memcpy(&n, r.data(), 8);
    return n;
  }
  at::Tensor compare_set(const std::string& key, const at::Tensor& expected, const at::Tensor& desired) {
    std::lock_guard<std::mutex> g(mu_);
    std::string d = bytes_of(desired);
    request(CAS, key, bytes_of(expected), &d);
    std::string out;
    response(&out);
    return to_tensor(out);
  }
  int64_t port() const { return port_; }
  int64_t world_size() const { return world_; }
  void set_timeout(int64_t ms) {
    timeout_ms_ = ms;
    set_rcv_timeout(fd_, ms);
  }

 private:
  std::string host_;
  int port_ = 0;
  int64_t world_, timeout_ms_;
  int fd_ = -1;
  std::mutex mu_;
  std::unique_ptr<StoreServer> server_;

  static std::string bytes_of(const at::Tensor& t) {
    auto c = t.contiguous().to(at::kCPU);
    return std::string(reinterpret_cast<const char*>(c.data_ptr()), c.numel() * c.element_size());
  }
  static at::Tensor to_tensor(const std::string& s) {
    auto t = at::empty({(int64_t)s.size()}, at::TensorOptions().dtype(at::kByte));
    if (!s.empty()) std::memcpy(t.data_ptr(), s.data(), s.size());
    return t;
  }
  // One request on the connection.  ``rcv_ms`` bounds the wait for its reply (a WAIT passes its
  // own timeout); every other request uses the store timeout.
  void request(uint8_t op, const std::string& key, const std::string& val, const std::string* val2,
               int64_t rcv_ms = -1) {
    if (fd_ < 0) {
      // the connection was dropped after a desync or a lost peer: one immediate attempt, so a
      // store whose server is gone fails at once instead of retrying for the whole timeout
      fd_ = try_connect_once();
      if (fd_ < 0) throw std::runtime_error("tds TCPStore: connection to the store at " + host_ + ":" +
                                            std::to_string(port_) + " lost (server gone?)");
    }
    set_rcv_timeout(fd_, rcv_ms > 0 ? rcv_ms : timeout_ms_);
    std::string msg;
    msg.push_back((char)op);
    put_u32(msg, (uint32_t)key.size());
    msg += key;
    put_u32(msg, (uint32_t)val.size());
    msg += val;
    if (val2) {
      put_u32(msg, (uint32_t)val2->size());
      msg += *val2;
    }
    try {
      send_all(fd_, msg.data(), msg.size());
    } catch (...) {
      drop_connection();
      throw;
    }
  }
  int try_connect_once() {
    try {
      int fd = connect_to(host_, port_, 0);  // a single attempt (no retry loop)
      set_rcv_timeout(fd, timeout_ms_);
      return fd;
    } catch (...) {
      return -1;
    }
  }
  void drop_connection() {
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
  }
  // The reply to the request just sent.  Two ways to fail, handled differently:
  //  * the receive timeout expired with the server still there: a blocked GET / WAIT stays
  //    registered and is answered when its key appears -- on this connection that late reply
  //    would be read as the answer to the NEXT request.  So the connection is replaced (one
  //    immediate connect attempt; the server drops the old one's waiters when it closes);
  //  * the server closed or reset the connection (it exited): no retry, the call fails now and
  //    the next one makes a single connect attempt, which fails fast too.
  // A reply cut off after its status byte leaves the stream desynced: the connection goes too.
  uint8_t response(std::string* out) {
    uint8_t st = 0;
    RecvStatus rs = recv_all_status(fd_, &st, 1);
    if (rs == RecvStatus::kOk) {
      uint32_t n = 0;
      rs = recv_all_status(fd_, &n, 4);
      std::string v(rs == RecvStatus::kOk ? n : 0, '\0');
      if (rs == RecvStatus::kOk && n) rs = recv_all_status(fd_, &v[0], n);
      if (rs == RecvStatus::kOk) {
        if (st == 2) throw std::runtime_error("tds TCPStore: server error: " + v);
        if (out) *out = std::move(v);
        return st;
      }
    }
    drop_connection();
    if (rs == RecvStatus::kTimeout) {
      fd_ = try_connect_once();
      throw std::runtime_error("tds TCPStore: timed out waiting for the store");
    }
    throw std::runtime_error("tds TCPStore: connection to the store lost (server closed it)");
  }
  std::string call(uint8_t op, const std::string& key, const std::string& val) {
    std::lock_guard<std::mutex> g(mu_);
    request(op, key, val, nullptr);
    std::string out;
    response(&out);
    return out;
  }
  uint8_t call_status(uint8_t op, const std::string& key, const std::string& val) {
    std::lock_guard<std::mutex> g(mu_);
    request(op, key, val, nullptr);
    return response(nullptr);
  }
};

}  // namespace tds_comm

TORCH_LIBRARY_FRAGMENT(tdsa, m) {
  m.class_<tds_comm::TCPStore>("TCPStore")
      .def(torch::init<std::string, int64_t, int64_t, bool, int64_t>())
      .def("set", &tds_comm::TCPStore::set)
      .def("get", &tds_comm::TCPStore::get)
      .def("add", &tds_comm::TCPStore::add)
      .def("check", &tds_comm::TCPStore::check)
      .def("wait", &tds_comm::TCPStore::wait)
      .def("delete_key", &tds_comm::TCPStore::delete_key)
      .def("num_keys", &tds_comm::TCPStore::num_keys)
      .def("compare_set", &tds_comm::TCPStore::compare_set)
      .def("port", &tds_comm::TCPStore::port)
      .def("world_size", &tds_comm::TCPStore::world_size)
      .def("set_timeout", &tds_comm::TCPStore::set_timeout);
}
