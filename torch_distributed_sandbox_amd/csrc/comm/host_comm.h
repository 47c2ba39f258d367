// Native host (CPU-tensor) collective backend over TCP — the gloo-equivalent of
// SURVEY.md §2.3 N2 (the reference falls back to gloo when no GPU is present,
// test_init.py:55,84-88).
//
// Topology: a ring.  Each rank listens on an ephemeral port, the addresses are
// exchanged through the rendezvous store (parallel/host_backend.py), then rank r
// connects to r+1 and accepts r-1.  Collectives:
//   all-reduce : ring reduce-scatter + ring all-gather (bandwidth-optimal,
//                2(W-1)/W of the buffer on each link), SUM/AVG/MAX/MIN/PRODUCT
//   broadcast  : pipelined along the ring from the root, 1 MiB chunks
//   all-gather : ring
//   barrier    : 1-element all-reduce
// Every transfer is full-duplex (send to next while receiving from prev) with
// poll() on non-blocking sockets, so large messages cannot deadlock, and every
// wait is bounded by the timeout.
#pragma once
#include <ATen/ATen.h>
#include <ATen/Dispatch.h>
#include <fcntl.h>
#include <poll.h>
#include <sys/socket.h>
#include <torch/custom_class.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <string>
#include <vector>

#include "comm/comm.h"
#include "comm/net.h"

namespace tds_comm {

class HostComm : public torch::CustomClassHolder, public CollectiveComm {
 public:
  HostComm(int64_t rank, int64_t world, int64_t timeout_ms) : rank_(rank), world_(world), timeout_ms_(timeout_ms) {
    TORCH_CHECK(world >= 1 && rank >= 0 && rank < world, "HostComm: bad rank/world");
    if (world_ > 1) listen_fd_ = listen_on(0, &port_);
  }
  ~HostComm() override { close_all(); }

  int64_t port() const { return port_; }
  int64_t rank() const { return rank_; }
  int64_t world_size() const { return world_; }
  int64_t comm_rank() const override { return rank_; }
  int64_t comm_world() const override { return world_; }

  // synchronous transport: the collective is done when this returns
  c10::intrusive_ptr<CommWork> allreduce_async(at::Tensor t, int64_t op) override {
    allreduce_(t, op);
    return c10::make_intrusive<DoneWork>();
  }

  // peers[i] = "host:port" of rank i
  void connect(std::vector<std::string> peers) {
    if (world_ == 1) return;
    TORCH_CHECK((int64_t)peers.size() == world_, "HostComm.connect: need one address per rank");
    const std::string& nxt = peers[(rank_ + 1) % world_];
    const auto colon = nxt.rfind(':');
    send_fd_ = connect_to(nxt.substr(0, colon), std::stoi(nxt.substr(colon + 1)), timeout_ms_);
    int32_t me = (int32_t)rank_;
    send_all(send_fd_, &me, 4);
    // accept the connection from rank-1 (bounded wait)
    pollfd pf{listen_fd_, POLLIN, 0};
    TORCH_CHECK(::poll(&pf, 1, (int)timeout_ms_) == 1, "HostComm: timed out waiting for rank ",
                (rank_ + world_ - 1) % world_, " to connect");
    recv_fd_ = ::accept(listen_fd_, nullptr, nullptr);
    TORCH_CHECK(recv_fd_ >= 0, "HostComm: accept failed");
    set_rcv_timeout(recv_fd_, timeout_ms_);
    int32_t who = -1;
    recv_all(recv_fd_, &who, 4);
    TORCH_CHECK(who == (rank_ + world_ - 1) % world_, "HostComm: ring miswired (got rank ", who, ")");
    ::fcntl(send_fd_, F_SETFL, ::fcntl(send_fd_, F_GETFL) | O_NONBLOCK);
    ::fcntl(recv_fd_, F_SETFL, ::fcntl(recv_fd_, F_GETFL) | O_NONBLOCK);
  }

  void allreduce_(at::Tensor t, int64_t op) {
    check_cpu(t);
    if (world_ == 1 || t.numel() == 0) return;
    const int64_t esz = t.element_size(), n = t.numel();
    char* base = static_cast<char*>(t.data_ptr());
    std::vector<int64_t> off(world_ + 1);  // segment boundaries (elements)
    for (int64_t i = 0; i <= world_; ++i) off[i] = n * i / world_;
    // reduce-scatter leaves the fully reduced segment (rank+1)%W here ...
    ring_reduce_scatter(t, base, off, 0, op == R_AVG ? R_SUM : op);
    // ... and the all-gather circulates the reduced segments
    for (int64_t s = 0; s < world_ - 1; ++s) {
      const int64_t sseg = (rank_ + 1 - s + world_) % world_, rseg = (rank_ - s + world_) % world_;
      duplex(base + off[sseg] * esz, (off[sseg + 1] - off[sseg]) * esz, base + off[rseg] * esz,
             (off[rseg + 1] - off[rseg]) * esz);
    }
    if (op == R_AVG) avg_(t);
  }

  // out: numel(in)/W elements = this rank's reduced slice of in (in is not modified)
  void reduce_scatter_(at::Tensor out, at::Tensor in, int64_t op) {
    check_cpu(out);
    check_cpu(in);
    TORCH_CHECK(in.numel() == out.numel() * world_ && out.scalar_type() == in.scalar_type(),
                "HostComm.reduce_scatter: input must hold world_size x output elements");
    if (world_ == 1) {
      out.copy_(in.view_as(out));
      return;
    }
    at::Tensor work = in.clone();
    const int64_t m = out.numel();
    std::vector<int64_t> off(world_ + 1);
    for (int64_t i = 0; i <= world_; ++i) off[i] = m * i;
    // shift 1: rank r finishes holding segment r
    ring_reduce_scatter(work, static_cast<char*>(work.data_ptr()), off, 1, op == R_AVG ? R_SUM : op);
    std::memcpy(out.data_ptr(), static_cast<char*>(work.data_ptr()) + off[rank_] * in.element_size(),
                m * in.element_size());
    if (op == R_AVG) avg_(out);
  }

  void broadcast_(at::Tensor t, int64_t root) {
    check_cpu(t);
    if (world_ == 1 || t.numel() == 0) return;
    char* p = static_cast<char*>(t.data_ptr());
    const int64_t bytes = t.numel() * t.element_size();
    const int64_t chunk = 1 << 20;
    const int64_t next = (rank_ + 1) % world_;
    for (int64_t o = 0; o < bytes; o += chunk) {
      const int64_t m = std::min(chunk, bytes - o);
      if (rank_ != root) duplex(nullptr, 0, p + o, m);
      if (next != root) duplex(p + o, m, nullptr, 0);
    }
  }

  // out: [world * numel(in)] contiguous
  void allgather(at::Tensor out, at::Tensor in) {
    check_cpu(out);
    check_cpu(in);
    TORCH_CHECK(out.numel() == in.numel() * world_ && out.scalar_type() == in.scalar_type(),
                "HostComm.allgather: output must hold world_size x input elements");
    const int64_t bytes = in.numel() * in.element_size();
    char* o = static_cast<char*>(out.data_ptr());
    std::memcpy(o + rank_ * bytes, in.data_ptr(), bytes);
    for (int64_t s = 0; s < world_ - 1; ++s) {
      const int64_t sidx = (rank_ - s + world_) % world_, ridx = (rank_ - s - 1 + world_) % world_;
      duplex(o + sidx * bytes, bytes, o + ridx * bytes, bytes);
    }
  }

  void barrier() {
    auto t = at::ones({1}, at::TensorOptions().dtype(at::kInt));
    allreduce_(t, R_SUM);
    TORCH_CHECK(t.item<int>() == world_, "HostComm.barrier: inconsistent result");
  }

  void close_all() {
    for (int* fd : {&send_fd_, &recv_fd_, &listen_fd_}) {
      if (*fd >= 0) ::close(*fd);
      *fd = -1;
    }
  }

 private:
  int64_t rank_, world_, timeout_ms_;
  int listen_fd_ = -1, send_fd_ = -1, recv_fd_ = -1;
  int port_ = 0;

  void avg_(at::Tensor& t) const {
    if (t.is_floating_point()) t.div_(world_);
    else t.div_(world_, "floor");
  }

  // W-1 ring steps; at step s rank r sends segment (r-s-shift) and reduces the
  // incoming segment (r-s-shift-1) into place.  Afterwards segment (r+1-shift)
  // holds the full reduction on rank r.
  void ring_reduce_scatter(const at::Tensor& like, char* base, const std::vector<int64_t>& off, int64_t shift,
                           int64_t op) {
    const int64_t esz = like.element_size();
    int64_t maxseg = 0;
    for (int64_t i = 0; i < world_; ++i) maxseg = std::max(maxseg, off[i + 1] - off[i]);
    std::vector<char> tmp(maxseg * esz);
    for (int64_t s = 0; s < world_ - 1; ++s) {
      const int64_t sseg = ((rank_ - s - shift) % world_ + world_) % world_;
      const int64_t rseg = ((rank_ - s - shift - 1) % world_ + world_) % world_;
      duplex(base + off[sseg] * esz, (off[sseg + 1] - off[sseg]) * esz, tmp.data(), (off[rseg + 1] - off[rseg]) * esz);
      reduce_into(like, base + off[rseg] * esz, tmp.data(), off[rseg + 1] - off[rseg], op);
    }
  }

  static void check_cpu(const at::Tensor& t) {
    TORCH_CHECK(t.device().is_cpu(), "host backend: tensors must live on the CPU (use the rccl backend for GPU)");
    TORCH_CHECK(t.is_contiguous(), "host backend: tensors must be contiguous");
  }

  // Send sn bytes to next while receiving rn bytes from prev (full duplex, bounded).
  void duplex(const char* sbuf, int64_t sn, char* rbuf, int64_t rn) {
    int64_t sd = 0, rd = 0;
    auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms_);
    while (sd < sn || rd < rn) {
      pollfd fds[2];
      int nf = 0, si = -1, ri = -1;
      if (sd < sn) { fds[nf] = {send_fd_, POLLOUT, 0}; si = nf++; }
      if (rd < rn) { fds[nf] = {recv_fd_, POLLIN, 0}; ri = nf++; }
      const int left = (int)std::chrono::duration_cast<std::chrono::milliseconds>(
                           deadline - std::chrono::steady_clock::now()).count();
      TORCH_CHECK(left > 0, "host backend: collective timed out after ", timeout_ms_, " ms (rank ", rank_,
                  ") - a peer is likely dead or hung");
      const int r = ::poll(fds, nf, std::min(left, 1000));
      if (r < 0) {
        if (errno == EINTR) continue;
        TORCH_CHECK(false, "host backend: poll failed: ", std::strerror(errno));
      }
      if (si >= 0 && (fds[si].revents & (POLLOUT | POLLERR | POLLHUP))) {
        const ssize_t w = ::send(send_fd_, sbuf + sd, (size_t)(sn - sd), MSG_NOSIGNAL);
        if (w > 0) {
          sd += w;
        } else if (w < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) {
          TORCH_CHECK(false, "host backend: send to rank ", (rank_ + 1) % world_, " failed: ", std::strerror(errno));
        }
      }
      if (ri >= 0 && (fds[ri].revents & (POLLIN | POLLERR | POLLHUP))) {
        const ssize_t g = ::recv(recv_fd_, rbuf + rd, (size_t)(rn - rd), 0);
        if (g > 0) {
          rd += g;
        } else if (g == 0) {
          TORCH_CHECK(false, "host backend: rank ", (rank_ + world_ - 1) % world_, " closed the ring");
        } else if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) {
          TORCH_CHECK(false, "host backend: recv failed: ", std::strerror(errno));
        }
      }
    }
  }

  static void reduce_into(const at::Tensor& like, char* dst, const char* src, int64_t n, int64_t op) {
    AT_DISPATCH_ALL_TYPES_AND3(at::kHalf, at::kBFloat16, at::kBool, like.scalar_type(), "host_reduce", [&] {
      scalar_t* d = reinterpret_cast<scalar_t*>(dst);
      const scalar_t* s = reinterpret_cast<const scalar_t*>(src);
      switch (op) {
        case R_SUM:
          for (int64_t i = 0; i < n; ++i) d[i] = static_cast<scalar_t>(d[i] + s[i]);
          break;
        case R_PROD:
          for (int64_t i = 0; i < n; ++i) d[i] = static_cast<scalar_t>(d[i] * s[i]);
          break;
        case R_MAX:
          for (int64_t i = 0; i < n; ++i) d[i] = s[i] > d[i] ? s[i] : d[i];
          break;
        case R_MIN:
          for (int64_t i = 0; i < n; ++i) d[i] = s[i] < d[i] ? s[i] : d[i];
          break;
        default:
          TORCH_CHECK(false, "host backend: unsupported reduce op ", op);
      }
    });
  }
};

}  // namespace tds_comm

