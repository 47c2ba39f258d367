// Host-side sanitizer harness for the native rendezvous store and the TCP ring backend
// (SURVEY.md §5 "Race detection / sanitizers": ASan + UBSan on host C++ only; GPU ASan is
// not available on MI355X boxes of this pool).
//
// One process, one thread per rank.  Every rank owns a TCPStore client (rank 0 also hosts
// the server thread) and a HostComm ring, exactly as parallel/host_backend.py wires them,
// and then:
//   * hammers the store concurrently (ADD counters, SET/GET, WAIT, compare-and-set),
//   * runs ring all-reduce SUM/AVG/MAX on sizes that do not divide by the world size,
//     broadcast, all-gather, reduce-scatter and barrier, checking every result exactly.
// Built and run by tests/test_sanitizers_cpu.py with -fsanitize=address,undefined; any
// sanitizer report aborts the process (halt_on_error) and fails the test.
#include "comm/host_comm.h"
#include "comm/tcp_store.cpp"

#include <cstdio>
#include <exception>
#include <string>
#include <thread>
#include <vector>

using tds_comm::HostComm;
using tds_comm::TCPStore;

namespace {

at::Tensor str_tensor(const std::string& s) {
  auto t = at::empty({(int64_t)s.size()}, at::TensorOptions().dtype(at::kByte));
  if (!s.empty()) std::memcpy(t.data_ptr(), s.data(), s.size());
  return t;
}
std::string tensor_str(const at::Tensor& t) {
  if (t.numel() == 0) return std::string();
  return std::string(reinterpret_cast<const char*>(t.data_ptr()), t.numel());
}

void check(bool ok, const std::string& what) {
  if (!ok) throw std::runtime_error("check failed: " + what);
}

void rank_main(int rank, int world, int port, std::string* err) {
  try {
    TCPStore store("127.0.0.1", port, world, /*is_server=*/false, 20000);
    // ---- store stress: concurrent counters, values, waits, CAS
    for (int i = 0; i < 200; ++i) store.add("ctr", 1);
    store.set("val/" + std::to_string(rank), str_tensor("v" + std::to_string(rank * 7)));
    for (int r = 0; r < world; ++r) {
      store.wait("val/" + std::to_string(r), 20000);
      check(tensor_str(store.get("val/" + std::to_string(r))) == "v" + std::to_string(r * 7), "store get");
    }
    // exactly one rank wins the CAS from "" to its own id: a winner sees its own id come back
    // (compare_set returns the value now stored) and counts itself
    const std::string me = std::to_string(rank);
    const std::string got = tensor_str(store.compare_set("owner", str_tensor(""), str_tensor(me)));
    const bool won = got == me;
    if (won) store.add("cas_wins", 1);
    store.add("arrive", 1);
    while (store.add("arrive", 0) < world) std::this_thread::sleep_for(std::chrono::milliseconds(1));
    check(store.add("ctr", 0) == 200 * world, "store counter");
    const std::string owner = tensor_str(store.get("owner"));
    check(!owner.empty() && std::stoi(owner) >= 0 && std::stoi(owner) < world, "store CAS owner");
    check(store.add("cas_wins", 0) == 1, "store CAS: exactly one winner");
    check(won == (owner == me), "store CAS: the winner is the stored owner");
    check(got == owner, "store CAS: every loser sees the winner's id");

    // ---- ring backend
    HostComm comm(rank, world, 20000);
    store.set("addr/" + std::to_string(rank), str_tensor("127.0.0.1:" + std::to_string(comm.port())));
    std::vector<std::string> peers;
    for (int r = 0; r < world; ++r) peers.push_back(tensor_str(store.get("addr/" + std::to_string(r))));
    comm.connect(peers);
    for (int64_t n : {1, 7, 1001, 65539}) {
      auto x = at::arange(n, at::kFloat) + (float)rank;
      comm.allreduce_(x, tds_comm::R_SUM);
      auto want = at::arange(n, at::kFloat) * (float)world + (float)(world * (world - 1) / 2);
      check(at::equal(x, want), "allreduce SUM n=" + std::to_string(n));
      auto m = at::full({n}, (double)rank, at::kDouble);
      comm.allreduce_(m, tds_comm::R_MAX);
      check(at::equal(m, at::full({n}, (double)(world - 1), at::kDouble)), "allreduce MAX");
      auto a = at::full({n}, (int64_t)(2 * rank), at::kLong);
      comm.allreduce_(a, tds_comm::R_AVG);
      check(at::equal(a, at::full({n}, (int64_t)(world - 1), at::kLong)), "allreduce AVG int64");
    }
    auto b = rank == 1 ? at::arange(333, at::kInt) : at::zeros({333}, at::kInt);
    comm.broadcast_(b, 1);
    check(at::equal(b, at::arange(333, at::kInt)), "broadcast");
    auto in = at::full({5}, (float)rank);
    auto out = at::empty({5 * world});
    comm.allgather(out, in);
    for (int r = 0; r < world; ++r) check(at::equal(out.slice(0, 5 * r, 5 * r + 5), at::full({5}, (float)r)), "allgather");
    auto rin = at::ones({4 * world}) * (float)(rank + 1);
    auto rout = at::empty({4});
    comm.reduce_scatter_(rout, rin, tds_comm::R_SUM);
    check(at::equal(rout, at::full({4}, (float)(world * (world + 1) / 2))), "reduce_scatter");
    comm.barrier();
    comm.close_all();
  } catch (const std::exception& e) {
    *err = "rank " + std::to_string(rank) + ": " + e.what();
  }
}

}  // namespace

int main(int argc, char** argv) {
  const int world = argc > 1 ? std::atoi(argv[1]) : 4;
  TCPStore server("127.0.0.1", 0, world, /*is_server=*/true, 20000);
  const int port = (int)server.port();
  std::vector<std::string> errs(world);
  std::vector<std::thread> ts;
  for (int r = 0; r < world; ++r) ts.emplace_back(rank_main, r, world, port, &errs[r]);
  for (auto& t : ts) t.join();
  int bad = 0;
  for (auto& e : errs)
    if (!e.empty()) {
      std::fprintf(stderr, "%s\n", e.c_str());
      ++bad;
    }
  if (bad) return 1;
  std::printf("sanitize_host_comm ok: world=%d\n", world);
  return 0;
}
