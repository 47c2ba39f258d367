// CPU test of the settle / abort / watchdog lock protocol of the native RCCL communicator
// (csrc/comm/settle.h, used by csrc/comm/rccl_comm.h).  No RCCL: a "call" that never settles
// stands in for a collective whose peer died.  Checks, with a 20 s call timeout:
//   1. the watchdog's async-error poll never blocks behind a settling call (try-lock);
//   2. an abort requested 100 ms into the settle is honoured within one poll: the settling call
//      returns kSettleAborted and the aborting thread gets the lock well under the timeout;
//   3. after the abort the lock is free and the poll runs again.
// Prints "settle protocol ok" and exits 0, or names the failed check and exits 1.
#include <chrono>
#include <cstdio>
#include <mutex>
#include <thread>

#include "comm/settle.h"

using namespace tds_comm;
using clk = std::chrono::steady_clock;

static double ms_since(clk::time_point t0) {
  return std::chrono::duration<double, std::milli>(clk::now() - t0).count();
}

int main() {
  std::mutex comm_mu;
  std::atomic<bool> aborted{false};
  std::atomic<bool> in_call{false};
  std::atomic<int> polls{0};
  int call_result = 0;
  bool comm_alive = true;  // guarded by comm_mu

  const auto t0 = clk::now();
  std::thread caller([&] {
    std::lock_guard<std::mutex> g(comm_mu);  // held for the whole call, as RcclComm::run does
    in_call = true;
    call_result = settle_wait([&] { ++polls; return kSettleInProgress; }, &aborted, 20000);
  });
  while (!in_call) std::this_thread::yield();

  // 1. the watchdog's poll does not wait for the settling call
  auto tw = clk::now();
  bool ran = try_poll_locked(comm_mu, [] {});
  if (ran || ms_since(tw) > 50.0) {
    std::printf("FAIL: watchdog poll ran=%d or blocked %.1f ms behind a settling call\n", (int)ran, ms_since(tw));
    return 1;
  }

  // 2. abort requested mid-settle
  std::this_thread::sleep_for(std::chrono::milliseconds(100));
  auto ta = clk::now();
  if (!claim_abort(aborted)) {
    std::printf("FAIL: first abort claim refused\n");
    return 1;
  }
  if (claim_abort(aborted)) {
    std::printf("FAIL: abort claimed twice\n");
    return 1;
  }
  abort_locked(comm_mu, [&] { comm_alive = false; });
  const double abort_ms = ms_since(ta);
  caller.join();
  if (call_result != kSettleAborted) {
    std::printf("FAIL: settling call returned %d, not kSettleAborted\n", call_result);
    return 1;
  }
  if (abort_ms > 1000.0 || ms_since(t0) > 5000.0) {
    std::printf("FAIL: abort took %.1f ms (call timeout 20000 ms)\n", abort_ms);
    return 1;
  }
  // 3. lock free again
  bool alive_seen = true;
  if (!try_poll_locked(comm_mu, [&] { alive_seen = comm_alive; }) || alive_seen) {
    std::printf("FAIL: poll after the abort did not run or saw a live communicator\n");
    return 1;
  }
  // a settle that completes normally still reports its state; a timeout reports kSettleTimeout
  std::atomic<bool> no_abort{false};
  int n = 0;
  if (settle_wait([&] { return ++n < 3 ? kSettleInProgress : 0; }, &no_abort, 1000) != 0) {
    std::printf("FAIL: normal settle\n");
    return 1;
  }
  if (settle_wait([] { return kSettleInProgress; }, &no_abort, 20) != kSettleTimeout) {
    std::printf("FAIL: timeout\n");
    return 1;
  }
  std::printf("settle protocol ok: abort honoured in %.2f ms after %d polls\n", abort_ms, polls.load());
  return 0;
}
