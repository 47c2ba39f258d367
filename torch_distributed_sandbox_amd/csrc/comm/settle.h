// The lock protocol between a thread settling a non-blocking RCCL call and the communicator's
// watchdog (csrc/comm/rccl_comm.h).  Header-only and RCCL-free so a CPU test can drive it
// (tests/native/settle_protocol.cpp, tests/test_sanitizers_cpu.py).
//
// A communicator created with ncclConfig_t.blocking = 0 may return ncclInProgress from any
// call; the caller then polls ncclCommGetAsyncError until the state settles.  The caller holds
// the state's comm_mu for the whole call (the communicator must not be aborted and freed under
// it), so the protocol must keep two things from waiting for that lock:
//
//  * an abort request: fail() first publishes `aborted` (an atomic, no lock), and the settle
//    loop re-reads it on every iteration, returning kSettleAborted at once; only then does
//    fail() take comm_mu to call ncclCommAbort.  So an abort requested during a settle is
//    honoured within one poll, not after the call's timeout.
//  * the watchdog's async-error poll: it only try-locks comm_mu.  While a call holds it the
//    caller's own settle loop is polling the same async state, so nothing is missed, and the
//    watchdog goes on checking the pending collectives' completion events and timeouts.
#pragma once

#include <atomic>
#include <chrono>
#include <cstdint>
#include <mutex>
#include <thread>

namespace tds_comm {

constexpr int kSettleInProgress = -1000001;  // poll(): the call is still in flight
constexpr int kSettleAborted = -1000002;     // settle_wait(): an abort was requested meanwhile
constexpr int kSettleTimeout = -1000003;     // settle_wait(): still in flight after timeout_ms

// Poll until the call settles: returns poll()'s final state, kSettleAborted as soon as
// `aborted` is set, or kSettleTimeout after timeout_ms.
template <class Poll>
inline int settle_wait(Poll&& poll, const std::atomic<bool>* aborted, int64_t timeout_ms) {
  const auto t0 = std::chrono::steady_clock::now();
  while (true) {
    const int st = poll();
    if (st != kSettleInProgress) return st;
    if (aborted != nullptr && aborted->load(std::memory_order_acquire)) return kSettleAborted;
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms)) return kSettleTimeout;
    std::this_thread::yield();
  }
}

// fail()'s side: publish the abort (false if another thread already did), then take `mu` --
// released within one poll by a call settling under it -- and run `abort_fn` under it.
inline bool claim_abort(std::atomic<bool>& aborted) {
  bool expected = false;
  return aborted.compare_exchange_strong(expected, true, std::memory_order_acq_rel);
}
template <class AbortFn>
inline void abort_locked(std::mutex& mu, AbortFn&& abort_fn) {
  std::lock_guard<std::mutex> g(mu);
  abort_fn();
}

// The watchdog's side: run `poll_fn` under `mu` only if it is free right now; returns whether
// it ran (a call holding `mu` polls the same state itself).
template <class PollFn>
inline bool try_poll_locked(std::mutex& mu, PollFn&& poll_fn) {
  std::unique_lock<std::mutex> g(mu, std::try_to_lock);
  if (!g.owns_lock()) return false;
  poll_fn();
  return true;
}

}  // namespace tds_comm
