// Native RCCL communicator for device tensors (SURVEY.md §2.3 N1 — the role
// ProcessGroupNCCL plays for the reference's init_process_group('nccl'),
// mnist_distributed.py:50, allreduce_toy.py:44).
//
// One communicator per process/GPU over xGMI, created eagerly from a unique id
// the Python side exchanges through the rendezvous store.  Collectives run on a
// dedicated high-priority HIP stream (so the big gradient all-reduce is
// scheduled ahead of compute work when both are ready):
//
//   caller stream --event--> comm stream: ncclX(...) --done event--> Work
//
// Work::wait() makes the caller's current stream wait on the done event (the host
// never blocks); Work::synchronize() blocks the host.  Buffers are registered with
// the caching allocator on the comm stream (recordStream) so they are not reused
// while the collective is in flight.
//
// A watchdog thread polls outstanding collectives and the communicator's async
// error state; a collective older than the timeout, or an RCCL async error,
// aborts the communicator (ncclCommAbort) and — by default — terminates the
// process so a launcher's fail-fast tears the job down (the same policy as
// torch's TORCH_NCCL_ASYNC_ERROR_HANDLING).  TDS_RCCL_ERROR_HANDLING=raise keeps
// the process alive and rethrows from the next wait/collective instead.
//
// TDS_DEBUG_SYNC=1 is the stream-ordering assertion mode: every collective is
// followed by a host wait on the comm stream and a check of the HIP and RCCL
// async error state, so a fault, a hang or a missing event fence shows up at
// the collective that caused it (named in the error), not steps later.
//
// Links against torch's bundled librccl (one RCCL per process; see _build.py).
#pragma once
#include <ATen/ATen.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <torch/custom_class.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "comm/comm.h"
#include "comm/settle.h"

// csrc/kernels/cu_budget.hip: stream confined to the CUs reserved for communication (or nullptr)
hipStream_t tds_cu_comm_stream(int device);

namespace tds_comm {

#define TDS_RCCL(cmd)                                                                   \
  do {                                                                                  \
    ncclResult_t r_ = (cmd);                                                            \
    TORCH_CHECK(r_ == ncclSuccess, "RCCL error '", ncclGetErrorString(r_), "' in ", #cmd); \
  } while (0)
// A communicator created non-blocking may return ncclInProgress from any call;
// the call has then been accepted and finishes asynchronously.  Poll the async
// state until it settles (bounded, and cut short by an abort request: settle.h),
// then check it like a blocking result.
inline ncclResult_t nccl_settle(ncclResult_t r, ncclComm_t c, int64_t timeout_ms, const std::atomic<bool>* aborted) {
  if (r != ncclInProgress || c == nullptr) return r;
  const int st = settle_wait(
      [c]() -> int {
        ncclResult_t a = ncclInProgress;
        if (ncclCommGetAsyncError(c, &a) != ncclSuccess) return (int)ncclInternalError;
        return a == ncclInProgress ? kSettleInProgress : (int)a;
      },
      aborted, timeout_ms);
  if (st == kSettleAborted) return ncclInvalidUsage;  // the watchdog is aborting the communicator
  if (st == kSettleTimeout) return ncclInProgress;
  return (ncclResult_t)st;
}
#define TDS_RCCL_C(c, cmd)                                                                   \
  do {                                                                                       \
    ncclResult_t r_ = nccl_settle((cmd), (c), st_->timeout_ms, &st_->aborted);               \
    TORCH_CHECK(r_ == ncclSuccess, "RCCL error '", ncclGetErrorString(r_), "' in ", #cmd,    \
                st_->aborted.load() ? " (communicator aborted while the call settled)" : ""); \
  } while (0)
#define TDS_HIP(cmd)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (cmd);                                                             \
    TORCH_CHECK(e_ == hipSuccess, "HIP error '", hipGetErrorString(e_), "' in ", #cmd); \
  } while (0)

inline ncclDataType_t nccl_dtype(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return ncclFloat32;
    case at::kDouble: return ncclFloat64;
    case at::kHalf: return ncclFloat16;
    case at::kBFloat16: return ncclBfloat16;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kChar: return ncclInt8;
    case at::kByte:
    case at::kBool: return ncclUint8;
    default: TORCH_CHECK(false, "rccl: unsupported dtype ", t);
  }
}

inline ncclRedOp_t nccl_op(int64_t op) {
  switch (op) {
    case R_SUM: return ncclSum;
    case R_AVG: return ncclAvg;
    case R_MAX: return ncclMax;
    case R_MIN: return ncclMin;
    case R_PROD: return ncclProd;
    default: TORCH_CHECK(false, "rccl: unsupported reduce op ", op);
  }
}

// State shared by the communicator, its works and the watchdog.
struct RcclState {
  // comm is read by the main thread (collectives, TDS_DEBUG_SYNC checks) and the
  // watchdog, and freed by fail(): every use after construction holds comm_mu, and
  // fail() clears it under the same lock before the communicator is aborted.
  ncclComm_t comm = nullptr;
  std::mutex comm_mu;
  int device = 0;
  int64_t rank = 0, world = 1, timeout_ms = 600000;
  bool exit_on_error = true;
  bool debug_sync = false;  // TDS_DEBUG_SYNC=1
  std::atomic<bool> aborted{false};
  std::mutex mu;
  std::string error;  // guarded by mu
  std::condition_variable cv;
  bool stop = false;  // guarded by mu

  // Completion events are pooled: a collective's event is shared by its Work and the
  // watchdog's pending entry and goes back to the pool when both have let go, so the hot
  // path (2-40 collectives per step on the exchange paths) creates no events after warm-up.
  std::mutex pool_mu;
  std::vector<hipEvent_t> event_pool;  // guarded by pool_mu
  ~RcclState() {
    for (hipEvent_t e : event_pool) (void)hipEventDestroy(e);
  }

  struct Pending {
    std::shared_ptr<hipEvent_t> done;
    std::chrono::steady_clock::time_point start;
    std::string what;
  };
  std::deque<Pending> pending;  // guarded by mu

  // A pooled event, returned to the pool (not destroyed) once the last holder drops it.
  static std::shared_ptr<hipEvent_t> take_event(const std::shared_ptr<RcclState>& self) {
    hipEvent_t e = nullptr;
    {
      std::lock_guard<std::mutex> g(self->pool_mu);
      if (!self->event_pool.empty()) {
        e = self->event_pool.back();
        self->event_pool.pop_back();
      }
    }
    if (e == nullptr) TDS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    std::weak_ptr<RcclState> weak = self;
    return std::shared_ptr<hipEvent_t>(new hipEvent_t(e), [weak](hipEvent_t* p) {
      if (auto st = weak.lock()) {
        std::lock_guard<std::mutex> g(st->pool_mu);
        st->event_pool.push_back(*p);
      } else {
        (void)hipEventDestroy(*p);
      }
      delete p;
    });
  }

  void check_ok() {
    if (aborted.load()) {
      std::lock_guard<std::mutex> g(mu);
      TORCH_CHECK(false, "rccl communicator (rank ", rank, ") was aborted: ", error);
    }
  }

  // Abort once; called from the watchdog (or a failing wait).  `aborted` is published before
  // comm_mu is taken: a call settling under comm_mu sees it on its next poll and returns, so
  // the abort waits one poll, not the call's timeout (settle.h).
  void fail(const std::string& why) {
    if (!claim_abort(aborted)) return;
    {
      std::lock_guard<std::mutex> g(mu);
      error = why;
    }
    std::fprintf(stderr, "[tds rccl] rank %lld: %s -- aborting communicator\n", (long long)rank, why.c_str());
    std::fflush(stderr);
    abort_locked(comm_mu, [this] {
      ncclComm_t c = comm;
      comm = nullptr;
      if (c) ncclCommAbort(c);
    });
    if (exit_on_error) {
      std::fprintf(stderr, "[tds rccl] rank %lld: terminating process (TDS_RCCL_ERROR_HANDLING=raise to disable)\n",
                   (long long)rank);
      std::fflush(stderr);
      std::_Exit(70);
    }
  }
};

struct RcclWork : CommWork {
  std::shared_ptr<RcclState> st;
  std::shared_ptr<hipEvent_t> done;  // pooled (RcclState::take_event)
  int device = 0;

  RcclWork(std::shared_ptr<RcclState> s, std::shared_ptr<hipEvent_t> e)
      : st(std::move(s)), done(std::move(e)), device(st->device) {}

  void wait() override {
    st->check_ok();
    c10::hip::HIPGuard g((c10::DeviceIndex)device);
    TDS_HIP(hipStreamWaitEvent(c10::hip::getCurrentHIPStream((c10::DeviceIndex)device).stream(), *done, 0));
  }
  bool is_completed() override {
    st->check_ok();
    return hipEventQuery(*done) == hipSuccess;
  }
  void synchronize() override {
    const auto t0 = std::chrono::steady_clock::now();
    while (true) {
      st->check_ok();
      hipError_t e = hipEventQuery(*done);
      if (e == hipSuccess) return;
      TORCH_CHECK(e == hipErrorNotReady, "rccl work: ", hipGetErrorString(e));
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(st->timeout_ms)) {
        st->fail("collective did not finish within the timeout (host wait)");
        st->check_ok();
      }
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }
};

class RcclComm : public torch::CustomClassHolder, public CollectiveComm {
 public:
  static at::Tensor unique_id() {
    ncclUniqueId id;
    TDS_RCCL(ncclGetUniqueId(&id));
    auto t = at::empty({(int64_t)sizeof(id)}, at::TensorOptions().dtype(at::kByte));
    std::memcpy(t.data_ptr(), &id, sizeof(id));
    return t;
  }

  // The communicator's stream: with CUs reserved for communication (utils/streams.py) the
  // stream confined to those CUs (cu_budget.hip), so RCCL's kernels never sit on a CU a
  // persistent compute workgroup waits for; otherwise a high-priority pool stream.
  static c10::hip::HIPStream comm_stream_for(int64_t device) {
    if (hipStream_t s = tds_cu_comm_stream((int)device))
      return c10::hip::getStreamFromExternal(s, (c10::DeviceIndex)device);
    return c10::hip::getStreamFromPool(/*isHighPriority=*/true, (c10::DeviceIndex)device);
  }

  RcclComm(int64_t rank, int64_t world, int64_t device, at::Tensor id, int64_t timeout_ms)
      : st_(std::make_shared<RcclState>()),
        stream_(comm_stream_for(device)) {
    TORCH_CHECK(id.numel() == (int64_t)sizeof(ncclUniqueId) && id.scalar_type() == at::kByte,
                "RcclComm: bad unique id");
    st_->rank = rank;
    st_->world = world;
    st_->device = (int)device;
    st_->timeout_ms = timeout_ms;
    const char* eh = std::getenv("TDS_RCCL_ERROR_HANDLING");
    st_->exit_on_error = !(eh && std::string(eh) == "raise");
    st_->debug_sync = env_flag("TDS_DEBUG_SYNC");
    ncclUniqueId uid;
    auto idc = id.contiguous().cpu();
    std::memcpy(&uid, idc.data_ptr(), sizeof(uid));
    c10::hip::HIPGuard g((c10::DeviceIndex)device);
    init_comm(uid);
    TDS_HIP(hipEventCreateWithFlags(&ready_, hipEventDisableTiming));
    watchdog_ = std::thread([s = st_] { watchdog_loop(s); });
  }

  ~RcclComm() override { shutdown(); }

  void shutdown() {
    if (watchdog_.joinable()) {
      {
        std::lock_guard<std::mutex> g(st_->mu);
        st_->stop = true;
      }
      st_->cv.notify_all();
      watchdog_.join();
    }
    if (!st_->aborted.load()) {
      std::lock_guard<std::mutex> cl(st_->comm_mu);
      if (st_->comm) {
        c10::hip::HIPGuard g((c10::DeviceIndex)st_->device);
        (void)hipStreamSynchronize(stream_.stream());
        ncclComm_t c = st_->comm;
        st_->comm = nullptr;
        ncclCommDestroy(c);
      }
    }
    if (ready_) {
      (void)hipEventDestroy(ready_);
      ready_ = nullptr;
    }
    // its storage was recorded on the comm stream: freed here, before a CU split's masked streams
    // are destroyed (utils/streams.py release_streams), not by the destructor at process exit,
    // where the allocator's event on the destroyed stream fails (hipErrorInvalidHandle)
    // After an abort a collective that was running may never finish, so the stream is not
    // waited on (as for the communicator above): the buffer is leaked on purpose instead -- its
    // block must not go back to the allocator while an aborted kernel may still write it.
    if (barrier_buf_.defined()) {
      if (!st_->aborted.load()) {
        (void)hipStreamSynchronize(stream_.stream());
        barrier_buf_ = at::Tensor();
      } else {
        new at::Tensor(std::move(barrier_buf_));  // NOLINT: intentional leak (a few bytes)
      }
    }
  }

  void abort(const std::string& why) {
    const bool keep = st_->exit_on_error;
    st_->exit_on_error = false;  // an explicit abort never terminates the process
    st_->fail(why.empty() ? "aborted by user" : why);
    st_->exit_on_error = keep;
  }

  int64_t comm_rank() const override { return st_->rank; }
  int64_t comm_world() const override { return st_->world; }
  int64_t rank() const { return st_->rank; }
  int64_t world_size() const { return st_->world; }
  int64_t device() const { return st_->device; }
  // ncclCommCount of the live communicator (the bench reports it as rccl_ranks)
  int64_t comm_count() {
    std::lock_guard<std::mutex> g(st_->comm_mu);
    st_->check_ok();
    int n = 0;
    TORCH_CHECK(st_->comm != nullptr, "rccl: communicator is gone");
    TDS_RCCL(ncclCommCount(st_->comm, &n));
    return n;
  }
  int64_t cta_budget_min() const { return min_ctas_; }
  int64_t cta_budget_max() const { return max_ctas_; }
  int64_t pending() {
    std::lock_guard<std::mutex> g(st_->mu);
    return (int64_t)st_->pending.size();
  }

  // ---------------------------------------------------------------- collectives
  c10::intrusive_ptr<CommWork> allreduce_async(at::Tensor t, int64_t op) override {
    check_dev(t);
    return run({t}, "allreduce", [&](ncclComm_t c, hipStream_t s) {
      TDS_RCCL_C(c, ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t.scalar_type()), nccl_op(op), c, s));
    });
  }
  c10::intrusive_ptr<CommWork> allreduce(at::Tensor t, int64_t op) { return allreduce_async(t, op); }

  c10::intrusive_ptr<CommWork> broadcast(at::Tensor t, int64_t root) {
    check_dev(t);
    return run({t}, "broadcast", [&](ncclComm_t c, hipStream_t s) {
      TDS_RCCL_C(c, ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t.scalar_type()), (int)root, c, s));
    });
  }

  // One grouped launch for many tensors (DDP's coalesced state/buffer broadcast, N5).
  c10::intrusive_ptr<CommWork> broadcast_coalesced(std::vector<at::Tensor> ts, int64_t root) {
    for (auto& t : ts) check_dev(t);
    return run(ts, "broadcast_coalesced", [&](ncclComm_t c, hipStream_t s) {
      TDS_RCCL(ncclGroupStart());
      for (auto& t : ts)
        TDS_RCCL_C(c, ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t.scalar_type()), (int)root, c, s));
      TDS_RCCL_C(c, ncclGroupEnd());
    });
  }

  c10::intrusive_ptr<CommWork> reduce(at::Tensor t, int64_t root, int64_t op) {
    check_dev(t);
    return run({t}, "reduce", [&](ncclComm_t c, hipStream_t s) {
      TDS_RCCL_C(c, ncclReduce(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t.scalar_type()), nccl_op(op), (int)root,
                          c, s));
    });
  }

  c10::intrusive_ptr<CommWork> allgather(at::Tensor out, at::Tensor in) {
    check_dev(out);
    check_dev(in);
    TORCH_CHECK(out.numel() == in.numel() * st_->world && out.scalar_type() == in.scalar_type(),
                "rccl allgather: output must hold world_size x input elements");
    return run({out, in}, "allgather", [&](ncclComm_t c, hipStream_t s) {
      TDS_RCCL_C(c, ncclAllGather(in.data_ptr(), out.data_ptr(), in.numel(), nccl_dtype(in.scalar_type()), c, s));
    });
  }

  c10::intrusive_ptr<CommWork> reduce_scatter(at::Tensor out, at::Tensor in, int64_t op) {
    check_dev(out);
    check_dev(in);
    TORCH_CHECK(in.numel() == out.numel() * st_->world && out.scalar_type() == in.scalar_type(),
                "rccl reduce_scatter: input must hold world_size x output elements");
    return run({out, in}, "reduce_scatter", [&](ncclComm_t c, hipStream_t s) {
      TDS_RCCL_C(c, ncclReduceScatter(in.data_ptr(), out.data_ptr(), out.numel(), nccl_dtype(in.scalar_type()),
                                 nccl_op(op), c, s));
    });
  }

  // equal splits: in/out are [world * n]
  c10::intrusive_ptr<CommWork> alltoall(at::Tensor out, at::Tensor in) {
    check_dev(out);
    check_dev(in);
    TORCH_CHECK(in.numel() == out.numel() && in.numel() % st_->world == 0, "rccl alltoall: bad sizes");
    const int64_t n = in.numel() / st_->world, esz = in.element_size();
    return run({out, in}, "alltoall", [&](ncclComm_t c, hipStream_t s) {
      const auto dt = nccl_dtype(in.scalar_type());
      TDS_RCCL(ncclGroupStart());
      for (int64_t r = 0; r < st_->world; ++r) {
        TDS_RCCL_C(c, ncclSend(static_cast<char*>(in.data_ptr()) + r * n * esz, n, dt, (int)r, c, s));
        TDS_RCCL_C(c, ncclRecv(static_cast<char*>(out.data_ptr()) + r * n * esz, n, dt, (int)r, c, s));
      }
      TDS_RCCL_C(c, ncclGroupEnd());
    });
  }

  c10::intrusive_ptr<CommWork> send(at::Tensor t, int64_t peer) {
    check_dev(t);
    return run({t}, "send", [&](ncclComm_t c, hipStream_t s) {
      TDS_RCCL_C(c, ncclSend(t.data_ptr(), t.numel(), nccl_dtype(t.scalar_type()), (int)peer, c, s));
    });
  }

  c10::intrusive_ptr<CommWork> recv(at::Tensor t, int64_t peer) {
    check_dev(t);
    return run({t}, "recv", [&](ncclComm_t c, hipStream_t s) {
      TDS_RCCL_C(c, ncclRecv(t.data_ptr(), t.numel(), nccl_dtype(t.scalar_type()), (int)peer, c, s));
    });
  }

  // Grouped point-to-point exchange: every (tensor, peer) pair in `sends` is sent and
  // every pair in `recvs` received inside one ncclGroupStart/End, so each peer pair
  // uses its own xGMI link concurrently.  The building block of the sharded fc
  // exchange (parallel/factored.py): strided all-to-all of activation shards and the
  // all-gather of gradient shards, uneven splits included.
  c10::intrusive_ptr<CommWork> sendrecv(std::vector<at::Tensor> sends, std::vector<int64_t> send_peers,
                                        std::vector<at::Tensor> recvs, std::vector<int64_t> recv_peers) {
    TORCH_CHECK(sends.size() == send_peers.size() && recvs.size() == recv_peers.size(),
                "rccl sendrecv: tensors and peers must pair up");
    std::vector<at::Tensor> all;
    for (auto& t : sends) { check_dev(t); all.push_back(t); }
    for (auto& t : recvs) { check_dev(t); all.push_back(t); }
    for (auto p : send_peers) TORCH_CHECK(p >= 0 && p < st_->world, "rccl sendrecv: bad peer ", p);
    for (auto p : recv_peers) TORCH_CHECK(p >= 0 && p < st_->world, "rccl sendrecv: bad peer ", p);
    return run(all, "sendrecv", [&](ncclComm_t c, hipStream_t s) {
      TDS_RCCL(ncclGroupStart());
      for (size_t i = 0; i < sends.size(); ++i)
        TDS_RCCL_C(c, ncclSend(sends[i].data_ptr(), sends[i].numel(), nccl_dtype(sends[i].scalar_type()),
                               (int)send_peers[i], c, s));
      for (size_t i = 0; i < recvs.size(); ++i)
        TDS_RCCL_C(c, ncclRecv(recvs[i].data_ptr(), recvs[i].numel(), nccl_dtype(recvs[i].scalar_type()),
                               (int)recv_peers[i], c, s));
      TDS_RCCL_C(c, ncclGroupEnd());
    });
  }

  // ProcessGroupNCCL semantics: a 1-element all-reduce, then the host waits for it.
  void barrier() {
    c10::hip::HIPGuard g((c10::DeviceIndex)st_->device);
    if (!barrier_buf_.defined())
      barrier_buf_ = at::zeros({1}, at::TensorOptions().dtype(at::kInt).device(at::kCUDA, st_->device));
    auto w = allreduce_async(barrier_buf_, R_SUM);
    w->synchronize();
  }

 private:
  std::shared_ptr<RcclState> st_;
  c10::hip::HIPStream stream_;
  hipEvent_t ready_ = nullptr;
  std::thread watchdog_;
  at::Tensor barrier_buf_;
  std::mutex run_mu_;  // the caller (main thread) and the reducer (autograd thread) may both enqueue
  int64_t min_ctas_ = 0, max_ctas_ = 0;  // 0 = RCCL's own choice

  static bool env_flag(const char* name) {
    const char* v = std::getenv(name);
    return v && *v && std::string(v) != "0";  // same rule as parallel/distributed.py
  }
  static int64_t env_int(const char* name, int64_t dflt) {
    const char* v = std::getenv(name);
    return (v && *v) ? std::atoll(v) : dflt;
  }

  // Communicator creation.  Default: ncclCommInitRankConfig with blocking=0, then a
  // bounded poll of the async state, so a rank that never joins turns into an error
  // (and an aborted communicator) after TDS_RCCL_INIT_TIMEOUT_MS instead of hanging
  // the others forever (the watchdog only exists once init has returned).
  // TDS_RCCL_MIN_CTAS / TDS_RCCL_MAX_CTAS bound the workgroups (CUs) RCCL's kernels
  // take from the compute kernels they overlap with.
  void init_comm(const ncclUniqueId& uid) {
    min_ctas_ = env_int("TDS_RCCL_MIN_CTAS", 0);
    max_ctas_ = env_int("TDS_RCCL_MAX_CTAS", 0);
    if (env_flag("TDS_RCCL_BLOCKING_INIT")) {
      TORCH_CHECK(min_ctas_ == 0 && max_ctas_ == 0, "TDS_RCCL_*_CTAS needs the config (non-blocking) init");
      TDS_RCCL(ncclCommInitRank(&st_->comm, (int)st_->world, uid, (int)st_->rank));
      return;
    }
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    if (min_ctas_ > 0) cfg.minCTAs = (int)min_ctas_;
    if (max_ctas_ > 0) cfg.maxCTAs = (int)max_ctas_;
    const int64_t limit_ms = env_int("TDS_RCCL_INIT_TIMEOUT_MS", st_->timeout_ms);
    ncclComm_t c = nullptr;
    ncclResult_t r = ncclCommInitRankConfig(&c, (int)st_->world, uid, (int)st_->rank, &cfg);
    TORCH_CHECK(r == ncclSuccess || r == ncclInProgress, "RCCL error '", ncclGetErrorString(r),
                "' in ncclCommInitRankConfig (rank ", st_->rank, " of ", st_->world, ")");
    const auto t0 = std::chrono::steady_clock::now();
    ncclResult_t state = r;
    while (state == ncclInProgress) {
      if (ncclCommGetAsyncError(c, &state) != ncclSuccess) state = ncclInternalError;
      if (state != ncclInProgress) break;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(limit_ms)) {
        ncclCommAbort(c);
        TORCH_CHECK(false, "rccl: communicator init did not complete within ", limit_ms, " ms on rank ", st_->rank,
                    " of ", st_->world, " (a rank did not join?)");
      }
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    if (state != ncclSuccess) {
      ncclCommAbort(c);
      TORCH_CHECK(false, "RCCL error '", ncclGetErrorString(state), "' during communicator init (rank ", st_->rank,
                  ")");
    }
    st_->comm = c;
  }

  void check_dev(const at::Tensor& t) const {
    TORCH_CHECK(t.is_cuda() && t.get_device() == st_->device, "rccl: tensor must be on cuda:", st_->device);
    TORCH_CHECK(t.is_contiguous(), "rccl: tensor must be contiguous");
  }

  template <class F>
  c10::intrusive_ptr<CommWork> run(const std::vector<at::Tensor>& ts, const char* what, F&& fn) {
    st_->check_ok();
    std::lock_guard<std::mutex> run_lock(run_mu_);
    c10::hip::HIPGuard g((c10::DeviceIndex)st_->device);
    hipStream_t cur = c10::hip::getCurrentHIPStream((c10::DeviceIndex)st_->device).stream();
    hipStream_t cs = stream_.stream();
    // comm stream waits for the producer work already queued on the caller's stream
    TDS_HIP(hipEventRecord(ready_, cur));
    TDS_HIP(hipStreamWaitEvent(cs, ready_, 0));
    // An RCCL error inside fn (including a non-blocking call that did not settle within the
    // timeout) aborts the communicator -- after comm_mu is released, so the abort (and the
    // watchdog, which polls under the same lock) can take it -- instead of leaving it in flight.
    std::string err;
    {
      std::lock_guard<std::mutex> cl(st_->comm_mu);
      st_->check_ok();
      try {
        fn(st_->comm, cs);
      } catch (const std::exception& e) {
        err = e.what();
      }
    }
    if (!err.empty()) {
      st_->fail(std::string(what) + ": " + err);
      st_->check_ok();
      TORCH_CHECK(false, what, ": ", err);
    }
    for (const auto& t : ts) c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(), stream_);
    // one pooled event serves the Work and the watchdog (which keeps it alive if the Work is
    // dropped before completion)
    auto done = RcclState::take_event(st_);
    TDS_HIP(hipEventRecord(*done, cs));
    {
      std::lock_guard<std::mutex> gl(st_->mu);
      st_->pending.push_back({done, std::chrono::steady_clock::now(), what});
    }
    if (st_->debug_sync) debug_sync_check(cs, what);
    return c10::make_intrusive<RcclWork>(st_, done);
  }

  // TDS_DEBUG_SYNC: block until this collective has finished and surface any error here
  void debug_sync_check(hipStream_t cs, const char* what) {
    const hipError_t he = hipStreamSynchronize(cs);
    TORCH_CHECK(he == hipSuccess, "TDS_DEBUG_SYNC: ", what, " on rank ", st_->rank, ": HIP error ",
                hipGetErrorString(he));
    st_->check_ok();  // a watchdog abort is reported as such, never as a use of a freed communicator
    ncclResult_t ae = ncclSuccess;
    {
      std::lock_guard<std::mutex> cl(st_->comm_mu);
      if (st_->comm) TDS_RCCL(ncclCommGetAsyncError(st_->comm, &ae));
    }
    TORCH_CHECK(ae == ncclSuccess, "TDS_DEBUG_SYNC: ", what, " on rank ", st_->rank, ": RCCL async error ",
                ncclGetErrorString(ae));
    st_->check_ok();
  }

  static void watchdog_loop(std::shared_ptr<RcclState> s) {
    (void)hipSetDevice(s->device);
    std::unique_lock<std::mutex> lk(s->mu);
    while (!s->stop) {
      s->cv.wait_for(lk, std::chrono::milliseconds(100));
      if (s->stop || s->aborted.load()) break;
      const auto now = std::chrono::steady_clock::now();
      std::string why;
      while (!s->pending.empty()) {
        auto& p = s->pending.front();
        hipError_t e = hipEventQuery(*p.done);
        if (e == hipSuccess) {
          s->pending.pop_front();  // back to the pool once the Work is gone too
          continue;
        }
        if (e != hipErrorNotReady) {
          why = std::string("HIP error on the comm stream: ") + hipGetErrorString(e);
        } else if (now - p.start > std::chrono::milliseconds(s->timeout_ms)) {
          why = "collective '" + p.what + "' did not complete within " + std::to_string(s->timeout_ms) + " ms";
        }
        break;  // collectives complete in order on the comm stream
      }
      if (why.empty()) {
        // try-lock only: while a call holds comm_mu its own settle loop polls this same async
        // state (settle.h), so the watchdog never stalls behind a settling call
        try_poll_locked(s->comm_mu, [&] {
          ncclResult_t ae = ncclSuccess;
          if (s->comm && ncclCommGetAsyncError(s->comm, &ae) == ncclSuccess && ae != ncclSuccess &&
              ae != ncclInProgress)
            why = std::string("RCCL async error: ") + ncclGetErrorString(ae);
        });
      }
      if (!why.empty()) {
        lk.unlock();
        s->fail(why);
        lk.lock();
        break;
      }
    }
  }
};

}  // namespace tds_comm
