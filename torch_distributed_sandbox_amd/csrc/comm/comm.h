// Transport-neutral collective interface shared by the native communicators
// (RcclComm: device tensors over RCCL/xGMI; HostComm: CPU tensors over the TCP
// ring) so the C++ gradient reducer (reducer.cpp) can drive either.
#pragma once
#include <ATen/ATen.h>
#include <torch/custom_class.h>

namespace tds_comm {

enum RedOp : int64_t { R_SUM = 0, R_AVG = 1, R_MAX = 2, R_MIN = 3, R_PROD = 4 };

// Handle of an enqueued collective.  wait() orders the *current* stream after the
// collective (device-side, host does not block) and rethrows communicator errors;
// synchronize() blocks the host until the collective has finished.
struct CommWork : torch::CustomClassHolder {
  virtual void wait() = 0;
  virtual void synchronize() = 0;
  virtual bool is_completed() = 0;
};

struct CollectiveComm {
  virtual ~CollectiveComm() = default;
  virtual c10::intrusive_ptr<CommWork> allreduce_async(at::Tensor t, int64_t op) = 0;
  virtual int64_t comm_rank() const = 0;
  virtual int64_t comm_world() const = 0;
};

// Work that is already complete (synchronous transports).
struct DoneWork : CommWork {
  void wait() override {}
  void synchronize() override {}
  bool is_completed() override { return true; }
};

}  // namespace tds_comm
