// Native gradient reducer for DistributedDataParallel (SURVEY.md §2.3 N4 — the
// role of torch's C++ Reducer behind nn.parallel.DistributedDataParallel,
// mnist_distributed.py:67).
//
// Layout (owned by parallel/ddp.py): one flat gradient buffer; every parameter
// has a fixed 256-byte aligned slot; slots are grouped into buckets in
// gradient-ready order.  The buffer may start SHORTER than the layout: the big
// layers' weight slots sit at its end and get storage on first use (grow(); at
// world size 1 the fc weight steps inside its backward kernel and never has a
// gradient, so those 720 MB -- 39 GiB at 23000^2 -- are never allocated).  The reducer:
//   * registers a post-hook on each parameter's AccumulateGrad node (C++ autograd,
//     no Python on the backward path),
//   * makes sure param.grad IS the bucket slot (kernels with a gradient sink
//     already wrote there; anything else is copied once and .grad re-pointed),
//   * counts ready parameters per bucket and launches the bucket's AVG all-reduce
//     on the communicator the moment the last one arrives — for the ConvNet the
//     720 MB fc bucket goes out right after the head backward and overlaps the
//     whole conv backward,
//   * queues an end-of-backward callback on the autograd engine that handles
//     unused parameters and orders the caller's stream after every bucket's
//     collective (device-side wait; the host never blocks).
#include <torch/csrc/autograd/engine.h>
#include <torch/csrc/autograd/function.h>
#include <torch/csrc/autograd/function_hook.h>
#include <torch/csrc/autograd/variable.h>
#include <torch/custom_class.h>
#include <torch/library.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <string>
#include <vector>

#include "comm/comm.h"
#include "comm/host_comm.h"
#include "comm/rccl_comm.h"

namespace tds_comm {

class Reducer;

struct ReadyHook : torch::autograd::FunctionPostHook {
  std::weak_ptr<std::atomic<Reducer*>> owner;
  int64_t index;
  ReadyHook(std::weak_ptr<std::atomic<Reducer*>> o, int64_t i) : owner(std::move(o)), index(i) {}
  torch::autograd::variable_list operator()(const torch::autograd::variable_list& outputs,
                                            const torch::autograd::variable_list& inputs) override;
};

class Reducer : public torch::CustomClassHolder {
 public:
  // param_slots: int64 [P, 3] = (offset, numel, bucket); bucket_slots: int64 [B, 2] = (offset, numel)
  Reducer(at::Tensor flat_grad, at::Tensor param_slots, at::Tensor bucket_slots, bool find_unused)
      : flat_grad_(flat_grad), find_unused_(find_unused), self_(std::make_shared<std::atomic<Reducer*>>(this)) {
    TORCH_CHECK(flat_grad.dim() == 1 && flat_grad.is_contiguous(), "Reducer: flat_grad must be a 1-D buffer");
    auto ps = param_slots.to(at::kLong).contiguous().cpu();
    auto bs = bucket_slots.to(at::kLong).contiguous().cpu();
    TORCH_CHECK(ps.dim() == 2 && ps.size(1) == 3 && bs.dim() == 2 && bs.size(1) == 2, "Reducer: bad slot tables");
    for (int64_t i = 0; i < ps.size(0); ++i) {
      const int64_t* r = ps.data_ptr<int64_t>() + 3 * i;
      p_off_.push_back(r[0]);
      p_num_.push_back(r[1]);
      p_bucket_.push_back(r[2]);
    }
    for (int64_t b = 0; b < bs.size(0); ++b) {
      const int64_t* r = bs.data_ptr<int64_t>() + 2 * b;
      b_off_.push_back(r[0]);
      b_num_.push_back(r[1]);
    }
    b_count_.assign(b_off_.size(), 0);
    for (int64_t bk : p_bucket_) {
      TORCH_CHECK(bk >= 0 && bk < (int64_t)b_off_.size(), "Reducer: param bucket out of range");
      ++b_count_[bk];
    }
    pending_ = b_count_;
    for (size_t i = 0; i < p_off_.size(); ++i) total_ = std::max(total_, p_off_[i] + p_num_[i]);
    for (size_t b = 0; b < b_off_.size(); ++b) total_ = std::max(total_, b_off_[b] + b_num_[b]);
    TORCH_CHECK(flat_grad.numel() <= total_, "Reducer: flat_grad longer than the slot layout");
    b_ready_.assign(b_off_.size(), false);
    b_skip_.assign(b_off_.size(), false);
    b_defer_.assign(b_off_.size(), false);
    works_.resize(b_off_.size());
    taken_.resize(b_off_.size());
  }

  ~Reducer() override {
    self_->store(nullptr);
    detach();
  }

  void set_rccl_comm(c10::intrusive_ptr<RcclComm> c) {
    rccl_ = c;
    comm_ = rccl_.get();
  }
  void set_host_comm(c10::intrusive_ptr<HostComm> c) {
    host_ = c;
    comm_ = host_.get();
  }

  // Register the AccumulateGrad post-hooks.  params[i] matches param_slots row i.
  void attach(std::vector<at::Tensor> params) {
    TORCH_CHECK(params.size() == p_off_.size(), "Reducer.attach: expected ", p_off_.size(), " params");
    detach();
    params_ = params;
    for (size_t i = 0; i < params_.size(); ++i) {
      TORCH_CHECK(params_[i].requires_grad(), "Reducer.attach: parameter ", i, " does not require grad");
      auto acc = torch::autograd::impl::grad_accumulator(params_[i]);
      TORCH_CHECK(acc, "Reducer.attach: no grad accumulator for parameter ", i);
      keys_.push_back(acc->add_post_hook(std::make_unique<ReadyHook>(self_, (int64_t)i)));
      accs_.push_back(acc);  // keep the AccumulateGrad nodes alive (torch's reducer does the same)
    }
  }

  void detach() {
    for (size_t i = 0; i < accs_.size(); ++i) accs_[i]->del_post_hook(keys_[i]);
    accs_.clear();
    keys_.clear();
  }

  // Called by the DDP forward: arm the per-bucket counters for the next backward.
  void prepare_for_backward(bool sync) {
    sync_ = sync;
    pending_ = b_count_;
    std::fill(b_ready_.begin(), b_ready_.end(), false);
    for (auto& w : works_) w.reset();
    callback_queued_ = false;
    ready_order_.clear();
  }

  // A skipped bucket's gradients are produced outside the hook/all-reduce path this
  // step (DDP's activation exchange, parallel/factored.py): no hooks are expected,
  // no all-reduce is launched.
  void set_bucket_skip(int64_t b, bool skip) {
    TORCH_CHECK(b >= 0 && b < (int64_t)b_skip_.size(), "Reducer.set_bucket_skip: bad bucket");
    b_skip_[b] = skip;
  }

  // A deferred bucket's collective is NOT waited at the end of backward; DDP takes
  // the work (take_work) and finishes it on a side stream together with the
  // optimizer update of that bucket (DistributedDataParallel(overlap_optimizer=True)).
  void set_bucket_deferred(int64_t b, bool deferred) {
    TORCH_CHECK(b >= 0 && b < (int64_t)b_defer_.size(), "Reducer.set_bucket_deferred: bad bucket");
    b_defer_[b] = deferred;
  }

  c10::optional<c10::intrusive_ptr<CommWork>> take_work(int64_t b) {
    TORCH_CHECK(b >= 0 && b < (int64_t)taken_.size(), "Reducer.take_work: bad bucket");
    auto w = taken_[b];
    taken_[b].reset();
    if (!w) return c10::nullopt;
    return w;
  }

  // The buffer as it is now (parallel/ddp.py reads it back after a grow()).
  at::Tensor flat_grad() const { return flat_grad_; }
  int64_t layout_numel() const { return total_; }

  // Give the whole layout storage: a new buffer, the resident prefix copied over, every
  // .grad that was a view of the old buffer re-pointed.  Collectives in flight on the old
  // buffer (in place) are ordered before the copy first.  The old buffer is kept alive:
  // a collective queued on the comm stream may still read it.
  void grow() {
    if (flat_grad_.numel() >= total_) return;
    for (auto& w : works_)
      if (w) w->wait();
    at::NoGradGuard ng;
    at::Tensor g = at::zeros({total_}, flat_grad_.options());
    if (flat_grad_.numel() > 0) g.narrow(0, 0, flat_grad_.numel()).copy_(flat_grad_);
    for (size_t i = 0; i < params_.size(); ++i) {
      at::Tensor& pg = params_[i].mutable_grad();
      if (pg.defined() && pg.storage().is_alias_of(flat_grad_.storage()))
        pg = g.narrow(0, p_off_[i], p_num_[i]).view(params_[i].sizes());
    }
    retired_.push_back(flat_grad_);
    flat_grad_ = g;
  }

  at::Tensor slot(int64_t i) {
    if (p_off_[i] + p_num_[i] > flat_grad_.numel()) grow();
    return flat_grad_.narrow(0, p_off_[i], p_num_[i]);
  }

  void on_ready(int64_t i) {
    auto& p = params_[i];
    at::Tensor& g = p.mutable_grad();
    if (!g.defined()) return;
    at::Tensor view = slot(i);
    if (g.data_ptr() != view.data_ptr() || !g.is_contiguous()) {
      // producer without a gradient sink: one copy into the slot, then .grad IS the slot
      at::NoGradGuard ng;
      view.copy_(g.reshape({-1}));
      g = view.view(p.sizes());
    }
    count_ready(i);
  }

  // A parameter whose optimizer step ran inside its backward kernel without materialising
  // the gradient (ops/fused_update.py, optimizer-in-backward semantics): ready, no .grad.
  void mark_ready(int64_t i) {
    TORCH_CHECK(i >= 0 && i < (int64_t)p_bucket_.size(), "Reducer.mark_ready: bad parameter index");
    count_ready(i);
  }

  void count_ready(int64_t i) {
    if (!callback_queued_) {
      callback_queued_ = true;
      std::weak_ptr<std::atomic<Reducer*>> w = self_;
      torch::autograd::Engine::get_default_engine().queue_callback([w] {
        if (auto s = w.lock())
          if (Reducer* r = s->load()) r->finalize();
      });
    }
    const int64_t b = p_bucket_[i];
    if (b_skip_[b]) return;
    if (--pending_[b] == 0) launch(b);
  }

  void finalize() {
    for (size_t b = 0; b < b_off_.size(); ++b) {
      if (b_ready_[b] || b_skip_[b]) continue;
      std::vector<int64_t> missing;
      for (size_t i = 0; i < params_.size(); ++i)
        if (p_bucket_[i] == (int64_t)b && !params_[i].grad().defined()) missing.push_back((int64_t)i);
      if (!find_unused_) {
        TORCH_CHECK(false, "DistributedDataParallel: bucket ", b, " never became ready (", missing.size(),
                    " parameters got no gradient); pass find_unused_parameters=True if parts of the model are unused");
      }
      at::NoGradGuard ng;
      for (int64_t i : missing) {
        at::Tensor v = slot(i);
        v.zero_();
        params_[i].mutable_grad() = v.view(params_[i].sizes());
      }
      launch((int64_t)b);
    }
    for (size_t b = 0; b < works_.size(); ++b) {
      auto& w = works_[b];
      if (w && b_defer_[b]) {
        taken_[b] = w;  // finished later on DDP's side stream
      } else if (w) {
        w->wait();  // caller stream waits on the collective (device-side)
      }
      w.reset();
    }
    callback_queued_ = false;
  }

  std::vector<int64_t> ready_order() const { return ready_order_; }
  int64_t num_buckets() const { return (int64_t)b_off_.size(); }

 private:
  at::Tensor flat_grad_;
  std::vector<at::Tensor> retired_;  // buffers replaced by grow()
  int64_t total_ = 0;                // elements of the whole slot layout
  bool find_unused_;
  std::shared_ptr<std::atomic<Reducer*>> self_;
  std::vector<int64_t> p_off_, p_num_, p_bucket_, b_off_, b_num_, b_count_, pending_, ready_order_;
  std::vector<bool> b_ready_, b_skip_, b_defer_;
  std::vector<c10::intrusive_ptr<CommWork>> works_, taken_;
  std::vector<at::Tensor> params_;
  std::vector<std::shared_ptr<torch::autograd::Node>> accs_;
  std::vector<uintptr_t> keys_;
  CollectiveComm* comm_ = nullptr;
  c10::intrusive_ptr<RcclComm> rccl_;
  c10::intrusive_ptr<HostComm> host_;
  bool sync_ = true;
  bool callback_queued_ = false;

  void launch(int64_t b) {
    b_ready_[b] = true;
    ready_order_.push_back(b);
    if (!sync_ || comm_ == nullptr || comm_->comm_world() == 1) return;
    if (b_off_[b] + b_num_[b] > flat_grad_.numel()) grow();
    works_[b] = comm_->allreduce_async(flat_grad_.narrow(0, b_off_[b], b_num_[b]), R_AVG);
  }
};

torch::autograd::variable_list ReadyHook::operator()(const torch::autograd::variable_list& outputs,
                                                     const torch::autograd::variable_list& /*inputs*/) {
  if (auto s = owner.lock())
    if (Reducer* r = s->load()) r->on_ready(index);
  return outputs;
}

}  // namespace tds_comm

TORCH_LIBRARY_FRAGMENT(tdsa, m) {
  m.class_<tds_comm::Reducer>("Reducer")
      .def(torch::init<at::Tensor, at::Tensor, at::Tensor, bool>())
      .def("set_rccl_comm", &tds_comm::Reducer::set_rccl_comm)
      .def("set_host_comm", &tds_comm::Reducer::set_host_comm)
      .def("attach", &tds_comm::Reducer::attach)
      .def("detach", &tds_comm::Reducer::detach)
      .def("prepare_for_backward", &tds_comm::Reducer::prepare_for_backward)
      .def("finalize", &tds_comm::Reducer::finalize)
      .def("set_bucket_skip", &tds_comm::Reducer::set_bucket_skip)
      .def("set_bucket_deferred", &tds_comm::Reducer::set_bucket_deferred)
      .def("take_work", &tds_comm::Reducer::take_work)
      .def("mark_ready", &tds_comm::Reducer::mark_ready)
      .def("ready_order", &tds_comm::Reducer::ready_order)
      .def("num_buckets", &tds_comm::Reducer::num_buckets)
      .def("flat_grad", &tds_comm::Reducer::flat_grad)
      .def("layout_numel", &tds_comm::Reducer::layout_numel)
      .def("grow", &tds_comm::Reducer::grow)
      .def("slot", &tds_comm::Reducer::slot);
}
