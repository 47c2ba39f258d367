"""ops/param_fence.py on the CPU: deferred updates run once at the first wait, and the fused head
forward's take() hands over the single deferred update while leaving any events for wait()."""
import torch

from torch_distributed_sandbox_amd.ops import param_fence


class _Upd:
    fused_kind = "zs_head"

    def __init__(self, log):
        self.log = log

    def __call__(self):
        self.log.append("ran")


def test_wait_runs_deferred_once():
    p = torch.zeros(3)
    log = []
    param_fence.defer(p, _Upd(log))
    assert param_fence.pending(p)
    param_fence.wait(p)
    param_fence.wait(p)
    assert log == ["ran"] and not param_fence.pending(p)


def test_take_leaves_events_for_wait():
    # DDP's overlapped optimizer fences every parameter of the deferred bucket with the side
    # stream's event after the exchange deferred the weight's update: take() must still hand the
    # update over (r5_s7: it returned None and the update ran as a separate sweep)
    p = torch.zeros(3)
    log = []
    upd = _Upd(log)
    param_fence.defer(p, upd)
    param_fence.set(p, "side-stream event")
    assert param_fence.take(p, "zs_head") is upd
    assert param_fence.pending(p)  # the event is still there for wait()
    param_fence.wait(p)
    assert not param_fence.pending(p) and log == []


def test_take_refuses_other_kinds_and_two_updates():
    p = torch.zeros(3)
    log = []
    param_fence.defer(p, _Upd(log))
    assert param_fence.take(p, "other") is None
    param_fence.defer(p, _Upd(log))
    assert param_fence.take(p, "zs_head") is None  # two deferred updates: run in order by wait()
    param_fence.wait(p)
    assert log == ["ran", "ran"]
    assert param_fence.take(None, "zs_head") is None
