"""ops/param_fence.py on the CPU: deferred updates run once at the first wait, and the fused head
forward's take() hands over the single deferred update while leaving any events for wait()."""
import torch

from torch_distributed_sandbox_amd.ops import param_fence


class _Upd:
    fused_kind = "groups"

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
    # update over
    p = torch.zeros(3)
    log = []
    upd = _Upd(log)
    param_fence.defer(p, upd)
    param_fence.set(p, "side-stream event")
    assert param_fence.take(p, "groups") is upd
    assert param_fence.pending(p)  # the event is still there for wait()
    param_fence.wait(p)
    assert not param_fence.pending(p) and log == []


def test_take_refuses_other_kinds_and_two_updates():
    p = torch.zeros(3)
    log = []
    param_fence.defer(p, _Upd(log))
    assert param_fence.take(p, "other") is None
    param_fence.defer(p, _Upd(log))
    assert param_fence.take(p, "groups") is None  # two deferred updates: run in order by wait()
    param_fence.wait(p)
    assert log == ["ran", "ran"]
    assert param_fence.take(None, "groups") is None


def _deferred_ddp(monkeypatch):
    """A CPU DDP over the ConvNet with its fc bucket deferred as DistributedDataParallel(
    overlap_optimizer=True) sets it up on the GPU, with the stream / event calls of
    _run_deferred_update replaced by recorders."""
    import contextlib

    from torch_distributed_sandbox_amd.models import ConvNet
    from torch_distributed_sandbox_amd.parallel import DistributedDataParallel

    class _Stream:
        def __init__(self):
            self.waits = 0

        def wait_stream(self, other):
            self.waits += 1

    class _Event:
        def record(self, stream=None):
            pass

    monkeypatch.setattr(torch.cuda, "current_stream", lambda device=None: _Stream())
    monkeypatch.setattr(torch.cuda, "stream", lambda s: contextlib.nullcontext())
    monkeypatch.setattr(torch.cuda, "Event", _Event)
    torch.manual_seed(0)
    m = ConvNet(image_shape=(256, 256))  # fc 10 x 131072: an exchange-candidate (deferred) layer
    ddp = DistributedDataParallel(m)
    ddp._side = _Stream()
    ddp._deferred = [ddp._layer_bucket[id(m.fc)]]
    return m, ddp


def test_inline_deferred_fast_path_steps_bias_once_and_sets_no_fence(monkeypatch):
    """World size 1, the fc weight stepped inside its backward (fused update): the optimizer takes
    the bias into its own sweep (take_inline_deferred), and the deferred runner then has nothing
    left -- no side-stream work, no parameter fence (parallel/ddp.py _run_deferred_update)."""
    m, ddp = _deferred_ddp(monkeypatch)
    ddp._fused_done = {id(m.fc.weight)}
    ranges = ddp.take_inline_deferred()
    assert ranges == [ddp._slots[id(m.fc.bias)]]
    calls = []
    ddp._run_deferred_update(lambda off, n: calls.append((off, n)))
    assert calls == [] and ddp.last_deferred_inline
    assert ddp._side.waits == 0
    assert not param_fence.pending(m.fc.weight) and not param_fence.pending(m.fc.bias)
    assert ddp._fused_done == set() and ddp._inline_done == set()  # state consumed for the next step


def test_inline_deferred_falls_back_when_weight_was_not_fused(monkeypatch):
    """A step whose fc weight was NOT updated in its backward (e.g. no fused kernel ran): nothing is
    taken inline, the runner updates the whole bucket on the side stream and fences both params."""
    m, ddp = _deferred_ddp(monkeypatch)
    ddp._fused_done = set()
    assert ddp.take_inline_deferred() == []
    calls = []
    ddp._run_deferred_update(lambda off, n: calls.append((off, n)))
    b = ddp._layer_bucket[id(m.fc)]
    assert calls == [(b.offset, b.numel)] and not ddp.last_deferred_inline
    assert ddp._side.waits == 1
    assert param_fence.pending(m.fc.weight) and param_fence.pending(m.fc.bias)
    assert ddp.flat_grad.numel() == ddp._total  # the update read the weight's slot: allocated


def test_deferred_runner_without_inline_call_uses_side_stream(monkeypatch):
    """The runner called without a matching take_inline_deferred() this step (another optimizer):
    the bias is updated by the runner itself, the fused weight skipped."""
    m, ddp = _deferred_ddp(monkeypatch)
    ddp.take_inline_deferred()  # a previous step's call ...
    ddp._run_deferred_update(lambda off, n: None)  # ... consumed there
    ddp._fused_done = {id(m.fc.weight)}
    calls = []
    ddp._run_deferred_update(lambda off, n: calls.append((off, n)))
    assert calls == [ddp._slots[id(m.fc.bias)]] and not ddp.last_deferred_inline
    assert param_fence.pending(m.fc.bias)
