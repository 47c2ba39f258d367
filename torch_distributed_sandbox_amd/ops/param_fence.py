"""Parameter fences: let an update of a parameter run elsewhere and make only the first
reader of that parameter wait for it.

``DistributedDataParallel(overlap_optimizer=True)`` finishes the fc layer's gradient
collective and its SGD update off the critical path while the next step's convolution
forward runs; the fused head / Linear forward calls :func:`wait` on the fc weight before
reading it.  A fence is a list of

* events (an update queued on a side stream: the current stream waits for it on the device,
  the host never blocks), and
* deferred updates (:func:`defer`: a callable that queues the update itself on the current
  stream when the parameter is first needed -- the fc gradient exchange's weight update,
  parallel/factored.py, which then runs on the whole GPU right before the head forward
  instead of competing with the backward's persistent kernels),

processed in the order they were added.
"""
from __future__ import annotations

import torch

_ATTR = "_tds_param_fence"


def _fences(param):
    f = getattr(param, _ATTR, None)
    if f is None:
        f = []
        setattr(param, _ATTR, f)
    return f


def set(param: torch.Tensor, event) -> None:  # noqa: A001 - mirrors a setter
    """Readers of ``param`` wait for ``event`` (after anything fenced before it)."""
    _fences(param).append(("event", event))


def defer(param: torch.Tensor, fn) -> None:
    """``fn()`` queues a pending update of ``param`` on the current stream; it runs once, at the
    first :func:`wait` on ``param``."""
    _fences(param).append(("fn", fn))


def wait(param) -> None:
    """Order the current stream after every pending update of ``param`` (running the deferred
    ones on it)."""
    if param is None:
        return
    f = getattr(param, _ATTR, None)
    if not f:
        return
    delattr(param, _ATTR)
    cur = torch.cuda.current_stream(param.device) if param.is_cuda else None
    for kind, v in f:
        if kind == "fn":
            v()
        elif cur is not None:
            cur.wait_event(v)


def take(param, kind: str):
    """The pending deferred update of ``param`` if it is its ONLY deferred item and offers the form
    ``kind`` (its ``fused_kind`` attribute), removed from the fence -- the caller runs it (the fused
    head forward runs the activation exchange's grouped update range by range,
    parallel/factored.py ``_Update.run_until``); else None and the fence is unchanged.  Events stay
    in the fence for the caller's :func:`wait` (under DDP's overlapped optimizer the end-of-backward
    side-stream step fences every parameter of its bucket, this one included)."""
    f = getattr(param, _ATTR, None) if param is not None else None
    if not f:
        return None
    fns = [i for i, (k, _) in enumerate(f) if k == "fn"]
    if len(fns) != 1 or getattr(f[fns[0]][1], "fused_kind", None) != kind:
        return None
    fn = f.pop(fns[0])[1]
    if not f:
        delattr(param, _ATTR)
    return fn


def pending(param) -> bool:
    return bool(getattr(param, _ATTR, None))
