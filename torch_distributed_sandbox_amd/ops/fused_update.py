"""Optimizer step fused into the backward kernel that produces the gradient.

At world size 1 the fc weight's SGD step (``p -= lr * g``, torch.optim.SGD without
momentum / weight decay) needs nothing but ``p`` and ``g`` — and the head backward
(``head_bwd_ya_kernel``) holds both in registers while it writes ``g``.  When DDP
(``parallel/ddp.py``, ``overlap_optimizer=True``) owns that update it registers a
provider here; the head backward asks :func:`take` for the learning rate, applies the
step in the same pass (saving the separate 2.2 GB SGD sweep at 3000²), and DDP's
deferred update then skips the parameter.  The gradient is still written to
``param.grad`` (the DDP bucket), so ``.grad`` semantics are unchanged; the observable
difference is that the fc weight already holds its updated value after ``backward()``
(as with ``torch.distributed.optim._apply_optimizer_in_backward``).
"""
from __future__ import annotations

_ATTR = "_tds_fused_update"


def register(param, provider) -> None:
    """``provider("query")`` returns the learning rate to apply now (or None);
    ``provider("applied")`` records that the backward applied it."""
    setattr(param, _ATTR, provider)


def unregister(param) -> None:
    if hasattr(param, _ATTR):
        delattr(param, _ATTR)


def take(param):
    """Learning rate for an in-backward update of ``param`` this step, or None."""
    if param is None:
        return None
    fn = getattr(param, _ATTR, None)
    return fn("query") if fn is not None else None


def applied(param) -> None:
    """The backward applied the update: the owner must not apply it again this step."""
    fn = getattr(param, _ATTR, None)
    if fn is not None:
        fn("applied")
