"""Optimizer step fused into the backward kernel that produces the gradient.

At world size 1 the fc weight's SGD step (``p -= lr * g``, torch.optim.SGD without
momentum / weight decay) needs nothing but ``p`` and ``g`` — and the head backward
(``head_bwd_ya_kernel``) holds both in registers while it writes ``g``.  When DDP
(``parallel/ddp.py``, ``overlap_optimizer=True``) owns that update it registers a
provider here; the head backward asks :func:`take` for the learning rate, applies the
step in the same pass (saving the separate 2.2 GB SGD sweep at 3000²), and DDP's
deferred update then skips the parameter.  The observable difference is that the fc
weight already holds its updated value after ``backward()``, as with
``torch.distributed.optim._apply_optimizer_in_backward``.

Gradient of the updated parameter: by default (``DistributedDataParallel(keep_fused_grads=
False)``) it is not materialised -- ``param.grad`` stays None, the semantics of torch's
optimizer-in-backward -- and the kernel writes only the updated weight (720 MB less HBM
traffic per step at 3000²).  With ``keep_fused_grads=True`` the gradient is also written
to ``param.grad`` (the DDP bucket).
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


def take(param, exchanged: bool = False):
    """Learning rate for an in-backward update of ``param`` this step, or None.

    ``exchanged=False``: asked by the kernel that produces the LOCAL gradient (world size 1
    only).  ``exchanged=True``: asked by the fc gradient exchange (parallel/factored.py), whose
    dW formation already sums every rank's rows, so the averaged step can be applied there at
    any world size."""
    if param is None:
        return None
    fn = getattr(param, _ATTR, None)
    if fn is None:
        return None
    return fn("query_exchange" if exchanged else "query")


def keep_grad(param) -> bool:
    """Whether the gradient of an in-backward update of ``param`` must also be written."""
    fn = getattr(param, _ATTR, None)
    return bool(fn("keep_grad")) if fn is not None else True


def applied(param, grad_written: bool = True) -> None:
    """The backward applied the update: the owner must not apply it again this step.
    ``grad_written=False``: no gradient reached autograd for ``param``; the owner counts the
    parameter as ready itself."""
    fn = getattr(param, _ATTR, None)
    if fn is not None:
        fn("applied" if grad_written else "applied_no_grad")
