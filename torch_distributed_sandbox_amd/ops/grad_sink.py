"""Gradient sinks: let a backward kernel write a parameter's gradient directly
into its communication bucket.

PyTorch's DDP reducer copies every gradient into a flat bucket (``aten::mul``
by 1/W) and copies it back afterwards.  Here
the DDP wrapper (``parallel/ddp.py``) registers, for each parameter, a
function returning a *fresh view* of that parameter's slot in the bucket.  A
backward that supports sinks computes its weight gradient into that view and
returns it; ``AccumulateGrad`` then steals the (single-reference) view as
``param.grad`` — so the gradient lands in the bucket with zero extra passes.

If ``param.grad`` is already defined (gradient accumulation across
micro-batches), the sink is bypassed and a temporary is returned instead, so
``AccumulateGrad`` adds it into the existing (bucket-view) gradient.
"""
from __future__ import annotations

import torch

_ATTR = "_tds_grad_sink"


def register(param: torch.Tensor, view_fn) -> None:
    setattr(param, _ATTR, view_fn)


def unregister(param: torch.Tensor) -> None:
    if hasattr(param, _ATTR):
        delattr(param, _ATTR)


def acquire(param, shape, like: torch.Tensor):
    """Destination tensor for ``param``'s gradient (bucket view if possible)."""
    if param is None:
        return None
    fn = getattr(param, _ATTR, None)
    if fn is not None and param.grad is None:
        v = fn()
        if v is not None and tuple(v.shape) == tuple(shape):
            return v
    return torch.empty(shape, device=like.device, dtype=like.dtype)
