"""Parameter fences: let an update of a parameter run on a side stream and make
only the first reader of that parameter wait for it.

``DistributedDataParallel(overlap_optimizer=True)`` finishes the fc layer's
gradient collective and its SGD update on a side stream while the next step's
convolution forward runs on the compute stream; the fused head / Linear forward
calls :func:`wait` on the fc weight before reading it, which orders the
compute stream after the update (a device-side event wait; the host never
blocks).
"""
from __future__ import annotations

import torch

_ATTR = "_tds_param_fence"


def set(param: torch.Tensor, event) -> None:  # noqa: A001 - mirrors a setter
    setattr(param, _ATTR, event)


def wait(param) -> None:
    """Order the current stream after a pending update of ``param`` (if any)."""
    if param is None:
        return
    ev = getattr(param, _ATTR, None)
    if ev is not None:
        torch.cuda.current_stream(param.device).wait_event(ev)
        delattr(param, _ATTR)


def pending(param) -> bool:
    return getattr(param, _ATTR, None) is not None
