"""Compute/communication CU split for overlapped collectives.

RCCL's kernels need CUs to make progress; this package's persistent conv kernels take one
workgroup per CU for their whole run, so a collective issued under them (the fc bucket
all-reduce or the chunked all-reduce of the head backward, overlapping the conv2 backward)
waits for free CUs.  ``reserve_cus_for_comm(n)`` keeps ``n`` CUs out of the compute: it
returns a CU-masked stream (``hipExtStreamCreateWithCUMask``, csrc/kernels/cu_budget.hip) for
the training step and makes the persistent kernels size their grids to the remaining CUs.
The RCCL side is bounded with ``TDS_RCCL_MIN_CTAS`` / ``TDS_RCCL_MAX_CTAS`` (the communicator's
``ncclConfig_t`` minCTAs / maxCTAs, csrc/comm/rccl_comm.h); ``bench.py --reserve-cus N
--rccl-max-ctas M`` sets both.  Off by default (n = 0).
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import _ext


def reserve_cus_for_comm(n: int, device: Optional[torch.device] = None) -> Optional[torch.cuda.Stream]:
    """Reserve ``n`` CUs (a multiple of 8: n/8 per XCD) for communication kernels; returns the
    CU-masked compute stream (None and no change when ``n`` is 0).  Create it before the model
    and DDP, and make it current for the whole training loop (autograd's accumulation nodes
    remember the stream they were created on)."""
    ops = _ext.ops()
    n = int(n)
    if n % 8:
        raise ValueError(f"reserve_cus_for_comm: n must be a multiple of 8 (n/8 CUs per XCD), got {n}")
    if n <= 0:
        ops.set_cu_reserve(0)
        return None
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    handle = ops.cu_masked_stream(dev.index, n)
    ops.set_cu_reserve(n)
    return torch.cuda.ExternalStream(handle, device=dev)


def compute_cus() -> int:
    """CUs the persistent kernels launch on (all minus the reserve)."""
    return int(_ext.ops().device_cus())
