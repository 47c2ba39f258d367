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

import os
from typing import Optional

import torch

from .. import _ext


def mask_layout() -> str:
    """CU-mask bit numbering (csrc/kernels/cu_budget.hip): ``TDS_CU_MASK_LAYOUT`` = striped
    (default) | blocked."""
    v = os.environ.get("TDS_CU_MASK_LAYOUT", "striped").strip().lower()
    if v not in ("striped", "blocked"):
        raise ValueError(f"TDS_CU_MASK_LAYOUT must be striped|blocked, got {v!r}")
    return v


def reserve_cus_for_comm(n: int, device: Optional[torch.device] = None) -> Optional[torch.cuda.Stream]:
    """Reserve ``n`` CUs (a multiple of 32: n/8 per XCD) for communication kernels; returns the
    CU-masked compute stream (None and no change when ``n`` is 0).  Create it before the model
    and DDP, and make it current for the whole training loop (autograd's accumulation nodes
    remember the stream they were created on)."""
    ops = _ext.ops()
    n = int(n)
    if n % 32:
        # n/8 CUs per XCD, and per XCD a multiple of its 4 shader engines: with 2 of an XCD's 32
        # CUs out, two engines keep 7 CUs, the dispatcher still deals the 30 persistent
        # workgroups 8/8/7/7 over the engines from wherever its round-robin stands, and a
        # workgroup waits a whole round (measured at reserve 16: conv2 backward 1.56 -> 3.07 ms,
        # step +60 %; reserve 32: +5 %, tools/gpu_sessions/r2_cuprobe2.sh)
        raise ValueError(f"reserve_cus_for_comm: n must be a multiple of 32 (4 CUs per XCD), got {n}")
    if n <= 0:
        ops.set_cu_reserve(0)
        return None
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    handle = ops.cu_masked_stream(dev.index, n, mask_layout() == "striped")
    ops.set_cu_reserve(n)
    return torch.cuda.ExternalStream(handle, device=dev)


def comm_stream(device: Optional[torch.device] = None) -> Optional[torch.cuda.Stream]:
    """The stream confined to the reserved CUs (what the native RCCL communicator launches on),
    or None when no CUs are reserved."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    h = int(_ext.ops().cu_comm_stream(dev.index))
    return torch.cuda.ExternalStream(h, device=dev) if h else None


def compute_cus() -> int:
    """CUs the persistent kernels launch on (all minus the reserve)."""
    return int(_ext.ops().device_cus())


def side_stream(device: Optional[torch.device] = None, side: Optional[str] = None) -> Optional[torch.cuda.Stream]:
    """A stream for DDP's side work (the fc exchange's dW formation, the deferred SGD step) that
    keeps to one side of the CU split: ``side`` = "any" (a plain stream: None here; default) |
    "comm" (the reserved CUs) | "compute".  ``TDS_SIDE_CUS`` overrides the default.  None when no
    CUs are reserved (then a plain stream is as good as any).

    Measured at world 1 with 32 CUs reserved and the exchange forced (tools/gpu_sessions/
    r3_s3.sh, docs/DISTRIBUTED.md): the 32 reserved CUs are far too few for the exchange's dW
    formation (activations 7.91 ms/step on "comm" vs 5.32 on "any" and 5.31 on "compute";
    sharded 8.44 / 5.25 / 5.11), so the default is a plain stream."""
    side = (side or os.environ.get("TDS_SIDE_CUS", "any")).strip().lower()
    if side not in ("comm", "compute", "any"):
        raise ValueError(f"side stream placement must be comm|compute|any, got {side!r}")
    if side == "any":
        return None
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    h = int(_ext.ops().cu_side_stream(dev.index, side == "comm"))
    return torch.cuda.ExternalStream(h, device=dev) if h else None


def release_streams() -> int:
    """End of a single-process run that used the split: synchronize, make the default stream
    current, and destroy every CU-masked stream (csrc/kernels/cu_budget.hip
    ``tds_cu_release_streams``); the compute reserve returns to 0.  Nothing may use the masked
    streams (or their ExternalStream wrappers) afterwards.  Left to process exit, the runtime's
    teardown of their queues races rocprofiler-sdk's finalization (an exit-time fault under
    rocprofv3 only).  Returns how many streams were destroyed."""
    if not torch.cuda.is_available():
        return 0
    torch.cuda.synchronize()
    torch.cuda.set_stream(torch.cuda.default_stream())
    return int(_ext.ops().cu_release_streams())
