"""Activation exchange: exact data-parallel gradients for a huge, skinny Linear
layer without all-reducing its weight gradient.

Data parallelism averages ``dW = dYᵀX`` over ranks.  The reference's DDP
(mnist_distributed.py:67) all-reduces the full gradient: for the 3000² ConvNet's
fc layer that is 720 MB per step for a matrix of rank ≤ 5
per rank.  Over xGMI — point-to-point links of ≈77 GB/s per direction — a ring
all-reduce moves ``2(W-1)/W × 720 MB`` per GPU, which at W = 2 means ≈9 ms on
the single link joining the pair: more than the whole compute step.

The same average can be formed from the factors: each rank contributes its
``B`` input rows ``X_r`` and output gradients ``dY_r``, and every rank computes
``dW = (1/W) Σ_r dY_rᵀ X_r`` locally (one skinny GEMM with ``W·B`` rows).  That
moves ``(W-1) × B × in × 4`` bytes per rank instead — 360 MB instead of 720 MB
at W = 2 — and the exchange can start as soon as the FORWARD has produced
``X_r``, so it overlaps the entire backward instead of only the part after the
fc gradient exists.  Per rank the bytes favour the exchange when
``B·W ≤ 2·out_features`` (W = 2, 3, 4 for the ConvNet: B = 5, 10 classes; at
equal bytes the exchange still wins because it starts a whole backward earlier);
at larger W the ring all-reduce is cheaper and is used.

The result is the same average DDP produces (floating-point summation order
differs, as it does between all-reduce algorithms), identical on every rank.

Protocol (driven by ``parallel/ddp.py``):

* ``arm(sync)`` each DDP forward: the exchange may run this step.
* the layer's forward calls ``begin(x)``; if the exchange is worthwhile it
  starts an async all-gather of ``x`` and tells DDP to leave this layer's bucket
  out of the bucket all-reduce; the layer then returns no weight/bias gradient.
* the layer's backward calls ``defer(dy)``: ``dy`` is kept and a callback is
  queued on the autograd engine.
* at the end of backward the callback all-gathers ``dy`` (a few hundred bytes),
  waits for ``x`` and writes ``dW``/``db`` straight into the bucket slots
  (``ops.linear_dw`` on the GPU: exact-fp32 MFMA, memory-bound).  Gradients
  accumulated locally under ``no_sync()`` are averaged with one all-reduce and
  this step's exchanged average is added, matching DDP's accumulation semantics.
"""
from __future__ import annotations

from typing import Optional

import torch

_ATTR = "_tds_activation_exchange"


def get(weight) -> Optional["ActivationExchange"]:
    return getattr(weight, _ATTR, None) if weight is not None else None


class ActivationExchange:
    def __init__(self, weight: torch.nn.Parameter, bias: Optional[torch.nn.Parameter], group, world: int,
                 mode: str, set_skip, weight_view, bias_view):
        if mode not in ("auto", "activations"):
            raise ValueError(f"ActivationExchange mode must be auto|activations, got {mode!r}")
        self.weight, self.bias = weight, bias
        self.group, self.world, self.mode = group, world, mode
        self._set_skip, self._wview, self._bview = set_skip, weight_view, bias_view
        self.armed = False
        self.active = False
        self.steps_exchanged = 0
        self.last_path = None  # "activation-exchange" once a step used it
        self._x_all = self._x_work = self._dy = None
        self.side_stream = None  # set by DDP(overlap_optimizer=True): dW is formed off the compute stream
        setattr(weight, _ATTR, self)

    def detach(self):
        if getattr(self.weight, _ATTR, None) is self:
            delattr(self.weight, _ATTR)

    # ---------------------------------------------------------------- policy
    def worthwhile(self, rows: int) -> bool:
        if self.mode == "activations":
            return True
        out_f = self.weight.shape[0]
        # equal bytes (B*W == 2*out) still favour the exchange: it starts a whole backward earlier
        return self.world > 1 and rows * self.world <= 2 * out_f

    def arm(self, sync: bool):
        self.armed = bool(sync)
        self.active = False
        self._set_skip(False)

    # ---------------------------------------------------------------- forward
    def _eligible(self, rows: int) -> bool:
        if not self.armed or self.active:
            return False
        return self.worthwhile(rows)

    def ready(self, rows: int) -> bool:
        """Would a forward with ``rows`` input rows (grad mode on) run the exchange?"""
        return torch.is_grad_enabled() and self._eligible(rows)

    def begin(self, x2d: torch.Tensor) -> bool:
        """Called from the layer's forward (possibly inside an autograd Function,
        i.e. under no_grad) with its [rows, in] input."""
        if not self._eligible(x2d.shape[0]):
            return False
        from . import distributed as tdist

        x2d = x2d.detach().contiguous()
        self._x_all = torch.empty((self.world * x2d.shape[0], x2d.shape[1]), device=x2d.device, dtype=x2d.dtype)
        self._x_work = tdist.all_gather_into_tensor(self._x_all, x2d, group=self.group, async_op=True)
        self._x_local = x2d  # keep alive until the gather completes
        self.active = True
        self._set_skip(True)
        return True

    # ---------------------------------------------------------------- backward
    def defer(self, dy: torch.Tensor):
        self._dy = dy.detach().contiguous()
        torch.autograd.Variable._execution_engine.queue_callback(self.finalize)

    def finalize(self):
        side = self.side_stream if (self.side_stream is not None and self._dy.is_cuda) else None
        if side is None:
            self._finish()
            return
        # the dy gather queues behind the big x gather on the comm stream: issue both
        # waits and the dW GEMM from the side stream so the compute stream runs on
        cur = torch.cuda.current_stream(self._dy.device)
        side.wait_stream(cur)
        keep = (self._dy, self._x_all, self._x_local)  # used on the side stream
        with torch.cuda.stream(side):
            for t in keep:
                t.record_stream(side)
            self._finish()

    def _finish(self):
        from .. import _ext
        from . import distributed as tdist

        dy = self._dy
        rows = dy.shape[0]
        dy_all = torch.empty((self.world * rows, dy.shape[1]), device=dy.device, dtype=dy.dtype)
        tdist.all_gather_into_tensor(dy_all, dy, group=self.group)
        self._x_work.wait()
        x_all = self._x_all
        scale = 1.0 / self.world
        with torch.no_grad():
            # gradients accumulated locally under no_sync() are averaged as they are
            # (one all-reduce), then this step's exchanged average is added
            grads = []
            for p, view_fn in ((self.weight, self._wview), (self.bias, self._bview)):
                if p is None:
                    grads.append(None)
                    continue
                if p.grad is not None:
                    tdist.all_reduce(p.grad, tdist.ReduceOp.AVG, group=self.group)
                    grads.append((p.grad, True))
                else:
                    grads.append((view_fn(), False))
            (dw, acc_w) = grads[0]
            db, acc_b = grads[1] if grads[1] is not None else (None, False)
            if dy.is_cuda and acc_w == acc_b:
                _ext.ops().linear_dw(dy_all, x_all, dw, db, scale, acc_w)
            else:
                upd = torch.mm(dy_all.t(), x_all).mul_(scale)
                dw.add_(upd) if acc_w else dw.copy_(upd)
                if db is not None:
                    s_b = dy_all.sum(0).mul_(scale)
                    db.add_(s_b) if acc_b else db.copy_(s_b)
        self.weight.grad = dw
        if self.bias is not None:
            self.bias.grad = db
        self._x_all = self._x_work = self._dy = self._x_local = None
        self.active = False
        self.steps_exchanged += 1
        self.last_path = "activation-exchange"
