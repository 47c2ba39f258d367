"""SGD with a multi-tensor gfx950 kernel (``torch.optim.SGD(params, lr)``, mnist_onegpu.py:49).

One launch updates every parameter (tensor table in the kernel arguments,
SURVEY.md §2.4 K26).  When the parameters live in one flat buffer (as laid
out by ``parallel.ddp.DistributedDataParallel``), the update is a single
contiguous sweep over that buffer and its flat gradient bucket.
"""
from __future__ import annotations

import torch

from .. import _ext


class SGD(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False):
        if lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay, nesterov=nesterov)
        super().__init__(params, defaults)
        self._flat = None  # (flat_param, flat_grad) when installed by DDP
        self._deferred = None  # ([(offset, numel)], runner) when DDP overlaps part of the update
        self._stepped = None  # predicate: parameter already stepped inside its backward (no .grad)

    def set_flat_buffers(self, flat_param: torch.Tensor, flat_grad, params):
        """Declare that ``params`` are views of ``flat_param`` with grads in ``flat_grad`` (a tensor,
        or a callable returning the buffer as it is at step time: DDP allocates the big layers'
        gradient slots at the buffer's end on first use, parallel/ddp.py ``_lazy_from``)."""
        ids = {id(p) for g in self.param_groups for p in g["params"]}
        if ids == {id(p) for p in params} and len(self.param_groups) == 1:
            self._flat = (flat_param, flat_grad, list(params))
        else:
            self._flat = None

    def set_deferred(self, ranges, runner, stepped=None):
        """DDP(overlap_optimizer=True): the flat ranges in ``ranges`` are updated by
        ``runner(update_fn)`` on DDP's side stream; the rest here, on the current stream.
        ``stepped(p)``: True for a parameter whose update already ran inside its backward
        kernel without a gradient (ops/fused_update.py); the runner skips it."""
        self._deferred = (sorted(ranges), runner) if ranges else None
        self._stepped = stepped

    def _flat_grad(self):
        fg = self._flat[1]
        return fg() if callable(fg) else fg

    def _flat_ok(self):
        if self._flat is None:
            return False
        fp, _, params = self._flat
        fg = self._flat_grad()
        if self._deferred is None and fg.numel() != fp.numel():
            return False  # (a gradient slot never allocated: no single sweep)
        for p in params:
            if p.grad is None:
                if self._deferred is not None and self._stepped is not None and self._stepped(p):
                    continue
                return False
            # grads must still be views of the flat bucket
            if p.grad.untyped_storage().data_ptr() != fg.untyped_storage().data_ptr():
                return False
        return True

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            lr, mom, damp = group["lr"], group["momentum"], group["dampening"]
            wd, nest = group["weight_decay"], group["nesterov"]
            if (self._flat is not None and mom == 0.0 and wd == 0.0 and self._flat_ok() and self._flat[0].is_cuda):
                fp, fg = self._flat[0], self._flat_grad()
                if self._deferred is None:
                    _ext.ops().sgd_step_([fp], [fg], [], lr, 0.0, 0.0, 0.0, False, False)
                    continue
                ranges, runner = self._deferred
                ps, gs, pos = [], [], 0
                for off, n in ranges + [(fp.numel(), 0)]:
                    if off > pos:
                        ps.append(fp[pos:off])
                        gs.append(fg[pos:off])
                    pos = off + n
                # small leftovers of the deferred ranges the owner wants stepped here, in this sweep
                owner = getattr(runner, "__self__", None)
                for off, n in (owner.take_inline_deferred() if hasattr(owner, "take_inline_deferred") else []):
                    ps.append(fp[off:off + n])
                    gs.append(fg[off:off + n])
                if ps:
                    _ext.ops().sgd_step_(ps, gs, [], lr, 0.0, 0.0, 0.0, False, False)
                runner(lambda off, n, _lr=lr: _ext.ops().sgd_step_([fp[off:off + n]], [self._flat_grad()[off:off + n]],
                                                                   [], _lr, 0.0, 0.0, 0.0, False, False))
                continue
            params, grads, bufs, first = [], [], [], False
            for p in group["params"]:
                if p.grad is None:
                    continue
                params.append(p)
                grads.append(p.grad)
                if mom != 0.0:
                    st = self.state[p]
                    if "momentum_buffer" not in st:
                        st["momentum_buffer"] = torch.zeros_like(p)
                        first = True
                    bufs.append(st["momentum_buffer"])
            if not params:
                continue
            if params[0].is_cuda:
                ok = all(p.is_contiguous() and g.is_contiguous() and p.dtype == torch.float32 for p, g in
                         zip(params, grads))
                if ok:
                    _ext.ops().sgd_step_(params, grads, bufs, lr, wd, mom, damp, nest, first)
                    continue
            # CPU / non-contiguous reference path (torch.optim.SGD semantics)
            for i, p in enumerate(params):
                d = grads[i]
                if wd != 0.0:
                    d = d.add(p, alpha=wd)
                if mom != 0.0:
                    b = bufs[i]
                    if first:
                        b.copy_(d)
                    else:
                        b.mul_(mom).add_(d, alpha=1.0 - damp)
                    d = d.add(b, alpha=mom) if nest else b
                p.add_(d, alpha=-lr)
        return loss
