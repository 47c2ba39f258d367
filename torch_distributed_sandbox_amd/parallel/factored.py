"""Exact data-parallel gradients for a huge, skinny Linear layer without a plain
all-reduce of its weight gradient.

Data parallelism averages ``dW = dYᵀX`` over ranks.  The reference's DDP
(mnist_distributed.py:67) all-reduces the full gradient: for the 3000² ConvNet's
fc layer that is 720 MB per step for a matrix of rank ≤ B
per rank.  The gradient can instead be formed from its factors — each rank's
fc input rows ``X_r`` [B, K] and output gradients ``dY_r`` [B, N] — and the
factors can be exchanged in two ways:

``activations``  all-gather X (and dY); every rank forms the whole averaged dW
                 locally (one skinny GEMM with W·B rows, ``ops.linear_dw``).
``sharded``      K is split into W contiguous column shards.  An all-to-all
                 sends each rank's X columns of shard s to rank s, which forms
                 ``dW[:, shard s]`` from every rank's rows; an all-gather of the
                 shards (grouped point-to-point, one xGMI link per peer pair)
                 then gives every rank the full averaged gradient.

Bytes each rank puts on each of its W-1 links per step (fully connected xGMI,
one link per peer pair; B rows, N outputs, K inputs, 4-byte floats):

    all-reduce (ring/tree)      2·N·K/W
    activations                 B·K
    sharded                     (B + N)·K/W

For the ConvNet (B = 5, N = 10, K = 18e6: 360 MB of X per rank, 720 MB of dW):
W = 2 → 720 / 360 / 540 MB;  W = 4 → 360 / 360 / 270 MB;  W = 8 → 180 / 360 / 135 MB.
``auto`` takes the cheapest, preferring ``activations`` on a tie (one phase, it
starts as soon as the forward has produced X).  Both exchanges start in the
forward, so they overlap the whole backward (and, with DDP's overlapped
optimizer, the next forward's convolutions) instead of only the conv backward.

In the all-reduce regime (more rows than outputs, e.g. large per-rank batches) the
dense gradient is the smallest message, and a third mode shortens its critical path:

``chunked``      the layer's weight gradient is produced in C column chunks (the fused
                 head: channel groups, one kernel launch each) and each chunk's N row
                 segments are all-reduced (AVG) the moment its launch lands, instead of
                 one 720 MB bucket all-reduce after the whole head backward.  Same bytes
                 as the all-reduce; the first chunk's collective starts (C-1)/C of the
                 head backward earlier and the chunks pipeline over the xGMI links.

The result is the average DDP produces (floating-point summation order differs,
as it does between all-reduce algorithms), bit-identical on every rank.

Zero suppression (``compress``, default on): X is a ReLU output, so the activation exchange
sends it zero-suppressed (parallel/zs.py: a bitmask plus the non-zero values, rebuilt bit for bit
on the receiver -- the gradient and the parameters after the step are bitwise those of the dense
exchange).  Two all-gathers: the fixed-size mask/offset record (3.2 % of the dense rows, with
each rank's non-zero count in its tail) and the values at a capacity ``cap`` kept from earlier
steps (the first step sends the dense size).  The host learns the counts from the first gather
only when the step's gradient is formed (``defer``, after the head backward is queued); a count
above the capacity sends the dense rows once more for that step.  The byte model takes the
measured ratio: ``link_bytes("activations")`` = B·K·4·ratio.

Pooled source (activation path, the fused ConvNet head; ``source="pooled"``, the default): the
fc input X = relu(BN2(pooled conv2 output)) is a pointwise function of the head's pooled input ya
(fp16, 2 bytes per column: half of X in fp32, and no encode) and of 128 head constants per rank (BN2's
affine of that rank's batch, ya's decode, the conv bias).  The ranks all-gather ya and those
constants right after the conv2 forward wrote them -- before the head forward starts -- and every
rank forms the fc step from them (``ops.head_update_pooled``), recomputing each rank's X with that
rank's constants and the head forward's own arithmetic: bitwise the rows the dense exchange would
have sent.  ``link_bytes`` prices it at x_ratio 0.5.

Column groups (activation path, zero-suppressed): the rows travel as ``groups`` column ranges
(whole channel planes on the fused head), each encoded and gathered on its own.  The fused head
forward runs one launch per group and hands each group's rows over as soon as its launch is
queued (``begin_groups`` / ``group_ready``), so the first gather starts a quarter of the way
through the head forward instead of after the whole forward and one encode of all rows; the
deferred update (next forward) runs group by group right before the head launch that reads those
columns (``_Update.run_until``), so a group's gathers only have to land before that launch.

Protocol (driven by ``parallel/ddp.py``):

* ``arm(sync)`` each DDP forward: the exchange may run this step.
* the layer's forward calls ``begin(x)``; if an exchange is chosen it starts the
  async all-gather / all-to-all of ``x`` and tells DDP to leave this layer's
  bucket out of the bucket all-reduce; the layer then returns no weight/bias
  gradient.
* the layer's backward calls ``defer(dy)``: ``dy`` is kept and a callback is
  queued on the autograd engine.
* at the end of backward the callback all-gathers ``dy`` (a few hundred bytes),
  waits for ``x`` and writes ``dW``/``db`` straight into the bucket slots
  (``ops.linear_dw`` on the GPU: exact-fp32 MFMA, memory-bound; the sharded path
  writes its column shard in place and all-gathers the others).  Gradients
  accumulated locally under ``no_sync()`` are averaged with one all-reduce and
  this step's exchanged average is added, matching DDP's accumulation semantics.
"""
from __future__ import annotations

import os

from typing import List, Optional, Tuple

import torch

_ATTR = "_tds_activation_exchange"
_SHARD_ALIGN = 64  # shard boundaries on 256-byte multiples


def _meta_row(m: int) -> int:
    """int32 words of one rank's record in the activation exchange: the m mask/offset words,
    one pad word when m is odd, then the int64 non-zero count at an 8-byte aligned offset."""
    return m + (m & 1) + 2


def _counts_of(meta_all: torch.Tensor, world: int, row: int) -> torch.Tensor:
    """The [world] int64 counts in the tails of the all-gathered records (row = _meta_row)."""
    return meta_all.view(world, row)[:, row - 2:].contiguous().view(torch.int64).view(world)


def get(weight) -> Optional["ActivationExchange"]:
    return getattr(weight, _ATTR, None) if weight is not None else None


def link_bytes(path: str, rows: int, out_f: int, in_f: int, world: int, elem: int = 4, x_ratio: float = 1.0) -> float:
    """Bytes one rank sends over each of its links per step for ``path`` (model above);
    ``x_ratio``: the zero-suppressed size of the activation rows relative to dense."""
    if world <= 1:
        return 0.0
    if path == "allreduce":
        return 2.0 * out_f * in_f * elem / world
    if path == "activations":
        return float(rows * in_f * elem) * x_ratio
    if path == "sharded":
        return float((rows * x_ratio + out_f) * in_f * elem) / world
    raise ValueError(path)


def choose_path(rows: int, out_f: int, in_f: int, world: int, x_ratio: float = 1.0) -> str:
    """Cheapest of allreduce / activations / sharded by per-link bytes (ties: earlier start)."""
    order = ("activations", "sharded", "allreduce")
    costs = {p: link_bytes(p, rows, out_f, in_f, world, x_ratio=x_ratio) for p in order}
    return min(order, key=lambda p: (costs[p], order.index(p)))


def pooled_plane(in_f: int, planes: int = 32) -> Optional[int]:
    """Elements per (image, channel) of the fused head's pooled input for an fc layer of ``in_f``
    inputs (csrc/kernels/pooled_layout.h: Q x Q padded to blocks of 4 rows x 8 columns), or None
    when in_f is not ``planes`` square planes."""
    if in_f % planes:
        return None
    qq = in_f // planes
    q = int(round(qq ** 0.5))
    if q * q != qq or q < 4:
        return None
    return ((q + 3) // 4 * 4) * ((q + 7) // 8 * 8)


def shard_bounds(in_f: int, world: int) -> List[Tuple[int, int]]:
    per = -(-in_f // world)
    per = -(-per // _SHARD_ALIGN) * _SHARD_ALIGN
    return [(min(in_f, r * per), min(in_f, (r + 1) * per)) for r in range(world)]


class ActivationExchange:
    """One exchange-capable Linear layer under DDP (see the module docstring)."""

    CAP_MARGIN = 1.03     # value capacity over the largest recent non-zero count
    CAP_ROUND = 1 << 16   # capacities rounded up to 64 Ki elements (stable allocations)

    def __init__(self, weight: torch.nn.Parameter, bias: Optional[torch.nn.Parameter], group, world: int,
                 mode: str, set_skip, weight_view, bias_view, chunks: int = 1, compress: bool = True,
                 groups: int = 4, source: str = "pooled"):
        if mode not in ("auto", "activations", "sharded", "chunked", "allreduce"):
            raise ValueError(f"ActivationExchange mode must be auto|activations|sharded|chunked|allreduce, got {mode!r}")
        self.weight, self.bias = weight, bias
        self.group, self.world, self.mode = group, world, mode
        self.chunks = max(1, int(chunks))
        self.groups = max(1, int(groups))  # column groups of the zero-suppressed activation path
        if source not in ("pooled", "rows"):
            raise ValueError(f"ActivationExchange source must be pooled|rows, got {source!r}")
        # "pooled": the activation path takes the fused head's pooled input when the layer offers
        # it (begin_pooled); "rows": always the fc input rows X (begin / begin_groups)
        self.source = source
        self._pooled = None  # this step's pooled exchange (dict), or None
        self._works = []  # chunked: the per-chunk all-reduce works of this step
        self._set_skip, self._wview, self._bview = set_skip, weight_view, bias_view
        self.armed = False
        self.active = None  # the path running this step, or None
        self.steps_exchanged = 0
        self.last_path = None  # "activation-exchange" | "sharded-exchange" once a step used it
        self._x_buf = self._x_work = self._dy = self._x_local = None
        self.side_stream = None  # DDP(overlap_optimizer=True): its update stream, which also finishes the exchange
        self._own_stream = None  # otherwise (GPU): a private side stream
        # zero-suppressed activation rows (parallel/zs.py)
        self.compress = bool(compress)
        self._zs = None  # this step's encoded exchange: dict (sharded) or list of per-group dicts (activations)
        self._step_zs = False  # this step's rows travelled encoded (last_path's "(zs)" tag)
        # value capacity (elements) per path, from that path's earlier counts: "activations" holds
        # a per-rank total, "sharded" a per-segment slot, so neither may seed the other
        self._cap = {}
        # measured zero-suppressed / dense bytes of the busiest rank's rows in the last compressed
        # step (one definition for both paths: the byte model prices the busiest link)
        self.x_ratio = 1.0
        self.zs_stats = {"steps": 0, "overflows": 0, "last_nnz": None}
        self._cap_once = None  # force_capacity_once
        self._planes_hint = 0  # the fused head's channel planes (its groups are whole planes), once seen
        setattr(weight, _ATTR, self)

    def detach(self):
        if getattr(self.weight, _ATTR, None) is self:
            delattr(self.weight, _ATTR)

    # ---------------------------------------------------------------- policy
    def path(self, rows: int) -> Optional[str]:
        """"activations" | "sharded" | "chunked" for a step with ``rows`` local rows, or None
        (plain bucket all-reduce)."""
        if self.mode in ("activations", "sharded"):
            return self.mode
        if self.mode == "chunked":
            return "chunked" if self.chunks > 1 else None
        if self.world <= 1 or self.mode != "auto":
            return None
        out_f, in_f = self.weight.shape
        ratio = 0.5 if self.pooled_capable() else (self.x_ratio if self.compress else 1.0)
        p = choose_path(rows, out_f, in_f, self.world, x_ratio=ratio)
        # auto's all-reduce regime is the plain bucket all-reduce: the chunked path costs more
        # compute than it saves on the links (W=1 forced: +4.4 ms/step, docs/DISTRIBUTED.md), so
        # it runs only when asked for
        return None if p == "allreduce" else p

    def needs_rows(self) -> bool:
        """Does the running exchange need the layer's input rows (X) from its forward?"""
        return self.active in ("activations", "sharded")

    # ---------------------------------------------------------------- chunked all-reduce
    def column_chunks(self, in_f: int, planes: int = 0):
        """The [k0, k1) column ranges of the chunked weight gradient: whole planes of
        in_f / planes columns when ``planes`` (the fused head: channels) else 64-aligned."""
        if planes:
            per = in_f // planes
            n = min(self.chunks, planes)
            cuts = [round(i * planes / n) for i in range(n + 1)]
            return [(cuts[i] * per, cuts[i + 1] * per) for i in range(n) if cuts[i + 1] > cuts[i]]
        return [(a, e) for a, e in shard_bounds(in_f, self.chunks) if e > a]

    def column_groups(self, in_f: int, planes: int = 0):
        """The [k0, k1) column ranges of the grouped activation exchange: ``groups`` ranges of whole
        planes (the fused head: channels) or 64-aligned."""
        if planes:
            per = in_f // planes
            n = min(self.groups, planes)
            cuts = [round(i * planes / n) for i in range(n + 1)]
            return [(cuts[i] * per, cuts[i + 1] * per) for i in range(n) if cuts[i + 1] > cuts[i]]
        return [(a, e) for a, e in shard_bounds(in_f, self.groups) if e > a]

    def chunk_ready(self, dw: torch.Tensor, k0: int, k1: int):
        """Columns [k0, k1) of ``dw`` are final on the current stream: all-reduce their N row
        segments now (async AVG; the collective's stream waits for the producer)."""
        from . import distributed as tdist

        for j in range(dw.shape[0]):
            self._works.append(tdist.all_reduce(dw[j, k0:k1], tdist.ReduceOp.AVG, group=self.group, async_op=True))

    def chunked_done(self, dw: torch.Tensor, db: Optional[torch.Tensor]):
        """All chunks issued: all-reduce the bias, then (end of backward) order the consumer
        stream after every chunk and publish the gradients."""
        from . import distributed as tdist

        if db is not None:
            self._works.append(tdist.all_reduce(db, tdist.ReduceOp.AVG, group=self.group, async_op=True))
        works, self._works = self._works, []

        def finish():
            side = self.side_stream
            if side is not None and dw.is_cuda:
                with torch.cuda.stream(side):  # DDP's overlapped optimizer consumes them there
                    for w in works:
                        w.wait()
            else:
                for w in works:
                    w.wait()
            self.weight.grad = dw
            if self.bias is not None:
                self.bias.grad = db
            self.last_path = "chunked-allreduce"
            self.active = None
            self.steps_exchanged += 1

        torch.autograd.Variable._execution_engine.queue_callback(finish)

    def chunk_targets(self):
        """(dW, accumulate), (db, accumulate) for the chunked path: the bucket slots, or the
        gradients accumulated locally under no_sync() -- this step's chunk is added and the
        chunk of the sum all-reduced, which is what DDP's bucket all-reduce averages."""
        out = []
        for p, view_fn in ((self.weight, self._wview), (self.bias, self._bview)):
            if p is None:
                out.append((None, False))
            elif p.grad is not None:
                out.append((p.grad, True))
            else:
                out.append((view_fn(), False))
        return out

    def chunked_linear_backward(self, dy: torch.Tensor, x2: torch.Tensor):
        """Generic layer (ops.functional.linear): dW = dYᵀX column chunk by column chunk into
        the bucket slot, each chunk all-reduced as soon as it is formed."""
        (dw, acc_w), (db, acc_b) = self.chunk_targets()
        with torch.no_grad():
            for k0, k1 in self.column_chunks(dw.shape[1]):
                _dw_rows(dy, x2[:, k0:k1].contiguous(), dw[:, k0:k1], None, 1.0, acc_w, False)
                self.chunk_ready(dw, k0, k1)
            if db is not None:
                s_b = dy.sum(0)
                db.add_(s_b) if acc_b else db.copy_(s_b)
        self.chunked_done(dw, db)

    def preflight(self, rows: int, timed) -> Optional[str]:
        """Issue once, at the sizes of a step with ``rows`` local rows, every collective the path
        ``auto`` (or the forced mode) picks would run, each through ``timed(name, nbytes, kind,
        issue)`` -- ``issue()`` starts it and returns its work (or None) -- so a launcher can bound
        and time them before any model work (bench.py's preflight).  Returns the path (None: the
        plain bucket all-reduce, which the caller preflights with the buckets)."""
        from . import distributed as tdist
        from . import zs

        path = self.path(rows)
        if path is None:
            return None
        W, g = self.world, self.group
        out_f, in_f = self.weight.shape
        dev = self.weight.device
        me = tdist.get_rank(g)

        def gather(name, numel, dtype):
            src = torch.zeros(numel, device=dev, dtype=dtype)
            dst = torch.empty(W * numel, device=dev, dtype=dtype)
            nb = dst.numel() * dst.element_size()
            timed(name, nb, "all_gather", lambda: tdist.all_gather_into_tensor(dst, src, group=g, async_op=True))

        def peers(name, numel, nrows):
            # one grouped exchange with every peer: nrows chunks of numel elements each way
            bufs_s = [torch.zeros(numel, device=dev) for _ in range(nrows)]
            bufs_r = [torch.empty(numel, device=dev) for _ in range(nrows * W)]
            sends = [(t, p) for p in range(W) if p != me for t in bufs_s]
            recvs = [(bufs_r[p * nrows + i], p) for p in range(W) if p != me for i in range(nrows)]
            nb = numel * 4 * nrows  # per peer (link)
            timed(name, nb, "sendrecv", lambda: tdist.sendrecv(sends, recvs, group=g, async_op=True))

        n = rows * in_f
        zs_ok = self.compress and n < (1 << 31)
        pb = pooled_plane(in_f) if self.pooled_capable() else None
        if path == "activations" and pb is not None:
            gather("head record all-gather", 128, torch.float32)
            gather("pooled input (ya) all-gather (fp16)", rows * 32 * pb, torch.float16)
            gather("dY all-gather", rows * out_f, torch.float32)
        elif path == "activations":
            if zs_ok:
                groups = self.column_groups(in_f, self._planes_hint)
                for gi, (k0, k1) in enumerate(groups):
                    ng = rows * (k1 - k0)
                    tag = f", group {gi}" if len(groups) > 1 else ""
                    gather(f"zs records all-gather{tag} (int32)", _meta_row(zs.meta_numel(ng)), torch.int32)
                    cap = self._cap.get(("activations", gi))
                    gather(f"zs values all-gather{tag} (first-step capacity)", min(ng, cap) if cap else ng,
                           torch.float32)
            else:
                gather("activation rows all-gather", n, torch.float32)
            gather("dY all-gather", rows * out_f, torch.float32)
        elif path == "sharded":
            longest = max(e - a for a, e in shard_bounds(in_f, W))
            if zs_ok:
                gather("zs segment counts all-gather (int64)", W * rows, torch.int64)
            peers("X column-shard exchange (per peer)", longest, rows)
            gather("dY all-gather", rows * out_f, torch.float32)
            peers("updated W shard exchange (per peer)", longest, out_f)
        elif path == "chunked":
            seg = torch.zeros(-(-in_f // self.chunks), device=dev)
            timed("chunk row-segment all-reduce (AVG)", seg.numel() * 4, "all_reduce",
                  lambda: tdist.all_reduce(seg, tdist.ReduceOp.AVG, group=g, async_op=True))
        return path

    def worthwhile(self, rows: int) -> bool:
        return self.path(rows) is not None

    def arm(self, sync: bool):
        self.armed = bool(sync)
        self.active = None
        self._set_skip(False)

    # ---------------------------------------------------------------- forward
    def _eligible(self, rows: int) -> Optional[str]:
        if not self.armed or self.active is not None:
            return None
        return self.path(rows)

    def planned(self, rows: int) -> Optional[str]:
        """The path a forward with ``rows`` rows would start now (None: plain bucket all-reduce)."""
        return self._eligible(rows)

    def ready(self, rows: int) -> bool:
        """Would a forward with ``rows`` input rows (grad mode on) run an exchange?"""
        return torch.is_grad_enabled() and self._eligible(rows) is not None

    def begin(self, x2d: Optional[torch.Tensor], rows: Optional[int] = None) -> bool:
        """Called from the layer's forward (possibly inside an autograd Function,
        i.e. under no_grad) with its [rows, in] input (None with ``rows`` when the chunked
        path, which needs no X, was agreed by ``ready``).  Every rank has the same rows."""
        path = self._eligible(x2d.shape[0] if x2d is not None else int(rows))
        if path is None:
            return False
        from . import distributed as tdist

        if path == "chunked":
            self.active = path
            self._set_skip(True)
            return True
        x2d = x2d.detach().contiguous()
        rows, in_f = x2d.shape
        # the zero-suppressed format's offsets are int32 (csrc/kernels/zs_exchange.hip): larger
        # inputs take the dense exchange of the same path
        zs_ok = self.compress and x2d.dtype == torch.float32 and x2d.numel() < (1 << 31)
        if path == "activations" and zs_ok:
            groups = self.begin_groups(rows, in_f, x2d.device)
            for gi, (k0, k1) in enumerate(groups):
                self.group_ready(gi, x2d[:, k0:k1].contiguous())
            return True
        elif path == "activations":
            self._x_buf = torch.empty((self.world * rows, in_f), device=x2d.device, dtype=x2d.dtype)
            self._x_work = tdist.all_gather_into_tensor(self._x_buf, x2d, group=self.group, async_op=True)
        elif zs_ok:
            self._begin_zs_sharded(x2d)
        else:
            # all-to-all of column shards: rank s receives every rank's rows of shard s
            bounds = shard_bounds(in_f, self.world)
            me = tdist.get_rank(self.group)
            k0, k1 = bounds[me]
            self._x_buf = torch.empty((self.world, rows, k1 - k0), device=x2d.device, dtype=x2d.dtype)
            sends = [(x2d[b, a:e], s) for s, (a, e) in enumerate(bounds) if e > a for b in range(rows)]
            recvs = [(self._x_buf[s, b], s) for s in range(self.world) if k1 > k0 for b in range(rows)]
            self._x_work = tdist.sendrecv(sends, recvs, group=self.group, async_op=True)
        self._x_local = x2d  # keep alive until the exchange completes
        self.active = path
        self._set_skip(True)
        return True

    def grouped(self, rows: int, in_f: int) -> bool:
        """Would a forward with ``rows`` rows of ``in_f`` run the grouped zero-suppressed activation
        exchange (begin_groups / group_ready)?"""
        return self.compress and self._eligible(rows) == "activations" and rows * in_f < (1 << 31)

    def pooled_capable(self) -> bool:
        """Can this layer's activation exchange run from the pooled input (source "pooled", a GPU
        weight whose inputs are the fused head's 32 square planes)?  The byte model and the preflight
        price it so; the fused ConvNet head then takes it (a generic Linear still sends its rows)."""
        return self.source == "pooled" and self.weight.is_cuda and pooled_plane(self.weight.shape[1]) is not None

    def pooled(self, rows: int) -> bool:
        """Would a forward with ``rows`` rows run the activation exchange from the pooled input
        (``begin_pooled``)?"""
        return self.source == "pooled" and self._eligible(rows) == "activations"

    def begin_pooled(self, ya: torch.Tensor, rec: torch.Tensor, P: int) -> None:
        """Start the activation exchange from the fused head's pooled input (module docstring): the
        all-gathers of this rank's head record (128 floats, ``ops.head_pooled_record``) and of ya
        ([rows, 32, PB] fp16), queued where the conv2 forward wrote ya, before the head forward."""
        from . import distributed as tdist

        ya = ya.detach().contiguous()
        rec = rec.detach().contiguous().view(-1)
        W = self.world
        rec_all = torch.empty((W, rec.numel()), device=rec.device, dtype=rec.dtype)
        w_rec = tdist.all_gather_into_tensor(rec_all.view(-1), rec, group=self.group, async_op=True)
        ya_all = torch.empty((W,) + tuple(ya.shape), device=ya.device, dtype=ya.dtype)
        w_ya = tdist.all_gather_into_tensor(ya_all.view(-1), ya.view(-1), group=self.group, async_op=True)
        self._pooled = {"ya_all": ya_all, "rec_all": rec_all, "w_ya": w_ya, "w_rec": w_rec, "P": int(P),
                        "keep": (ya, rec)}
        self._zs = None
        self._step_zs = False
        self._x_local = ya  # keep alive until the exchange completes
        self._x_work = None
        out_f, in_f = self.weight.shape
        self.x_ratio = (ya.numel() * ya.element_size() + rec.numel() * 4) / float(ya.shape[0] * in_f * 4)
        self.active = "activations"
        self._set_skip(True)

    def _pooled_update(self, p, dy_all, out, scale: float, lr: float, acc: bool = False):
        """The fc step from the gathered pooled inputs on the current stream, after both gathers:
        lr > 0: the weight itself, W -= lr·scale·dy_allᵀX; else ``out`` (=/+=) scale·dy_allᵀX."""
        from .. import _ext

        p["w_rec"].wait()
        p["w_ya"].wait()
        mode = 0 if lr else (2 if acc else 1)
        _ext.ops().head_update_pooled(dy_all, p["ya_all"], p["rec_all"], self.weight.data, None if lr else out,
                                      p["P"], scale, float(lr or 0.0), mode)

    def begin_groups(self, rows: int, in_f: int, dev, planes: int = 0):
        """Start a grouped zero-suppressed activation exchange: returns the column groups; the caller
        hands each group's [rows, k1 - k0] rows to ``group_ready`` in order (the fused head: right
        after that group's launch).  Every rank uses the same groups."""
        if planes:
            self._planes_hint = int(planes)
        groups = self.column_groups(in_f, planes)
        self._zs = []
        self._zs_groups = groups
        self._x_local = []
        self._step_zs = True
        self._x_work = None
        self.active = "activations"
        self._set_skip(True)
        return groups

    def group_ready(self, gi: int, xg: torch.Tensor):
        """Group ``gi``'s rows are final on the current stream: encode them and start their two
        gathers (records with the count in their tail, then the values at this group's capacity)."""
        k0, k1 = self._zs_groups[gi]
        if len(self._zs) != gi or tuple(xg.shape) != (xg.shape[0], k1 - k0):
            raise RuntimeError(f"activation exchange: group {gi} out of order or of the wrong width")
        xg = xg.detach().contiguous()
        z = self._begin_zs(xg, gi)
        z["k0"], z["k1"], z["x_local"] = k0, k1, xg
        self._zs.append(z)
        self._x_local.append(xg)  # keep alive until the exchange completes

    def force_capacity_once(self, cap: int) -> None:
        """Fault injection (tests): the next encoded step sends its values at capacity ``cap``
        (elements; the sharded path: per segment), whatever the earlier counts gave -- a cap below
        the step's counts drives the overflow path (the dense re-send)."""
        self._cap_once = max(1, int(cap))

    def _take_cap(self, path: str, n: int, gi: Optional[int] = None) -> int:
        if self._cap_once is not None:
            cap, self._cap_once = min(n, self._cap_once), None
            return cap
        cap = self._cap.get((path, gi)) if gi is not None else None
        if cap is None:  # (a path-level capacity: the first step, or set by a test)
            cap = self._cap.get(path)
        return min(n, cap) if cap else n

    def _begin_zs(self, x2d: torch.Tensor, gi: int = 0):
        """Zero-suppressed all-gather of one column group's rows (module docstring): encode, gather
        the fixed-size mask/offset records with each rank's count in their tail, then the values at
        the group's capacity.  The counts are copied to the host asynchronously after the first
        gather, so the consumer can check them without waiting for the values.  Returns the group's
        state."""
        from . import distributed as tdist
        from . import zs

        dev, n, shape = x2d.device, x2d.numel(), tuple(x2d.shape)
        W = self.world
        M = zs.meta_numel(n)
        R = _meta_row(M)
        cap = self._take_cap("activations", n, gi)
        meta = torch.empty(R, device=dev, dtype=torch.int32)
        vals = torch.empty(cap, device=dev, dtype=torch.float32)
        nnz = zs.encode(x2d, meta[:M], vals)
        meta[R - 2:].view(torch.int64).copy_(nnz.view(1).to(dev))
        meta_all = torch.empty(W * R, device=dev, dtype=torch.int32)
        w_meta = tdist.all_gather_into_tensor(meta_all, meta, group=self.group, async_op=True)
        counts_host = counts_ev = None
        if dev.type == "cuda":
            # the counts to the host behind the first gather only (not behind the values)
            cstream = self._count_stream(dev)
            with torch.cuda.stream(cstream):
                w_meta.wait()
                counts = _counts_of(meta_all, W, R)
                counts_host = torch.empty(W, dtype=torch.int64, pin_memory=True)
                counts_host.copy_(counts, non_blocking=True)
                counts_ev = torch.cuda.Event()
                counts_ev.record(cstream)
                meta_all.record_stream(cstream)
        vals_all = torch.empty(W * cap, device=dev, dtype=torch.float32)
        w_vals = tdist.all_gather_into_tensor(vals_all, vals, group=self.group, async_op=True)
        return {"n": n, "M": M, "R": R, "cap": cap, "meta": meta, "vals": vals, "meta_all": meta_all,
                "vals_all": vals_all, "w_meta": w_meta, "w_vals": w_vals, "counts_host": counts_host,
                "counts_ev": counts_ev, "rows": shape[0], "in_f": shape[1], "gi": gi}

    def _layouts(self, rows: int, in_f: int, dev):
        """(send, receive) segment layouts of the sharded exchange (parallel/zs.py SegLayout),
        cached per shape: send = (destination shard s, row b) slices of X, destination-major;
        receive = (source rank r, row b) rows of this rank's shard in the dense buffer."""
        from . import distributed as tdist
        from . import zs

        key = (rows, in_f, str(dev))
        lays = getattr(self, "_lays", None)
        if lays is None or lays[0] != key:
            bounds = shard_bounds(in_f, self.world)
            me = tdist.get_rank(self.group)
            k0, k1 = bounds[me]
            send = zs.SegLayout([(b * in_f + a, e - a) for (a, e) in bounds for b in range(rows)], dev)
            n_me = k1 - k0
            recv = zs.SegLayout([((r * rows + b) * n_me, n_me) for r in range(self.world) for b in range(rows)], dev)
            self._lays = lays = (key, send, recv, bounds)
        return lays[1], lays[2], lays[3]

    def _begin_zs_sharded(self, x2d: torch.Tensor):
        """Zero-suppressed column-shard all-to-all: each (destination, row) slice is a segment
        of its own (fixed-size records + a value slot of this step's capacity per segment);
        every rank's segment counts are all-gathered, so all ranks take the same capacity and
        overflow decisions."""
        from . import distributed as tdist
        from . import zs

        W, dev = self.world, x2d.device
        rows, in_f = x2d.shape
        send, recv, bounds = self._layouts(rows, in_f, dev)
        me = tdist.get_rank(self.group)
        n_me = bounds[me][1] - bounds[me][0]
        longest = max(e - a for a, e in bounds)
        cap = max(1, self._take_cap("sharded", longest))
        meta_send = torch.empty(send.meta_numel, device=dev, dtype=torch.int32)
        vals_send = torch.empty(send.nseg * cap, device=dev, dtype=torch.float32)
        nnz = zs.seg_encode(x2d, send, meta_send, vals_send, cap).to(dev)
        nnz_all = torch.empty(W * send.nseg, device=dev, dtype=torch.int64)
        w_cnt = tdist.all_gather_into_tensor(nnz_all, nnz, group=self.group, async_op=True)
        counts_host = counts_ev = None
        if dev.type == "cuda":
            cstream = self._count_stream(dev)
            with torch.cuda.stream(cstream):
                w_cnt.wait()
                counts_host = torch.empty(W * send.nseg, dtype=torch.int64, pin_memory=True)
                counts_host.copy_(nnz_all, non_blocking=True)
                counts_ev = torch.cuda.Event()
                counts_ev.record(cstream)
                nnz_all.record_stream(cstream)
        mr = recv.meta_numel // W  # one source's records for this rank's shard
        meta_recv = torch.empty(W * mr, device=dev, dtype=torch.int32)
        sends, recvs = [], []
        for s_ in range(W):
            m0, m1 = send.meta_range(s_ * rows, (s_ + 1) * rows)
            if m1 > m0:
                sends.append((meta_send[m0:m1], s_))
        if mr > 0:
            recvs = [(meta_recv[r * mr:(r + 1) * mr], r) for r in range(W)]
        w_meta = tdist.sendrecv(sends, recvs, group=self.group, async_op=True)
        vals_recv = torch.empty(W * rows * cap, device=dev, dtype=torch.float32)
        span = rows * cap
        sends_v = [(vals_send[s_ * span:(s_ + 1) * span], s_) for s_ in range(W) if bounds[s_][1] > bounds[s_][0]]
        recvs_v = [(vals_recv[r * span:(r + 1) * span], r) for r in range(W)] if n_me > 0 else []
        w_vals = tdist.sendrecv(sends_v, recvs_v, group=self.group, async_op=True)
        self._x_buf = torch.empty((W, rows, n_me), device=dev, dtype=x2d.dtype)
        self._zs = {"kind": "sharded", "n": longest, "cap": cap, "w_cnt": w_cnt, "nnz_all": nnz_all,
                    "counts_host": counts_host, "counts_ev": counts_ev, "w_meta": w_meta, "w_vals": w_vals,
                    "meta_recv": meta_recv, "vals_recv": vals_recv, "recv": recv, "keep": (meta_send, vals_send),
                    "meta_bytes": send.meta_numel, "dense": x2d.numel(), "nseg": send.nseg}
        self._step_zs = True
        self._x_work = None

    def _count_stream(self, dev):
        st = getattr(self, "_cstream", None)
        if st is None:
            st = self._cstream = torch.cuda.Stream(device=dev)
        return st

    def _zs_counts(self, z):
        """The all-gathered non-zero counts of an encoded step, on the host (CUDA: from the pinned
        copy queued behind the first, small gather; by the time a caller asks -- the end of the
        backward, or the next forward's head -- it has landed, so the wait is a formality)."""
        W = self.world
        if z.get("kind") == "sharded":
            if z["counts_ev"] is not None:
                z["counts_ev"].synchronize()
                return [int(v) for v in z["counts_host"].tolist()]
            z["w_cnt"].wait()
            return [int(v) for v in z["nnz_all"].tolist()]
        if z["counts_ev"] is not None:
            z["counts_ev"].synchronize()
            return [int(v) for v in z["counts_host"].tolist()]
        z["w_meta"].wait()  # CPU: the gathers are synchronous enough to read directly
        return [int(v) for v in _counts_of(z["meta_all"], W, z["R"]).tolist()]

    def _zs_check(self, z) -> bool:
        """Account one encoded step: statistics, the path's capacity for the next steps and the
        measured ratio; True when some count exceeded this step's capacity (its values did not
        all travel: the step must use the dense rows)."""
        counts = self._zs_counts(z)
        self.zs_stats["steps"] += 1
        if z.get("kind") == "sharded":
            mx = max(counts) if counts else 0
            self.zs_stats["last_nnz"] = mx
            self._cap["sharded"] = max(1, min(z["n"], -(-int(mx * self.CAP_MARGIN) // self.CAP_ROUND) * self.CAP_ROUND))
            per_rank = [sum(counts[r * z["nseg"]:(r + 1) * z["nseg"]]) for r in range(self.world)]
            self.x_ratio = (max(per_rank) + z["meta_bytes"]) / z["dense"]  # busiest rank vs its dense rows
        else:
            mx = max(counts)
            self.zs_stats["last_nnz"] = counts
            self._cap["activations"] = min(z["n"], -(-int(mx * self.CAP_MARGIN) // self.CAP_ROUND) * self.CAP_ROUND)
            self.x_ratio = (mx + z["R"] * 1.0) / z["n"]  # bytes relative to dense (4-byte words both)
        if mx > z["cap"]:
            self.zs_stats["overflows"] += 1
            return True
        return False

    def _zs_check_groups(self, zl) -> List[bool]:
        """The count check of a grouped activation step (every group's counts are in by then): per
        group, did some rank's count exceed the group's capacity?  Sets each group's capacity for the
        next steps, the statistics (one step) and the measured ratio over all groups."""
        W = self.world
        over, tot, dense, per_rank = [], 0.0, 0, [0] * W
        for z in zl:
            counts = self._zs_counts(z)
            mx = max(counts)
            gi = z["gi"]
            self._cap[("activations", gi)] = min(z["n"], -(-int(mx * self.CAP_MARGIN) // self.CAP_ROUND) * self.CAP_ROUND)
            over.append(mx > z["cap"])
            tot += mx + z["R"]
            dense += z["n"]
            for r in range(W):
                per_rank[r] += counts[r]
        self.zs_stats["steps"] += 1
        self.zs_stats["last_nnz"] = per_rank
        if any(over):
            self.zs_stats["overflows"] += 1
        self.x_ratio = tot / max(1, dense)  # bytes relative to dense (4-byte words both)
        return over

    def _zs_materialize_groups(self, zl, over):
        """The paths that form the gradient from dense rows (CPU; the GPU side-stream finish, on
        the side stream): the full [W * rows, in_f] rows in self._x_buf, each group decoded into its
        columns -- or, after its overflow, that group's rows gathered dense."""
        from . import distributed as tdist

        rows, in_f = zl[0]["rows"], self.weight.shape[1]
        dev = zl[0]["meta"].device
        W = self.world
        self._x_buf = torch.empty((W * rows, in_f), device=dev, dtype=torch.float32)
        for z, o in zip(zl, over):
            tmp = torch.empty((W * rows, z["k1"] - z["k0"]), device=dev, dtype=torch.float32)
            if o:
                z["w_vals"].wait()
                tdist.all_gather_into_tensor(tmp, z["x_local"], group=self.group)
            else:
                self._zs_decode_into(z, tmp)
            self._x_buf[:, z["k0"]:z["k1"]].copy_(tmp)
        self._x_work = _DoneWork()

    def _zs_resolve(self):
        """Host side of the zero-suppressed exchange (CPU, and the GPU side-stream finish, which
        runs from an end-of-backward callback): check the counts, then set up the dense rows
        self._x_buf -- rebuilt from the encodings, or, after an overflow, a dense re-send of this
        step's rows (every rank saw the same counts, so all take the same branch)."""
        from . import distributed as tdist

        z, self._zs = self._zs, None
        if isinstance(z, list):  # grouped activation step: check now, rebuild where the gradient is formed
            self._zs_decode_pending = ("groups", z, self._zs_check_groups(z))
            return
        overflow = self._zs_check(z)
        if z.get("kind") == "sharded":
            if overflow:  # some segment overflowed its slot: the dense all-to-all, once
                z["w_meta"].wait()
                z["w_vals"].wait()
                x2d = self._x_local
                rows, in_f = x2d.shape
                bounds = shard_bounds(in_f, self.world)
                me = tdist.get_rank(self.group)
                k0, k1 = bounds[me]
                sends = [(x2d[b, a:e], s_) for s_, (a, e) in enumerate(bounds) if e > a for b in range(rows)]
                recvs = [(self._x_buf[s_, b], s_) for s_ in range(self.world) if k1 > k0 for b in range(rows)]
                self._x_work = tdist.sendrecv(sends, recvs, group=self.group, async_op=True)
                return
            self._zs_decode_pending = z
            return
        if overflow:  # a count above this step's capacity: the dense rows, once
            rows, in_f = z["rows"], z["in_f"]
            self._x_buf = torch.empty((self.world * rows, in_f), device=z["meta"].device, dtype=torch.float32)
            z["w_vals"].wait()
            self._x_work = tdist.all_gather_into_tensor(self._x_buf, self._x_local, group=self.group,
                                                        async_op=True)
            return
        self._zs_decode_pending = z

    def _zs_decode(self):
        """Rebuild every rank's rows into self._x_buf (current stream = where the gradient is
        formed), after the values gather."""
        z = getattr(self, "_zs_decode_pending", None)
        if z is None:
            return
        self._zs_decode_pending = None
        if isinstance(z, tuple):
            self._zs_materialize_groups(z[1], z[2])
            return
        if self._x_buf is None:
            self._x_buf = torch.empty((self.world * z["rows"], z["in_f"]), device=z["meta"].device, dtype=torch.float32)
        self._zs_decode_into(z, self._x_buf)

    def _zs_fused(self, z, targets=()) -> bool:
        """Can the gathered activation rows feed the dW formation encoded (``linear_dw_zs``:
        decoded in registers, no dense rows written and read back)?  That kernel takes N in
        {10, 16} outputs, K % 4 == 0 and 16-byte aligned rows of every tensor it writes
        (zs_exchange.hip tds_linear_dw_zs); anything else decodes and runs ``linear_dw``."""
        if not isinstance(z, dict) or z.get("kind") == "sharded" or not z["meta"].is_cuda:
            return False
        n_out, k = self.weight.shape
        if n_out not in (10, 16) or k % 4:
            return False
        for t in targets:
            if t is None:
                continue
            if t.stride(1) != 1 or t.stride(0) % 4 or t.data_ptr() % 16:
                return False
        return True

    def _dw_zs(self, z, dy_all, dw, db, scale: float, acc: bool, lr: float = 0.0):
        """dW (=/+=) scale·dy_allᵀX (or the update-only W -= lr·scale·dy_allᵀX) straight from the
        all-gathered encodings, on the current stream after both gathers."""
        from .. import _ext

        z["w_meta"].wait()
        z["w_vals"].wait()
        W, R, cap = self.world, z["R"], z["cap"]
        _ext.ops().linear_dw_zs(dy_all, z["meta_all"].view(W, R), z["vals_all"].view(W, cap), z["rows"], dw, db,
                                scale, acc, lr)

    def _zs_decode_into(self, z, x_buf):
        """Every rank's rows of one encoded tensor (a sharded step, or one activation group) into
        x_buf [W * rows, width] (contiguous)."""
        from . import zs

        z["w_meta"].wait()
        z["w_vals"].wait()
        if z.get("kind") == "sharded":
            zs.seg_decode(z["meta_recv"], z["recv"], z["vals_recv"], z["cap"], x_buf)
            return
        W, n, M, R, cap = self.world, z["n"], z["M"], z["R"], z["cap"]
        meta_all = z["meta_all"].view(W, R)
        vals_all = z["vals_all"].view(W, cap)
        out = x_buf.view(W, n)
        for r in range(W):
            zs.decode(meta_all[r, :M], vals_all[r], out[r])

    # ---------------------------------------------------------------- backward
    def defer(self, dy: torch.Tensor, x2: Optional[torch.Tensor] = None):
        """Called from the layer's backward with dY.  The host never waits here: on the GPU the
        rest of the exchange (dY gather, the zero-suppressed count check, dW formation, shard
        all-gather) is either left to the weight's first reader in the next forward
        (``_defer_update_inline``) or issued on a side stream from an end-of-backward callback,
        i.e. after every backward kernel is queued, so a count check that has to wait for the
        gathered counts cannot open a gap between the head backward and the conv2 backward.
        The compute stream waits for the side stream at the end of backward (or, under DDP's
        overlapped optimizer, the optimizer's side stream does).  On the CPU it all runs from
        an end-of-backward callback.  ``chunked``: the weight gradient is formed here from ``x2``
        chunk by chunk, each chunk all-reduced."""
        if self.active == "chunked":
            self.chunked_linear_backward(dy.detach().contiguous(), x2.detach())
            return
        self._dy = dy.detach().contiguous()
        if not self._dy.is_cuda:
            if self._zs is not None:
                self._zs_resolve()
            torch.autograd.Variable._execution_engine.queue_callback(self._finish)
            return
        if self._defer_update_inline():
            return
        torch.autograd.Variable._execution_engine.queue_callback(self._finish_on_side)

    def _finish_on_side(self):
        """GPU finish of the exchange on a side stream (end-of-backward callback)."""
        dev = self._dy.device
        if self._zs is not None:
            self._zs_resolve()
        side = self.side_stream
        join = side is None
        if side is None:
            if self._own_stream is None:
                from ..utils.streams import side_stream

                # the reserved CUs when a CU split is active (utils/streams.py), else a plain stream
                self._own_stream = side_stream(dev) or torch.cuda.Stream(device=dev)
            side = self._own_stream
        cur = torch.cuda.current_stream(dev)
        side.wait_stream(cur)
        keep = (self._dy, self._x_buf, self._x_local)  # used on the side stream
        keep = tuple(t for t in keep if not isinstance(t, list)) + tuple(self._x_local or ()) \
            if isinstance(self._x_local, list) else keep
        if self._pooled is not None:
            keep = keep + (self._pooled["ya_all"], self._pooled["rec_all"]) + self._pooled["keep"]
        z = getattr(self, "_zs_decode_pending", None)
        if isinstance(z, tuple):  # grouped activation step: every group's buffers
            for zg in z[1]:
                keep = keep + (zg["meta_all"], zg["vals_all"], zg["meta"], zg["vals"])
        elif z is not None:
            if z.get("kind") == "sharded":
                keep = keep + (z["meta_recv"], z["vals_recv"]) + z["keep"]
            else:
                keep = keep + (z["meta_all"], z["vals_all"], z["meta"], z["vals"])
        with torch.cuda.stream(side):
            for t in keep:
                if t is not None:
                    t.record_stream(side)
            self._finish()
        if join:
            cur.wait_stream(side)

    def _defer_update_inline(self) -> bool:
        """Activations path under DDP's overlapped optimizer with the step fused in (plain SGD):
        leave the weight update -- the count check, decode, dW formation and ``W -= lr·dW`` in one
        ``linear_dw`` sweep over the 720 MB weight -- to the first reader of the weight, the next
        forward's head, where it runs on the compute stream across the whole GPU (ops/param_fence.py:
        ``defer``).  Run beside the backward's persistent kernels on a side stream the same
        sweep took 1.7-2.0 ms and slowed the conv2 / layer-1 backward by ~0.8 ms (world 1,
        forced exchange, profiles/r3_exchange_side_vs_inline.md).  The host reads the gathered
        counts only there (they landed during this step's backward); after an overflow the
        update re-sends this step's rows dense from that point (all ranks saw the same counts).
        The bias keeps its side-stream path (dY gather, bias gradient, the optimizer's step),
        which needs dY only.  ``TDS_EXCHANGE_UPDATE=side`` keeps the whole finish on the side
        stream."""
        import os

        from ..ops import fused_update, param_fence
        from . import distributed as tdist

        if self.active != "activations" or self.side_stream is None:
            return False
        if os.environ.get("TDS_EXCHANGE_UPDATE", "inline").strip().lower() != "inline":
            return False
        lr = fused_update.take(self.weight, exchanged=True)
        if not lr:
            return False
        dy = self._dy
        dev = dy.device
        rows = dy.shape[0]
        scale = 1.0 / self.world
        cur = torch.cuda.current_stream(dev)
        side = self.side_stream
        side.wait_stream(cur)
        dy_all = torch.empty((self.world * rows, dy.shape[1]), device=dev, dtype=dy.dtype)
        with torch.cuda.stream(side), torch.no_grad():
            dy.record_stream(side)
            tdist.all_gather_into_tensor(dy_all, dy, group=self.group)
            (_, _), (db, acc_b) = self._targets()
            if db is not None:
                s_b = dy_all.sum(0).mul_(scale)
                db.add_(s_b) if acc_b else db.copy_(s_b)
                self.bias.grad = db
            ev_dy = torch.cuda.Event()
            ev_dy.record(side)
        z, self._zs = self._zs, None
        pooled, self._pooled = self._pooled, None
        x_work, x_dense = self._x_work, self._x_buf
        xl = self._x_local  # (captured: _done() below clears the attribute before update() runs)
        in_f = self.weight.shape[1]
        weight, lr, group, world = self.weight, float(lr), self.group, self.world

        ex = self

        class _Update:
            """The deferred update (param_fence.defer), queued on the current stream when called: the
            count check, then the update from the gathered encodings (or, after an overflow, from
            this step's rows re-sent dense).  A grouped step (a list of column groups) also runs
            group by group: ``run_until(k)`` queues the groups that start below column k -- the fused
            head forward calls it right before each of its range launches (``fused_kind``), so a
            group's gathers only have to land before the launch that reads its columns.  (Applying
            the update inside the head forward while it streams the weight measured even with this
            separate sweep, 0.585 vs 0.570 ms, r5_s8.)"""

            fused_kind = "groups" if isinstance(z, list) else None

            def __init__(self):
                self.over = None  # per group: did its counts overflow the capacity?
                self.next = 0     # the next group to queue

            def run_until(self, k_end):
                from .. import _ext

                torch.cuda.current_stream(dev).wait_event(ev_dy)
                with torch.no_grad():
                    if not isinstance(z, list):
                        if self.next == 0:
                            self.next = 1
                            self._whole()
                        return
                    if self.over is None:
                        self.over = ex._zs_check_groups(z)
                    while self.next < len(z) and z[self.next]["k0"] < k_end:
                        zg, o = z[self.next], self.over[self.next]
                        self.next += 1
                        wcols = weight.data[:, zg["k0"]:zg["k1"]]
                        if not o and ex._zs_fused(zg, (wcols,)):
                            ex._dw_zs(zg, dy_all, wcols, None, scale, False, lr)
                            continue
                        x_buf = torch.empty((world * rows, zg["k1"] - zg["k0"]), device=dev, dtype=torch.float32)
                        if o:  # overflow: this group's rows, dense, from every rank
                            zg["w_vals"].wait()
                            tdist.all_gather_into_tensor(x_buf, zg["x_local"], group=group)
                        else:
                            ex._zs_decode_into(zg, x_buf)
                        _ext.ops().linear_dw(dy_all, x_buf, wcols, None, scale, False, lr)

            def _whole(self):
                from .. import _ext

                x_buf = None
                if pooled is not None:
                    ex._pooled_update(pooled, dy_all, None, scale, lr)
                    return
                if z is not None:
                    if not ex._zs_check(z):
                        if ex._zs_fused(z, (weight.data,)):
                            ex._dw_zs(z, dy_all, weight.data, None, scale, False, lr)
                            return
                        x_buf = torch.empty((world * rows, in_f), device=dev, dtype=torch.float32)
                        ex._zs_decode_into(z, x_buf)
                    else:  # overflow: this step's rows, dense, from every rank
                        z["w_vals"].wait()
                        x_buf = torch.empty((world * rows, in_f), device=dev, dtype=torch.float32)
                        tdist.all_gather_into_tensor(x_buf, xl, group=group)
                else:
                    x_work.wait()
                    x_buf = x_dense
                _ext.ops().linear_dw(dy_all, x_buf, weight.data, None, scale, False, lr)

            def __call__(self):
                self.run_until(float("inf"))

        param_fence.defer(weight, _Update())
        fused_update.applied(weight)
        self._pooled_tag = pooled is not None
        self._done()
        return True

    def _targets(self, weight: bool = True):
        """(dW, accumulate_w), (db, accumulate_b) — gradients accumulated under no_sync()
        are averaged first (one all-reduce), this step's exchanged average is added.
        ``weight=False``: the bias only (dW is (None, False)); the weight's bucket slot is not
        requested, so DDP never allocates it (parallel/ddp.py ``_lazy_from``)."""
        from . import distributed as tdist

        out = []
        for p, view_fn in ((self.weight if weight else None, self._wview), (self.bias, self._bview)):
            if p is None:
                out.append((None, False))
            elif p.grad is not None:
                tdist.all_reduce(p.grad, tdist.ReduceOp.AVG, group=self.group)
                out.append((p.grad, True))
            else:
                out.append((view_fn(), False))
        return out

    def _finish(self):
        from . import distributed as tdist

        dy = self._dy
        rows = dy.shape[0]
        dy_all = torch.empty((self.world * rows, dy.shape[1]), device=dy.device, dtype=dy.dtype)
        tdist.all_gather_into_tensor(dy_all, dy, group=self.group)
        pooled, self._pooled = self._pooled, None
        if pooled is not None:
            self._finish_pooled(pooled, dy_all)
            return
        zf = getattr(self, "_zs_decode_pending", None)
        # (the bucket slot dW may be written to is 256-byte aligned with rows of K % 4 == 0 floats,
        # which _zs_fused checks; it is not requested here, so the update-only path never allocates it)
        targets = (self.weight.data, self.weight.grad)
        if self.active == "activations" and self._zs_fused(zf, targets):
            self._zs_decode_pending = None  # formed from the encodings below (_dw_zs)
        else:
            zf = None
            if getattr(self, "_zs_decode_pending", None) is not None:
                self._zs_decode()
            else:
                self._x_work.wait()
        scale = 1.0 / self.world
        from ..ops import fused_update

        # optimizer-in-backward (DDP overlap_optimizer, plain SGD, ops/fused_update.py): the
        # averaged step is applied to the weight while its gradient is formed -- no dW in HBM and
        # no separate SGD sweep over the 720 MB weight; .grad stays None
        lr = fused_update.take(self.weight, exchanged=True) if dy.is_cuda else None
        if lr:
            with torch.no_grad():
                self._finish_update(dy_all, rows, scale, float(lr), zf)
            fused_update.applied(self.weight)
            self._done()
            return
        with torch.no_grad():
            (dw, acc_w), (db, acc_b) = self._targets()
            if zf is not None:
                if db is not None and acc_b != acc_w:
                    s_b = dy_all.sum(0).mul_(scale)
                    db.add_(s_b) if acc_b else db.copy_(s_b)
                    self._dw_zs(zf, dy_all, dw, None, scale, acc_w)
                else:
                    self._dw_zs(zf, dy_all, dw, db, scale, acc_w)
            elif self.active == "activations":
                _dw_rows(dy_all, self._x_buf, dw, db, scale, acc_w, acc_b)
            else:
                bounds = shard_bounds(dw.shape[1], self.world)
                me = tdist.get_rank(self.group)
                k0, k1 = bounds[me]
                x_rows = self._x_buf.view(self.world * rows, k1 - k0)
                _dw_rows(dy_all, x_rows, dw[:, k0:k1], db, scale, acc_w, acc_b)
                # all-gather of the column shards: N row pieces per peer, straight into dW
                n_out = dw.shape[0]
                sends = [(dw[c, k0:k1], s) for s in range(self.world) if s != me and k1 > k0 for c in range(n_out)]
                recvs = [(dw[c, a:e], s) for s, (a, e) in enumerate(bounds) if s != me and e > a
                         for c in range(n_out)]
                w = tdist.sendrecv(sends, recvs, group=self.group, async_op=True)
                w.wait()
        self.weight.grad = dw
        if self.bias is not None:
            self.bias.grad = db
        self._done()

    def _finish_pooled(self, pooled, dy_all):
        """``_finish`` of a pooled step: the update-only step (optimizer-in-backward), or dW into
        the bucket slot (accumulated under no_sync as ``_targets`` sets up) and db."""
        from ..ops import fused_update

        scale = 1.0 / self.world
        lr = fused_update.take(self.weight, exchanged=True)
        with torch.no_grad():
            if lr:
                (_, _), (db, acc_b) = self._targets(weight=False)
                self._pooled_update(pooled, dy_all, None, scale, float(lr))
            else:
                (dw, acc_w), (db, acc_b) = self._targets()
                self._pooled_update(pooled, dy_all, dw, scale, 0.0, acc_w)
                self.weight.grad = dw
            if db is not None:
                s_b = dy_all.sum(0).mul_(scale)
                db.add_(s_b) if acc_b else db.copy_(s_b)
        if self.bias is not None:
            self.bias.grad = db
        if lr:
            fused_update.applied(self.weight)
        self._pooled_tag = True
        self._done()

    def _done(self):
        self.last_path = "activation-exchange" if self.active == "activations" else "sharded-exchange"
        if self._step_zs:  # (under the deferred update the count check runs in the next forward)
            self.last_path += "(zs)"
        elif getattr(self, "_pooled_tag", False):
            self.last_path += "(pooled)"
        self._step_zs = self._pooled_tag = False
        self._x_buf = self._x_work = self._dy = self._x_local = None
        self.active = None
        self.steps_exchanged += 1

    def _finish_update(self, dy_all, rows: int, scale: float, lr: float, zf=None):
        """Update-only finish: W -= lr * scale * dy_allᵀ X (activations: every column here;
        sharded: this rank's column shard, then an all-gather of the UPDATED shards straight
        into W); the bias keeps its gradient path (tiny, stepped by the optimizer)."""
        from .. import _ext
        from . import distributed as tdist

        (_, _), (db, acc_b) = self._targets(weight=False)
        W = self.weight.data
        ops = _ext.ops()
        if self.active == "activations" and zf is not None:
            self._dw_zs(zf, dy_all, W, db, scale, acc_b, lr)
        elif self.active == "activations":
            ops.linear_dw(dy_all, self._x_buf, W, db, scale, acc_b, lr)
        else:
            bounds = shard_bounds(W.shape[1], self.world)
            me = tdist.get_rank(self.group)
            k0, k1 = bounds[me]
            if k1 > k0:
                x_rows = self._x_buf.view(self.world * rows, k1 - k0)
                ops.linear_dw(dy_all, x_rows, W[:, k0:k1], db, scale, acc_b, lr)
            elif db is not None:
                s_b = dy_all.sum(0).mul_(scale)
                db.add_(s_b) if acc_b else db.copy_(s_b)
            n_out = W.shape[0]
            sends = [(W[c, k0:k1], s) for s in range(self.world) if s != me and k1 > k0 for c in range(n_out)]
            recvs = [(W[c, a:e], s) for s, (a, e) in enumerate(bounds) if s != me and e > a for c in range(n_out)]
            if sends or recvs:
                tdist.sendrecv(sends, recvs, group=self.group, async_op=True).wait()
        if self.bias is not None:
            self.bias.grad = db


def _dw_rows(dy_all, x_rows, dw, db, scale: float, acc_w: bool, acc_b: bool):
    """dW (=/+=) scale·dy_allᵀ·x_rows, db (=/+=) scale·Σ dy_all; dw may be a column slice."""
    from .. import _ext

    if dy_all.is_cuda and (db is None or acc_w == acc_b):
        _ext.ops().linear_dw(dy_all, x_rows, dw, db, scale, acc_w)
        return
    upd = torch.mm(dy_all.t(), x_rows).mul_(scale)
    dw.add_(upd) if acc_w else dw.copy_(upd)
    if db is not None:
        s_b = dy_all.sum(0).mul_(scale)
        db.add_(s_b) if acc_b else db.copy_(s_b)


class _DoneWork:
    """A finished work (the rows are already in place)."""

    def wait(self):
        return None
