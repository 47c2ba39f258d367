"""DistributedDataParallel for one-process-per-GPU training over RCCL/xGMI.

API mirrors ``torch.nn.parallel.DistributedDataParallel(model, device_ids=[gpu])``
(mnist_distributed.py:67) and reproduces its semantics:
rank-0 parameter/buffer broadcast at construction (C5), rank-0 buffer
broadcast before every forward when ``broadcast_buffers`` (C6), gradients
averaged over ranks with bucketed asynchronous all-reduce overlapped with the
backward (C7/C8), ``no_sync()`` for accumulation.

What is different (MI355X-first):

* **Flat parameter + gradient buffers.**  Parameters are re-homed into one
  flat buffer (``param.data`` becomes a view; the Parameter objects — and so
  optimizer references and state_dict names — are unchanged) and gradients
  live in a flat bucket buffer with the same layout.  Broadcast at
  construction is one call, the optimizer step is one sweep
  (``ops.optim.SGD``), and there is no copy-in/copy-out of gradients
  (torch's reducer does ``grad * 1/W`` into the bucket and copies back,
  SURVEY.md §2.4 K15).
* **Gradient sinks.**  Backward kernels that support it (the skinny Linear and
  the fused ConvNet plan) write weight gradients straight into their bucket
  slot (``ops/grad_sink.py``).
* **Averaging in the collective.**  Buckets are all-reduced with ``AVG``
  (``ncclAvg`` in RCCL) instead of being pre-scaled by 1/W in a separate pass.
* **Static bucket order** = reverse parameter order (the order gradients
  become ready), so there is no iteration-0 single-bucket pass and no bucket
  rebuild.
* **Native reducer.**  With this package's communicators (``rccl-native``,
  ``host``) — or at world size 1 — bucket bookkeeping runs in C++
  (``csrc/comm/reducer.cpp``): AccumulateGrad post-hooks, per-bucket ready
  counters, all-reduce launch on the comm stream and the end-of-backward
  stream fence, with no Python on the backward path.  With torch's own
  process groups (``nccl``/``gloo``) the same logic runs from Python hooks.
* Buckets follow torch's size rule (add a tensor, close the bucket once it
  reaches ``bucket_cap_mb``, default 25), which for the ConvNet gives the
  measured reference layout ``[[fc.bias, fc.weight], [8 conv/BN tensors]]``:
  the 720 MB fc gradient goes out as soon as the fc backward finishes and
  overlaps the whole conv backward.
"""
from __future__ import annotations

import contextlib
import hashlib
import weakref
from typing import List, Optional

import torch
import torch.nn as nn

from ..ops import grad_sink
from . import distributed as tdist
from . import factored

class _weak_call:
    """``obj.<name>`` as a callable that holds ``obj`` weakly (a no-op once it is gone).  Hooks and
    providers attached to parameters or to autograd nodes must not keep the wrapper alive: the
    cycle parameter -> hook -> wrapper -> module -> parameter runs through C++ that Python's
    collector cannot see, and every model built after it would find its predecessor's buffers
    still allocated (round 6: 0.72 GB per ConvNet at 3000^2, tools/oom_demo.py).  ``__self__``
    names the live owner as a bound method's does (ops/optim.py finds the deferred runner's owner
    through it)."""

    __slots__ = ("_ref", "_name")

    def __init__(self, obj, name: str):
        self._ref = weakref.ref(obj)
        self._name = name

    @property
    def __self__(self):
        return self._ref()

    def __call__(self, *args):
        o = self._ref()
        return None if o is None else getattr(o, self._name)(*args)


_ALIGN_ELEMS = 64  # 256-byte alignment of every parameter slot in the flat buffers


def _ext_loaded() -> bool:
    from .. import _ext

    return bool(_ext.load())


def _align(n: int) -> int:
    return (n + _ALIGN_ELEMS - 1) // _ALIGN_ELEMS * _ALIGN_ELEMS


class _Bucket:
    __slots__ = ("index", "params", "offset", "numel", "pending", "work", "ready", "skip")

    def __init__(self, index, offset):
        self.index, self.params, self.offset, self.numel = index, [], offset, 0
        self.pending, self.work, self.ready, self.skip = 0, None, False, False


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, device_ids=None, output_device=None, broadcast_buffers: bool = True,
                 process_group=None, bucket_cap_mb: Optional[float] = None, find_unused_parameters: bool = False,
                 gradient_as_bucket_view: bool = True, flat_params: bool = True, static_graph: bool = False,
                 reducer: str = "auto", grad_exchange: str = "auto", overlap_optimizer: bool = False,
                 fuse_update_in_backward: bool = True, keep_fused_grads: bool = False,
                 allreduce_chunks: Optional[int] = None, exchange_compress: bool = True,
                 exchange_groups: Optional[int] = None, exchange_source: str = "pooled"):
        super().__init__()
        self.module = module
        self.device_ids = device_ids
        self.broadcast_buffers = broadcast_buffers
        self.process_group = process_group
        self.find_unused_parameters = find_unused_parameters
        self.world_size = tdist.get_world_size(process_group)
        self.rank = tdist.get_rank(process_group)
        self.require_backward_grad_sync = True
        self._params: List[nn.Parameter] = [p for p in module.parameters() if p.requires_grad]
        if not self._params:
            raise RuntimeError("DistributedDataParallel: module has no parameters that require grad")
        dev = self._params[0].device
        dtype = self._params[0].dtype
        for p in self._params:
            if p.device != dev or p.dtype != dtype:
                raise RuntimeError("DistributedDataParallel: all parameters must share one device and dtype")
        self.device = dev
        self._verify_param_shapes()

        # ---- flat layout in gradient-ready order (reverse definition order)
        if grad_exchange not in ("auto", "allreduce", "activations", "sharded", "chunked"):
            raise ValueError(f"grad_exchange must be auto|allreduce|activations|sharded|chunked, got {grad_exchange!r}")
        self.grad_exchange = grad_exchange
        # K-chunked all-reduce of a big layer's weight gradient (parallel/factored.py, "chunked"):
        # default 4 chunks on the GPU, off on the CPU
        if allreduce_chunks is None:
            allreduce_chunks = 4 if dev.type == "cuda" else 1
        self.allreduce_chunks = max(1, int(allreduce_chunks))
        if grad_exchange == "chunked" and self.allreduce_chunks < 2:
            raise ValueError("grad_exchange='chunked' needs allreduce_chunks >= 2")
        big_layers = self._exchange_candidates(module)
        exch_layers = big_layers if grad_exchange != "allreduce" else []  # "allreduce": the plain bucket path
        layer_of = {id(p): lyr for lyr in big_layers for p in (lyr.weight, lyr.bias) if p is not None}
        order = list(reversed(self._params))
        cap_mb = 25.0 if bucket_cap_mb is None else float(bucket_cap_mb)
        limit = max(1, int(cap_mb * 1024 * 1024 // self._params[0].element_size()))
        # bucket membership, in gradient-ready order (torch's _compute_bucket_assignment_by_size)
        self._buckets: List[_Bucket] = []
        self._layer_bucket = {}  # id(exchange-candidate layer) -> bucket
        cur, size = _Bucket(0, 0), 0
        for p in order:
            n = p.numel()
            lyr = layer_of.get(id(p))
            if lyr is not None:
                # an activation-exchange candidate gets a bucket of its own (weight + bias only)
                lb = self._layer_bucket.get(id(lyr))
                if lb is None:
                    if cur.params:
                        self._buckets.append(cur)
                        cur, size = _Bucket(len(self._buckets), 0), 0
                    lb = cur
                    self._layer_bucket[id(lyr)] = lb
                lb.params.append(p)
                if len(lb.params) == sum(q is not None for q in (lyr.weight, lyr.bias)):
                    self._buckets.append(lb)
                    cur, size = _Bucket(len(self._buckets), 0), 0
                continue
            cur.params.append(p)
            size += _align(n)
            if size >= limit:
                self._buckets.append(cur)
                cur, size = _Bucket(len(self._buckets), 0), 0
        if cur.params:
            self._buckets.append(cur)
        # offsets: the big layers' buckets go last, each with its weight after its bias, so their
        # weight slots form the tail of the flat layout.  The gradient buffer starts without that
        # tail (``_lazy_from``): at world size 1 the fc weight steps inside its backward kernel and
        # on the exchange paths its update is formed in the exchange, so its 720 MB slot (39 GiB at
        # 23000^2) is only allocated when some path writes a gradient there (_slot / the
        # native reducer's grow()).  Bucket indices keep the ready order above.
        big = {id(b) for b in self._layer_bucket.values()}
        self._slots = {}  # id(param) -> (offset, numel)
        off = 0
        lazy_from = None
        for b in [b for b in self._buckets if id(b) not in big] + [b for b in self._buckets if id(b) in big]:
            b.offset = off
            if id(b) in big:
                b.params.sort(key=lambda q: q.dim() >= 2)  # bias (if any) first, then the weight
            for p in b.params:
                if id(b) in big and p.dim() >= 2 and lazy_from is None:
                    lazy_from = off
                self._slots[id(p)] = (off, p.numel())
                off += _align(p.numel())
            b.numel = off - b.offset
        self._total = off
        self._lazy_from = off if lazy_from is None else lazy_from
        self._bucket_of = {id(p): b for b in self._buckets for p in b.params}

        self._native = None
        self._retired_grads = []
        with torch.no_grad():
            self._flat_grad = torch.zeros(self._lazy_from, device=dev, dtype=dtype)
            if flat_params:
                # one parameter at a time, the big weights first: copy, re-point, and the original's
                # block goes back to the caching allocator -- the flat buffer and at most one
                # original are held together (the gradient tail above is not allocated yet)
                self.flat_param = torch.zeros(self._total, device=dev, dtype=dtype)
                for p in sorted(order, key=lambda q: -q.numel()):
                    o, n = self._slots[id(p)]
                    self.flat_param[o:o + n].copy_(p.detach().reshape(-1))
                    p.data = self.flat_param[o:o + n].view_as(p)
            else:
                self.flat_param = None

        # ---- rank-0 state broadcast: one call for all params
        self._sync_module_states()

        # ---- gradient sinks + readiness hooks
        for p in self._params:
            grad_sink.register(p, self._make_view_fn(p))
        self._callback_queued = False
        self._native = self._make_native_reducer(reducer)
        if self._native is None:
            self._hooks = [p.register_post_accumulate_grad_hook(_weak_call(self, "_on_grad_ready")) for p in self._params]
        else:
            self._hooks = []
            self._native.attach(self._params)

        # ---- activation exchange for huge skinny Linear layers (parallel/factored.py)
        self._exchanges = []
        forced = grad_exchange in ("activations", "sharded", "chunked")
        if exch_layers and (self.world_size > 1 or (forced and tdist.is_initialized())):
            for lyr in exch_layers:
                b = self._layer_bucket[id(lyr)]
                self._exchanges.append(factored.ActivationExchange(
                    lyr.weight, lyr.bias, process_group, self.world_size, grad_exchange,
                    self._make_skip_fn(b), self._make_view_fn(lyr.weight),
                    self._make_view_fn(lyr.bias) if lyr.bias is not None else None, chunks=self.allreduce_chunks,
                    compress=exchange_compress,
                    # column groups of the zero-suppressed activation exchange: they start its gathers
                    # a group's head launch in (earlier window) for ~0.2 ms of launch and tail cost at
                    # the bench shape, worth it only when links carry the rows (world > 1)
                    groups=exchange_groups if exchange_groups else (4 if self.world_size > 1 else 1),
                    # the fused head's pooled input instead of the fc rows X (factored.py "pooled")
                    source=exchange_source))

        # ---- overlapped optimizer: the big layers' buckets finish (collective + SGD
        # update) on a side stream while the next forward's convolutions run
        self.overlap_optimizer = bool(overlap_optimizer) and dev.type == "cuda" and self.flat_param is not None
        self.fuse_update_in_backward = bool(fuse_update_in_backward)
        # a parameter updated inside its backward kernel gets no .grad unless asked (torch's
        # optimizer-in-backward semantics; ops/fused_update.py)
        self.keep_fused_grads = bool(keep_fused_grads)
        self._param_index = {id(p): i for i, p in enumerate(self._params)}
        self._fused_done = set()  # ids of params whose step ran inside their backward kernel
        self._deferred: List[_Bucket] = []
        self._deferred_works = {}
        self.last_deferred_inline = False  # the last step's deferred leftovers went into the optimizer's sweep
        self._side = None
        if self.overlap_optimizer and big_layers:
            # with CUs split off for the collectives (utils/streams.py) the side work keeps to the
            # reserved CUs, off the persistent compute kernels' CUs (TDS_SIDE_CUS=compute|any)
            from ..utils.streams import side_stream

            self._side = (side_stream(dev) if _ext_loaded() else None) or torch.cuda.Stream(device=dev)
            self._deferred = [self._layer_bucket[id(lyr)] for lyr in big_layers]
            for b in self._deferred:
                if self._native is not None:
                    self._native.set_bucket_deferred(b.index, True)
            for ex in self._exchanges:
                ex.side_stream = self._side

    def _make_native_reducer(self, mode: str):
        if mode not in ("auto", "native", "python"):
            raise ValueError(f"reducer must be auto|native|python, got {mode!r}")
        if mode == "python":
            return None
        from .. import _ext
        from .rccl_backend import native_comm_of

        comm, kind = native_comm_of(self.process_group) if self.world_size > 1 else (None, None)
        if self.world_size > 1 and comm is None:
            if mode == "native":
                raise RuntimeError("reducer='native' needs a native process group (backend rccl-native or host)")
            return None  # torch's own PG (nccl/gloo): Python hooks drive it
        if not _ext.load():
            if mode == "native" or self.device.type == "cuda":
                _ext.ops()  # raises with the load error
            return None
        idx = {id(p): i for i, p in enumerate(self._params)}
        ps = torch.zeros(len(self._params), 3, dtype=torch.int64)
        for b in self._buckets:
            for p in b.params:
                o, n = self._slots[id(p)]
                ps[idx[id(p)]] = torch.tensor([o, n, b.index])
        bs = torch.tensor([[b.offset, b.numel] for b in self._buckets], dtype=torch.int64)
        r = _ext.classes().Reducer(self._flat_grad, ps, bs, bool(self.find_unused_parameters))
        if kind == "rccl":
            r.set_rccl_comm(comm)
            self._rccl_comm = comm
        elif kind == "host":
            r.set_host_comm(comm)
        return r

    @property
    def reducer_kind(self) -> str:
        return "native" if self._native is not None else "python"

    def fc_grad_path(self) -> str:
        """How the big fc layer's gradient was averaged in the steps run so far."""
        used = sorted({ex.last_path for ex in self._exchanges if ex.last_path})
        if used:  # (at world 1 only when an exchange was forced)
            return "+".join(used)
        return "local" if self.world_size == 1 else "allreduce"

    # ------------------------------------------------------------------ setup helpers
    @staticmethod
    def _exchange_candidates(module):
        """This package's Linear layers (their forward routes through ops.functional.linear /
        the fused head, which implement the exchange) big enough that exchanging activations
        can beat all-reducing the weight gradient; the decision itself is made per step
        from the batch rows."""
        from ..ops.modules import Linear as TdsLinear

        out = []
        for m in module.modules():
            if isinstance(m, TdsLinear):
                w, b = m.weight, m.bias
                if w.requires_grad and w.numel() >= (1 << 20) and w.shape[0] <= 16 and (b is None or b.requires_grad):
                    out.append(m)
        return out

    def _make_skip_fn(self, b: _Bucket):
        ref = weakref.ref(self)

        def set_skip(flag: bool):
            b.skip = bool(flag)
            s = ref()
            if s is not None and s._native is not None:
                s._native.set_bucket_skip(b.index, bool(flag))

        return set_skip

    @property
    def exchanges(self):
        return list(self._exchanges)

    @property
    def flat_grad(self) -> torch.Tensor:
        """The flat gradient buffer as it is now: without the big layers' weight slots until a
        path writes a gradient there (see ``_lazy_from``); ``grad_view`` / the gradient sinks
        grow it on demand."""
        if self._native is not None:
            return self._native.flat_grad()
        return self._flat_grad

    def _grow_flat_grad(self):
        """Storage for the whole layout: a new buffer, the resident prefix copied, every .grad
        that viewed the old buffer re-pointed (in-place collectives on it are ordered first)."""
        if self._native is not None:
            self._native.grow()
            return
        old = self._flat_grad
        if old.numel() >= self._total:
            return
        for b in self._buckets:
            if b.work is not None:
                b.work.wait()
        with torch.no_grad():
            new = torch.zeros(self._total, device=old.device, dtype=old.dtype)
            new[:old.numel()].copy_(old)
            ptr = old.untyped_storage().data_ptr()
            for p in self._params:
                if p.grad is not None and p.grad.untyped_storage().data_ptr() == ptr:
                    o, n = self._slots[id(p)]
                    p.grad = new.narrow(0, o, n).view(p.shape)
        self._retired_grads.append(old)  # a queued collective may still read it
        self._flat_grad = new

    def grad_storage_bytes(self) -> int:
        """Bytes of gradient storage allocated so far (the layout may be larger, ``_total``)."""
        return self.flat_grad.numel() * self.flat_grad.element_size()

    def _slot(self, o: int, n: int) -> torch.Tensor:
        if o + n > self.flat_grad.numel():
            self._grow_flat_grad()
        return self.flat_grad.narrow(0, o, n)

    def _make_view_fn(self, p):
        o, n = self._slots[id(p)]
        shape = p.shape
        ref = weakref.ref(self)

        def view():  # (None once the wrapper is gone: grad_sink.acquire then returns a plain tensor)
            s = ref()
            return None if s is None else s._slot(o, n).view(shape)

        return view

    def grad_view(self, p):
        o, n = self._slots[id(p)]
        return self._slot(o, n).view(p.shape)

    def _verify_param_shapes(self):
        """Same check as torch's _verify_param_shape_across_processes (C4): a hash
        of every parameter shape, compared with MAX/MIN all-reduces."""
        if self.world_size == 1:
            return
        h = hashlib.sha1(repr([tuple(p.shape) for p in self._params]).encode()).digest()
        v = int.from_bytes(h[:7], "little")
        dev = self.device if self.device.type == "cuda" else torch.device("cpu")
        t = torch.tensor([v, -v], dtype=torch.int64, device=dev)
        tdist.all_reduce(t, tdist.ReduceOp.MAX, group=self.process_group)
        if int(t[0].item()) != v or int(t[1].item()) != -v:
            raise RuntimeError("DistributedDataParallel: parameter shapes differ across ranks")

    def _sync_module_states(self):
        if self.world_size == 1:
            return
        with torch.no_grad():
            if self.flat_param is not None:
                tdist.broadcast(self.flat_param, 0, group=self.process_group)
            else:
                for p in self._params:
                    tdist.broadcast(p.data, 0, group=self.process_group)
            self._broadcast_buffers_now()

    def _broadcast_buffers_now(self):
        bufs = [b for b in self.module.buffers() if b is not None]
        if not bufs:
            return
        comm = getattr(self, "_rccl_comm", None)
        if comm is not None and all(b.is_contiguous() and b.is_cuda for b in bufs):
            # one grouped RCCL launch, no flatten/copy-back
            comm.broadcast_coalesced(bufs, 0).wait()
            return
        by_dtype = {}
        for b in bufs:
            by_dtype.setdefault((b.dtype, b.device), []).append(b)
        for (_, _), group in by_dtype.items():
            flat = torch.cat([b.reshape(-1) for b in group])
            tdist.broadcast(flat, 0, group=self.process_group)
            o = 0
            for b in group:
                n = b.numel()
                b.copy_(flat[o:o + n].view_as(b))
                o += n

    # ------------------------------------------------------------------ preflight
    def preflight(self, rows: int, timed) -> dict:
        """Issue once, on the live process group and its streams, every collective a synchronised
        training step with ``rows`` local rows will run -- the rank-0 buffer broadcast, the
        all-reduce of every bucket the fc gradient path leaves to the reducer, and each exchange's
        own collectives (parallel/factored.py ``preflight``) -- each through ``timed(name,
        nbytes, kind, issue)`` (see bench.py ``_preflight``: a bounded wait and a time per
        collective).  RCCL sets up its point-to-point channels and algorithms on first use, so
        that cost (and any failure) lands here instead of in the first training step.  Returns
        {"fc_path": ...}."""
        if self.world_size == 1 and not self._exchanges:
            return {"fc_path": "local"}
        g = self.process_group
        paths = {}
        for ex in self._exchanges:
            paths[id(self._bucket_of[id(ex.weight)])] = ex.preflight(rows, timed)
        if self.broadcast_buffers and self.world_size > 1 and any(True for _ in self.module.buffers()):
            nb = sum(b.numel() * b.element_size() for b in self.module.buffers())
            timed("BN buffer broadcast (coalesced)", nb, "broadcast", lambda: self._broadcast_buffers_now())
        for b in self._buckets:
            if paths.get(id(b)) is not None or self.world_size == 1:
                continue  # this bucket's gradient travels by its exchange (world 1: no all-reduce)
            seg = torch.zeros(b.numel, device=self.device, dtype=self.flat_grad.dtype)
            timed(f"bucket {b.index} all-reduce (AVG)", b.numel * seg.element_size(), "all_reduce",
                  lambda seg=seg: tdist.all_reduce(seg, tdist.ReduceOp.AVG, group=g, async_op=True))
            del seg
        used = [p for p in paths.values() if p is not None]
        return {"fc_path": "+".join(used) if used else "allreduce"}

    # ------------------------------------------------------------------ forward
    def forward(self, *args, **kwargs):
        if self.broadcast_buffers and self.world_size > 1:
            with torch.no_grad():
                self._broadcast_buffers_now()  # C6: rank-0 BN running stats each forward
        if self._native is not None:
            self._native.prepare_for_backward(bool(self.require_backward_grad_sync))
        else:
            self._reset_bucket_state()
        sync = bool(self.require_backward_grad_sync) and torch.is_grad_enabled()
        for ex in self._exchanges:
            ex.arm(sync)
        return self.module(*args, **kwargs)

    @contextlib.contextmanager
    def no_sync(self):
        old = self.require_backward_grad_sync
        self.require_backward_grad_sync = False
        try:
            yield
        finally:
            self.require_backward_grad_sync = old

    # ------------------------------------------------------------------ backward
    def _reset_bucket_state(self):
        for b in self._buckets:
            b.pending = len(b.params)
            b.work = None
            b.ready = False
        self._callback_queued = False

    def _on_grad_ready(self, p):
        o, n = self._slots[id(p)]
        view = self._slot(o, n)
        g = p.grad
        if g is None:
            return
        if not (g.data_ptr() == view.data_ptr() and g.is_contiguous()):
            # a producer without a sink: copy into the bucket once and re-point .grad
            with torch.no_grad():
                view.copy_(g.reshape(-1))
            p.grad = view.view(p.shape)
        if not self._callback_queued:
            self._callback_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize_backward)
        b = self._bucket_of[id(p)]
        if b.skip:
            return
        b.pending -= 1
        if b.pending == 0:
            self._launch(b)

    def _launch(self, b: _Bucket):
        b.ready = True
        if self.world_size == 1 or not self.require_backward_grad_sync:
            return
        seg = self._slot(b.offset, b.numel)
        b.work = tdist.all_reduce(seg, tdist.ReduceOp.AVG, group=self.process_group, async_op=True)

    def _finalize_backward(self):
        for b in self._buckets:
            if not b.ready and not b.skip:
                if not self.find_unused_parameters:
                    missing = [i for i, p in enumerate(b.params) if p.grad is None]
                    raise RuntimeError(
                        f"DistributedDataParallel: bucket {b.index} never became ready ({len(missing)} params got no "
                        "gradient); pass find_unused_parameters=True if parts of the model are unused")
                # unused params: their slots hold zeros / stale values -> zero and launch
                for p in b.params:
                    if p.grad is None:
                        v = self.grad_view(p)
                        v.zero_()
                        p.grad = v
                self._launch(b)
        deferred = {id(b) for b in self._deferred}
        for b in self._buckets:
            if b.work is not None:
                if id(b) in deferred:
                    self._deferred_works[b.index] = b.work  # finished on the side stream (optimizer step)
                else:
                    b.work.wait()
                b.work = None
        self._callback_queued = False

    # ------------------------------------------------------------------ misc
    def bucket_layout(self):
        """[(bucket index, bytes, [param shapes])] — for tests and logs."""
        return [(b.index, b.numel * self.flat_grad.element_size(), [tuple(p.shape) for p in b.params])
                for b in self._buckets]

    def attach_optimizer(self, optimizer):
        """Let ``ops.optim.SGD`` update the flat buffer in one sweep (and, with
        ``overlap_optimizer``, hand the deferred buckets' update to the side stream).
        At world size 1 the deferred big weights' plain-SGD step is fused into their
        backward kernel instead (ops/fused_update.py): nothing to average, and the
        kernel already holds the weight and its gradient."""
        if self.flat_param is not None and hasattr(optimizer, "set_flat_buffers"):
            ref = weakref.ref(self)
            optimizer.set_flat_buffers(self.flat_param, lambda: ref().flat_grad, self._params)
            if self._deferred and hasattr(optimizer, "set_deferred"):
                optimizer.set_deferred([(b.offset, b.numel) for b in self._deferred],
                                       _weak_call(self, "_run_deferred_update"),
                                       lambda p: ref() is not None and id(p) in ref()._fused_done)
                if self.fuse_update_in_backward and (self.world_size == 1 or self._exchanges):
                    self._register_fused_updates(optimizer)
        return optimizer

    def _register_fused_updates(self, optimizer):
        from ..ops import fused_update

        def plain_sgd_lr():
            if len(optimizer.param_groups) != 1:
                return None
            g = optimizer.param_groups[0]
            if g.get("momentum", 0.0) != 0.0 or g.get("weight_decay", 0.0) != 0.0 or g.get("nesterov", False):
                return None
            if g.get("maximize", False):
                return None
            return float(g["lr"])

        ref = weakref.ref(self)
        for b in self._deferred:
            for p in b.params:
                if p.dim() < 2:
                    continue  # biases: tiny, updated by the optimizer as usual

                def provider(what, p=p):
                    self = ref()  # (the provider lives on the parameter: no strong reference back)
                    if self is None:
                        return None
                    if what == "keep_grad":
                        return self.keep_fused_grads
                    if what in ("applied", "applied_no_grad"):
                        self._fused_done.add(id(p))
                        if what == "applied_no_grad":
                            self._mark_ready_without_grad(p)
                        return None
                    # only a plain synchronised step whose gradient lands straight in the bucket;
                    # a local gradient ("query") only at world size 1, the exchange's averaged one
                    # ("query_exchange", parallel/factored.py) at any world size
                    if what == "query" and self.world_size != 1:
                        return None
                    if what == "query_exchange" and self.keep_fused_grads:
                        return None
                    if not self.require_backward_grad_sync or p.grad is not None or id(p) in self._fused_done:
                        return None
                    return plain_sgd_lr()

                fused_update.register(p, provider)

    def _mark_ready_without_grad(self, p):
        """Count ``p`` as ready for its bucket although autograd produced no gradient for it
        (its update ran in the backward kernel, ops/fused_update.py)."""
        if self._native is not None:
            self._native.mark_ready(self._param_index[id(p)])
            return
        if not self._callback_queued:
            self._callback_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize_backward)
        b = self._bucket_of[id(p)]
        if b.skip:
            return
        b.pending -= 1
        if b.pending == 0:
            self._launch(b)

    # (leftovers of the deferred buckets at most this many elements, with no collective behind them,
    # are updated inline by the optimizer's own sweep: at world size 1 the fc weight's step runs in
    # its backward kernel and only the fc bias is left -- on the side stream it cost the next head
    # forward a cross-stream wait, an ~11 us gap in the step's timeline, r5_s36)
    _INLINE_DEFERRED_MAX = 1 << 16

    def take_inline_deferred(self):
        """Flat (offset, numel) ranges of the deferred buckets the optimizer should update in its
        own sweep on the current stream this step (see _INLINE_DEFERRED_MAX); they are skipped by
        _run_deferred_update, which then fences only what it updates itself."""
        self._inline_done = set()
        if self.world_size != 1 or not self._deferred:
            return []
        left = [p for b in self._deferred for p in b.params if id(p) not in self._fused_done]
        if not left or sum(p.numel() for p in left) > self._INLINE_DEFERRED_MAX:
            return []
        self._inline_done = {id(p) for p in left}
        return [self._slots[id(p)] for p in left]

    def _run_deferred_update(self, update_fn):
        """Finish the deferred buckets on the side stream: wait for this step's
        backward (compute stream) and the bucket collective, apply ``update_fn(offset,
        numel)`` (the optimizer's flat-slice update), then fence the parameters so
        their first reader in the next forward waits (ops/param_fence.py).

        Contract with the optimizer (``ops.optim.SGD.step``, which finds this runner's owner
        through ``runner.__self__``): per step, the optimizer MAY call ``take_inline_deferred()``
        first and step the returned ranges in its own sweep on the current stream; it then MUST
        call this runner in the same step.  Both consume the step's state (``_fused_done``,
        ``_inline_done``).  A runner call without a preceding ``take_inline_deferred()`` (any other
        optimizer) updates everything not stepped in its backward here, on the side stream.  Fast
        path: when every deferred parameter was stepped in its backward or inline, no side work is
        queued and no fence is set (``last_deferred_inline``).  Tests:
        tests/test_param_fence_cpu.py."""
        from ..ops import param_fence

        cur = torch.cuda.current_stream(self.device)
        side = self._side
        done, self._fused_done = self._fused_done, set()
        inline, self._inline_done = getattr(self, "_inline_done", set()), set()
        works = {}
        for b in self._deferred:
            w = self._deferred_works.pop(b.index, None)
            if w is None and self._native is not None:
                w = self._native.take_work(b.index)
            works[b.index] = w
        self.last_deferred_inline = bool(inline) and all(w is None for w in works.values()) and all(
            id(p) in done or id(p) in inline for b in self._deferred for p in b.params)
        if self.last_deferred_inline:
            return  # everything was stepped in its backward or inline by the optimizer: no side work, no fence
        done = done | inline
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for b in self._deferred:
                w = works[b.index]
                if w is not None:
                    w.wait()  # side stream waits for the bucket all-reduce
                if not done:
                    self._slot(b.offset, b.numel)  # (storage for the whole bucket)
                    update_fn(b.offset, b.numel)
                    continue
                for p in b.params:  # the backward already stepped some of them
                    if id(p) not in done:
                        off, n = self._slots[id(p)]
                        update_fn(off, n)
            ev = torch.cuda.Event()
            ev.record(side)
        for b in self._deferred:
            for p in b.params:
                param_fence.set(p, ev)

    def wait_pending_updates(self):
        """Order the current stream after any deferred parameter update (call before
        reading the parameters outside the model's forward, e.g. checkpointing)."""
        from ..ops import param_fence

        for b in self._deferred:
            for p in b.params:
                param_fence.wait(p)
