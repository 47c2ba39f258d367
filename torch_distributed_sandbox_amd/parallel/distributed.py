"""torch.distributed-style process-group API.

Same call surface the reference uses — ``init_process_group``, ``new_group``,
``all_reduce``, ``barrier``, ``destroy_process_group``, ``ReduceOp`` — plus the
collectives DDP needs (``broadcast``, ``all_gather``, ``reduce_scatter``).

Backends
--------
``"rccl"`` / ``"nccl"``  device collectives over RCCL/xGMI (torch's ProcessGroupNCCL
                         *is* RCCL on ROCm).  One process per GPU.
``"gloo"``               CPU collectives (tests / CPU rehearsals).
``"host"``               this package's C++ TCP ring backend (``csrc/comm``),
                         registered with torch.distributed as a custom backend.
``"rccl-native"``        this package's C++ RCCL communicator (own comm stream,
                         event works, watchdog/abort; ``parallel/rccl_backend.py``).
``None`` / ``"auto"``     ``rccl-native`` when a GPU is visible, else ``gloo``
                         (the reference's auto-switch, test_init.py:84-88).

Fixes vs the reference (documented deviations):

* ``new_group(ranks)`` is cached by (ranks, backend): the reference creates a
  new communicator every step (allreduce_toy.py:26-27, mnist_distributed.py:99-100);
  we keep its semantics (all ranks must call it) without the per-step init.
* ``init_method`` / ``MASTER_ADDR`` / ``MASTER_PORT`` are honoured for
  multi-node (the reference hard-codes loopback, mnist_distributed.py:124-125).
"""
from __future__ import annotations

import datetime
import os
import warnings
from typing import Optional, Sequence

import torch
import torch.distributed as dist

DEFAULT_TIMEOUT = datetime.timedelta(minutes=10)  # torch's default_pg_nccl_timeout


class ReduceOp:
    SUM = dist.ReduceOp.SUM
    AVG = dist.ReduceOp.AVG
    MAX = dist.ReduceOp.MAX
    MIN = dist.ReduceOp.MIN
    PRODUCT = dist.ReduceOp.PRODUCT


_state = {
    "backend": None,  # normalised backend name
    "groups": {},  # (ranks tuple, backend) -> ProcessGroup
}


def default_backend(on_gpu: Optional[bool] = None) -> str:
    """The tuned stack every entry point uses unless told otherwise (bench.py, the trainers,
    the toy): this package's RCCL communicator + C++ reducer on the GPU, gloo on the CPU."""
    if on_gpu is None:
        on_gpu = torch.cuda.is_available()
    return "rccl-native" if on_gpu else "gloo"


def is_device_backend(backend: Optional[str]) -> bool:
    """Does ``backend`` move device (GPU) tensors (RCCL: torch's or this package's)?"""
    return _normalise_backend(backend) in ("rccl", "rccl-native")


def _normalise_backend(backend: Optional[str]) -> str:
    if backend is None or backend == "auto":
        return default_backend()
    b = backend.lower()
    if b in ("nccl", "rccl", "cuda", "hip"):
        return "rccl"
    if b in ("gloo", "cpu"):
        return "gloo"
    if b == "host":
        return "host"
    if b in ("rccl-native", "rccl_native", "tds_rccl", "native"):
        return "rccl-native"
    raise ValueError(f"unknown backend {backend!r} (expected rccl|nccl|gloo|host|rccl-native)")


def _torch_backend(b: str) -> str:
    if b == "rccl":
        return "nccl"
    if b == "host":
        from . import host_backend

        host_backend.register()
        return host_backend.BACKEND_NAME
    if b == "rccl-native":
        from . import rccl_backend

        return rccl_backend.register()
    return b


def is_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def init_process_group(backend: Optional[str] = None, init_method: Optional[str] = None, rank: Optional[int] = None,
                       world_size: Optional[int] = None, timeout: datetime.timedelta = DEFAULT_TIMEOUT,
                       device_id: Optional[int] = None, store=None, comm_cus: Optional[int] = None) -> None:
    """Initialise the default group.  ``rank``/``world_size`` default to the
    ``RANK``/``WORLD_SIZE`` environment (torchrun); ``init_method`` defaults to
    ``env://`` (``MASTER_ADDR``/``MASTER_PORT``), which rendezvouses through this package's
    C++ TCP store (parallel/store.py ``rendezvous``: c10d's store at ``MASTER_ADDR:MASTER_PORT``
    only locates it, and is the agreed fallback if it cannot be used on some rank).
    ``store="c10d"`` / ``TDS_STORE=c10d``, an explicit ``init_method`` or a
    ``torch.distributed.Store`` object use that instead; so does ``backend="rccl"`` (torch's
    ProcessGroupNCCL: torch's stack top to bottom, bench.py's fallback tiers).  ``store_kind()``
    reports which store the group rendezvoused on.

    ``comm_cus`` (``rccl-native`` only): CUs split off for communication
    (utils/streams.py, docs/DISTRIBUTED.md) -- a CU-masked compute stream is made
    current on this thread and the communicator's stream is confined to the other
    CUs, with RCCL's CTAs bounded to the same count.  Default (None):
    ``TDS_COMM_CUS`` or 32 at world size > 1, 0 at world size 1."""
    b = _normalise_backend(backend)
    if rank is None:
        rank = int(os.environ.get("RANK", "0"))
    if world_size is None:
        world_size = int(os.environ.get("WORLD_SIZE", "1"))
    _state["comm_cus"] = 0
    kind = "c10d" if init_method is not None else "given"
    if store is None and init_method is None:
        store = "c10d" if b == "rccl" else os.environ.get("TDS_STORE", "native") or "native"
    if isinstance(store, str):
        if store not in ("native", "c10d"):
            raise ValueError(f"unknown store {store!r} (expected 'native', 'c10d' or a torch.distributed.Store)")
        from .store import rendezvous

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        store, kind = rendezvous(rank, world_size, timeout=timeout, prefer=store)
    kwargs = dict(backend=_torch_backend(b), rank=rank, world_size=world_size, timeout=timeout)
    if store is not None:
        kwargs["store"] = store
    else:
        if init_method is None:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            init_method = "env://"
        kwargs["init_method"] = init_method
    if b in ("rccl", "rccl-native"):
        if device_id is None:
            device_id = int(os.environ.get("LOCAL_RANK", rank % max(1, torch.cuda.device_count())))
        torch.cuda.set_device(device_id)
        if b == "rccl":
            # eager communicator init (bound to this GPU) instead of lazy first-collective init
            kwargs["device_id"] = torch.device("cuda", device_id)
        # (rccl-native always creates its communicator eagerly in the backend constructor)
    if b == "rccl-native":
        if comm_cus is None:
            comm_cus = int(os.environ.get("TDS_COMM_CUS", "32")) if world_size > 1 else 0
        if comm_cus > 0:
            from ..utils.streams import reserve_cus_for_comm

            if comm_cus % 32:
                raise ValueError(f"comm_cus must be a multiple of 32 (one CU per shader engine), got {comm_cus}")
            # before the communicator exists: its stream takes the complement mask
            try:
                stream = reserve_cus_for_comm(comm_cus, torch.device("cuda", device_id))
            except RuntimeError as e:  # no CU masking here: run unsplit
                warnings.warn(f"init_process_group: CU split of {comm_cus} CUs unavailable ({e}); "
                              "collectives share the CUs with the compute")
                reserve_cus_for_comm(0)
            else:
                if "TDS_RCCL_MAX_CTAS" not in os.environ:
                    os.environ["TDS_RCCL_MAX_CTAS"] = str(comm_cus)
                    _state["set_max_ctas"] = True
                _state["prev_stream"] = torch.cuda.current_stream(device_id)
                torch.cuda.set_stream(stream)
                _state["comm_cus"] = comm_cus
    try:
        dist.init_process_group(**kwargs)
    except BaseException:
        _undo_cu_split()
        raise
    _state["backend"] = b
    _state["groups"] = {}
    _state["store_kind"] = kind
    _state["store"] = store  # (rank 0 serves it: alive as long as the group)


def store_kind() -> Optional[str]:
    """The store the default group rendezvoused on: "native" (parallel/store.py), "c10d",
    "c10d (fallback: ...)", or "given" (a store object passed in)."""
    return _state.get("store_kind") if is_initialized() else None


def _undo_cu_split() -> None:
    """Reverse what init_process_group's CU split changed in this process: the persistent
    kernels' CU reserve, the current (CU-masked) stream and a TDS_RCCL_MAX_CTAS it exported."""
    if _state.pop("set_max_ctas", False):
        os.environ.pop("TDS_RCCL_MAX_CTAS", None)
    prev = _state.pop("prev_stream", None)
    if _state.get("comm_cus", 0):
        from .. import _ext

        _ext.ops().set_cu_reserve(0)
        if prev is not None:
            torch.cuda.set_stream(prev)
    _state["comm_cus"] = 0


def comm_cus() -> int:
    """CUs split off for communication by ``init_process_group`` (0: none)."""
    return int(_state.get("comm_cus", 0))


def destroy_process_group(group=None) -> None:
    if not is_initialized():
        return
    if group is None:
        # the native communicator ends here (torch's teardown shuts down only its own NCCL
        # backends): its comm stream, watchdog and buffers go before the CU split is undone,
        # whatever Python references to it outlive the group
        from .rccl_backend import native_comm_of

        comm, kind = native_comm_of(None)
        if kind == "rccl" and hasattr(comm, "shutdown"):
            comm.shutdown()
        _state["groups"] = {}
        _state["backend"] = None
        dist.destroy_process_group()
        _undo_cu_split()
    else:
        for k, g in list(_state["groups"].items()):
            if g is group:
                del _state["groups"][k]
        dist.destroy_process_group(group)


def get_rank(group=None) -> int:
    return dist.get_rank(group) if is_initialized() else 0


def get_world_size(group=None) -> int:
    return dist.get_world_size(group) if is_initialized() else 1


def get_backend(group=None) -> Optional[str]:
    return _state["backend"] if is_initialized() else None


def new_group(ranks: Optional[Sequence[int]] = None, backend: Optional[str] = None, timeout=DEFAULT_TIMEOUT):
    """Collective over the default group (like torch), cached by (ranks, backend)."""
    world = get_world_size()
    key_ranks = tuple(sorted(ranks)) if ranks is not None else tuple(range(world))
    b = _normalise_backend(backend) if backend is not None else _state["backend"]
    key = (key_ranks, b)
    g = _state["groups"].get(key)
    if g is None:
        if key_ranks == tuple(range(world)) and b == _state["backend"]:
            g = dist.group.WORLD
        else:
            g = dist.new_group(ranks=list(key_ranks), backend=_torch_backend(b), timeout=timeout)
        _state["groups"][key] = g
    return g


def _needs_avg_emulation(group) -> bool:
    b = dist.get_backend(group)
    return b not in ("nccl", "tds_host", "tds_rccl")


def all_reduce(tensor: torch.Tensor, op=ReduceOp.SUM, group=None, async_op: bool = False):
    """In-place all-reduce.  AVG is native on RCCL (ncclAvg) and on the host ring
    backend, and emulated as SUM + divide on gloo (which has no AVG)."""
    if op == ReduceOp.AVG and _needs_avg_emulation(group):
        work = dist.all_reduce(tensor, op=ReduceOp.SUM, group=group, async_op=async_op)
        n = get_world_size(group)
        if async_op:
            return _debug_sync(_PostOpWork(work, lambda: _div_(tensor, n)), "all_reduce", tensor)
        _div_(tensor, n)
        return _debug_sync(None, "all_reduce", tensor)
    return _debug_sync(dist.all_reduce(tensor, op=op, group=group, async_op=async_op), "all_reduce", tensor)


def debug_sync_enabled() -> bool:
    """TDS_DEBUG_SYNC=1: stream-ordering assertion mode.  Every collective
    issued through this module is waited for and the device synchronised right after it
    is enqueued, so an async fault or a missing stream fence surfaces at the collective that
    caused it.  The native RCCL communicator honours the same variable in C++
    (csrc/comm/rccl_comm.h), which also covers the C++ reducer's bucket all-reduces."""
    return os.environ.get("TDS_DEBUG_SYNC", "0") not in ("", "0")


def _debug_sync(work, what: str, tensor: torch.Tensor):
    if not debug_sync_enabled():
        return work
    if work is not None:
        work.wait()
    if tensor.is_cuda:
        try:
            torch.cuda.synchronize(tensor.device)
        except RuntimeError as e:
            raise RuntimeError(f"TDS_DEBUG_SYNC: {what} on rank {get_rank()}: {e}") from e
    return work


def _div_(t: torch.Tensor, n: int):
    if t.is_floating_point():
        t.div_(n)
    else:
        t.floor_divide_(n)


class _PostOpWork:
    def __init__(self, work, fn):
        self._work, self._fn, self._done = work, fn, False

    def wait(self, timeout=None):
        if timeout is None:
            self._work.wait()
        else:
            self._work.wait(timeout)
        if not self._done:
            self._fn()
            self._done = True
        return True

    def is_completed(self):
        return self._work.is_completed()


def broadcast(tensor: torch.Tensor, src: int = 0, group=None, async_op: bool = False):
    return _debug_sync(dist.broadcast(tensor, src=src, group=group, async_op=async_op), "broadcast", tensor)


def all_gather(tensor_list, tensor, group=None, async_op: bool = False):
    return _debug_sync(dist.all_gather(tensor_list, tensor, group=group, async_op=async_op), "all_gather", tensor)


def all_gather_into_tensor(output, input, group=None, async_op: bool = False):
    return _debug_sync(dist.all_gather_into_tensor(output, input, group=group, async_op=async_op),
                       "all_gather_into_tensor", output)


def reduce_scatter_tensor(output, input, op=ReduceOp.SUM, group=None, async_op: bool = False):
    return _debug_sync(dist.reduce_scatter_tensor(output, input, op=op, group=group, async_op=async_op),
                       "reduce_scatter_tensor", output)


class _DoneWork:
    def wait(self, timeout=None):
        return True

    def is_completed(self):
        return True


class _Works:
    def __init__(self, works):
        self._works = [w for w in works if w is not None]

    def wait(self, timeout=None):
        for w in self._works:
            w.wait()
        return True

    def is_completed(self):
        return all(w.is_completed() for w in self._works)


def sendrecv(sends, recvs, group=None, async_op: bool = True):
    """Grouped point-to-point exchange: ``sends``/``recvs`` are lists of
    ``(tensor, peer)``; chunks between one pair of ranks are matched in list order.
    Pairs with ``peer == rank`` are local copies.

    * ``rccl-native``: one ncclGroupStart/End of ncclSend/ncclRecv on the comm
      stream (``RcclComm.sendrecv``): every peer pair streams over its own xGMI link.
    * torch's ``nccl`` and ``gloo`` (CPU tensors): ``batch_isend_irecv``.
    * anything else (the ring-only ``host`` backend, gloo with GPU tensors in the
      one-GPU rehearsal): an all-gather of per-destination packed buffers — same
      result, more bytes; rehearsal paths only.
    """
    me = get_rank(group)
    local_s = [(t, p) for t, p in sends if p == me]
    local_r = [(t, p) for t, p in recvs if p == me]
    if len(local_s) != len(local_r):
        raise ValueError("sendrecv: self-sends and self-receives must pair up")
    for (src, _), (dst, _) in zip(local_s, local_r):
        dst.copy_(src)
    sends = [(t, p) for t, p in sends if p != me]
    recvs = [(t, p) for t, p in recvs if p != me]
    debug = debug_sync_enabled()
    from .rccl_backend import native_comm_of

    comm, kind = native_comm_of(group)
    if kind == "rccl":
        w = comm.sendrecv([t for t, _ in sends], [p for _, p in sends], [t for t, _ in recvs],
                          [p for _, p in recvs])
        w = _NativeWork(w)
        if debug or not async_op:
            w.wait()
            if debug:
                torch.cuda.synchronize()
        return w if async_op else None
    backend = dist.get_backend(group)
    all_cpu = all(t.device.type == "cpu" for t, _ in sends + recvs)
    if backend == "nccl" or (backend == "gloo" and all_cpu):
        ops = []
        tags = {}
        for t, p in sends:
            k = ("s", p)
            tags[k] = tags.get(k, -1) + 1
            ops.append(dist.P2POp(dist.isend, t.contiguous(), p, group=group, tag=tags[k]))
        for t, p in recvs:
            k = ("r", p)
            tags[k] = tags.get(k, -1) + 1
            ops.append(dist.P2POp(dist.irecv, t, p, group=group, tag=tags[k]))
        works = dist.batch_isend_irecv(ops) if ops else []
        w = _Works(works)
        if not async_op or debug:
            w.wait()
        return w if async_op else None
    _sendrecv_packed(sends, recvs, group, me)
    return _DoneWork() if async_op else None


class _NativeWork:
    def __init__(self, native):
        self._native = native

    def wait(self, timeout=None):
        self._native.wait()
        return True

    def is_completed(self):
        return self._native.is_completed()


def _sendrecv_packed(sends, recvs, group, me):
    world = get_world_size(group)
    dtypes = {t.dtype for t, _ in sends + recvs}
    if len(dtypes) > 1:
        raise ValueError("sendrecv (packed fallback): all chunks must share one dtype")
    ref = (sends + recvs)[0][0] if sends or recvs else None
    dev = ref.device if ref is not None else torch.device("cpu")
    dt = ref.dtype if ref is not None else torch.float32
    per_dst = [[] for _ in range(world)]
    for t, p in sends:
        per_dst[p].append(t.reshape(-1))
    sizes = [sum(t.numel() for t in lst) for lst in per_dst]
    mx = torch.tensor([max(sizes) if sizes else 0], dtype=torch.int64, device=dev)
    all_reduce(mx, ReduceOp.MAX, group=group)
    n = int(mx.item())
    if n == 0:
        return
    buf = torch.zeros((world, n), dtype=dt, device=dev)
    for p, lst in enumerate(per_dst):
        if lst:
            buf[p, :sizes[p]] = torch.cat(lst)
    out = torch.empty((world, world, n), dtype=dt, device=dev)
    all_gather_into_tensor(out.view(-1), buf.view(-1), group=group)
    offs = [0] * world
    for t, p in recvs:
        k = t.numel()
        t.copy_(out[p, me, offs[p]:offs[p] + k].view_as(t))
        offs[p] += k


def barrier(group=None) -> None:
    """Barrier.  On RCCL this is a 1-element all-reduce plus a stream sync
    (ProcessGroupNCCL semantics)."""
    if not is_initialized():
        return
    if dist.get_backend(group) == "nccl":
        dist.barrier(group=group, device_ids=[torch.cuda.current_device()])
    else:
        dist.barrier(group=group)
