"""``"rccl-native"`` backend: device collectives on this package's own C++ RCCL
communicator (``csrc/comm/rccl_comm.h``), registered with ``torch.distributed``
as the custom backend ``"tds_rccl"``.

What it adds over the stock ``ProcessGroupNCCL`` path:

* eager communicator creation bound to this rank's GPU (unique id exchanged
  through the rendezvous store, so no lazy first-collective init),
* one high-priority HIP comm stream; works are HIP events — ``wait()`` is a
  device-side stream wait, the host never blocks,
* a watchdog thread with a timeout and RCCL async-error polling that aborts the
  communicator and (by default) terminates the rank so the launcher fails fast,
* grouped (coalesced) broadcast used by DDP for the per-forward BN-buffer sync
  and the construction-time state broadcast,
* direct hand-off of the communicator to the C++ gradient reducer.

The collectives themselves are RCCL's (ring / tree over the xGMI links), from
the same ``librccl`` torch loads.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist

from .host_backend import _op_code

BACKEND_NAME = "tds_rccl"


class _Work(dist.Work):
    """torch Work wrapping a native CommWork (event on the comm stream)."""

    def __init__(self, native, result=None):
        super().__init__()
        self._native, self._result = native, result

    def wait(self, timeout=None):
        self._native.wait()
        return True

    def is_completed(self):
        return self._native.is_completed()

    def synchronize(self):
        self._native.synchronize()

    def result(self):
        return self._result


def exchange_unique_id(store, rank: int, key: str = "rccl_uid") -> torch.Tensor:
    """The communicator's ncclUniqueId (128 bytes): made by rank 0 (ncclGetUniqueId, no GPU
    needed) and published through the rendezvous store -- this package's C++ store by default
    (parallel/store.py) -- every other rank blocks in ``get`` until it is there."""
    from .._ext import classes

    if rank == 0:
        uid = classes().RcclComm.unique_id()
        store.set(key, bytes(uid.numpy().tobytes()))
        return uid
    raw = store.get(key)
    return torch.frombuffer(bytearray(raw), dtype=torch.uint8)


class RcclProcessGroup(dist.ProcessGroup):
    def __init__(self, store, rank: int, world_size: int, timeout: datetime.timedelta):
        super().__init__(rank, world_size)
        from .._ext import classes

        self._rank, self._world = rank, world_size
        dev = torch.cuda.current_device()
        uid = exchange_unique_id(store, rank)
        ms = int(timeout.total_seconds() * 1000) if timeout is not None else 600_000
        self._comm = classes().RcclComm(rank, world_size, dev, uid, ms)
        self.device_index = dev

    def size(self):
        return self._world

    def rank(self):
        return self._rank

    def getBackendName(self):
        return BACKEND_NAME

    def __repr__(self):
        return f"RcclProcessGroup(rank={self._rank}, world_size={self._world}, device=cuda:{self.device_index})"

    @property
    def native(self):
        return self._comm

    # ---- collectives ----------------------------------------------------
    def allreduce(self, tensor_list, opts=None):
        op = _op_code(opts.reduceOp if opts is not None else dist.ReduceOp.SUM)
        w = None
        for t in tensor_list:
            w = self._comm.allreduce(t, op)
        return _Work(w, tensor_list)

    def allreduce_coalesced(self, tensor_list, opts=None):
        return self.allreduce(tensor_list, opts)

    def broadcast(self, tensor_list, opts=None):
        root = opts.rootRank if opts is not None else 0
        if len(tensor_list) == 1:
            return _Work(self._comm.broadcast(tensor_list[0], root), tensor_list)
        return _Work(self._comm.broadcast_coalesced(list(tensor_list), root), tensor_list)

    def reduce(self, tensor_list, opts=None):
        op = _op_code(opts.reduceOp if opts is not None else dist.ReduceOp.SUM)
        root = opts.rootRank if opts is not None else 0
        w = None
        for t in tensor_list:
            w = self._comm.reduce(t, root, op)
        return _Work(w, tensor_list)

    def _allgather_base(self, output, input, opts=None):
        return _Work(self._comm.allgather(output.view(-1), input.contiguous().view(-1)), output)

    def allgather(self, output_tensors, input_tensor, opts=None):
        w = None
        for outs, inp in zip(output_tensors, input_tensor):
            flat = torch.empty(self._world * inp.numel(), dtype=inp.dtype, device=inp.device)
            self._comm.allgather(flat, inp.contiguous().view(-1)).wait()
            for r, o in enumerate(outs):
                o.copy_(flat[r * inp.numel():(r + 1) * inp.numel()].view_as(o))
        return _Work(_DoneNative(), output_tensors) if w is None else _Work(w, output_tensors)

    def allgather_into_tensor_coalesced(self, outputs, inputs, opts=None):
        w = None
        for o, i in zip(outputs, inputs):
            w = self._comm.allgather(o.view(-1), i.contiguous().view(-1))
        return _Work(w, outputs)

    def _reduce_scatter_base(self, output, input, opts=None):
        op = _op_code(opts.reduceOp if opts is not None else dist.ReduceOp.SUM)
        return _Work(self._comm.reduce_scatter(output.view(-1), input.contiguous().view(-1), op), output)

    def reduce_scatter(self, output_tensors, input_tensors, opts=None):
        w = None
        for out, ins in zip(output_tensors, input_tensors):
            flat = torch.cat([t.reshape(-1) for t in ins])
            w = self._reduce_scatter_base(out, flat, opts)
        return w

    def reduce_scatter_tensor_coalesced(self, outputs, inputs, opts=None):
        w = None
        for o, i in zip(outputs, inputs):
            w = self._reduce_scatter_base(o, i, opts)
        return w

    def alltoall_base(self, output, input, output_split_sizes, input_split_sizes, opts=None):
        if output_split_sizes or input_split_sizes:
            raise NotImplementedError("rccl-native: uneven all_to_all_single is not supported")
        return _Work(self._comm.alltoall(output.view(-1), input.contiguous().view(-1)), output)

    def send(self, tensors, dst, tag=0):
        w = None
        for t in tensors:
            w = self._comm.send(t, dst)
        return _Work(w, tensors)

    def recv(self, tensors, src, tag=0):
        w = None
        for t in tensors:
            w = self._comm.recv(t, src)
        return _Work(w, tensors)

    def barrier(self, opts=None):
        self._comm.barrier()
        return _Work(_DoneNative(), None)

    def shutdown(self):
        self._comm.shutdown()

    def abort(self):
        self._comm.abort("abort requested")


class _DoneNative:
    def wait(self):
        pass

    def is_completed(self):
        return True

    def synchronize(self):
        pass


def _create(store, rank, world_size, timeout):
    return RcclProcessGroup(store, rank, world_size, timeout)


_registered = False


def register() -> str:
    global _registered
    if not _registered:
        if BACKEND_NAME not in dist.Backend.backend_list:
            dist.Backend.register_backend(BACKEND_NAME, _create, devices=["cuda"])
        _registered = True
    return BACKEND_NAME


def native_comm_of(group):
    """(C++ communicator, "rccl"|"host") behind a process group; (None, None) for torch's own PGs."""
    from .host_backend import HostProcessGroup

    if group is None:
        group = dist.group.WORLD
    if isinstance(group, RcclProcessGroup):
        return group._comm, "rccl"
    if isinstance(group, HostProcessGroup):
        return group._comm, "host"
    return None, None
