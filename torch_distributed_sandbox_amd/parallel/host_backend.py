"""``"host"`` backend: CPU collectives over this package's native C++ TCP ring
(``csrc/comm/host_backend.cpp``), registered with ``torch.distributed`` as the
custom backend ``"tds_host"``.

It fills the role gloo plays in the reference (the CPU fallback of
test_init.py:84-88 and the CPU rehearsal path of SURVEY.md §4): a second,
independent transport that multi-process tests can run without a GPU, with
bounded waits (every socket wait honours the process-group timeout, so a dead
or hung peer surfaces as an error instead of a hang).

GPU tensors are staged through host memory (as gloo does); for device
collectives use the ``rccl`` backend.
"""
from __future__ import annotations

import datetime
import os
import socket

import torch
import torch.distributed as dist

BACKEND_NAME = "tds_host"


def _op_code(op) -> int:
    # opts.reduceOp is a ReduceOp instance; it compares equal (but does not hash
    # equal) to the RedOpType constants
    R = dist.ReduceOp
    for code, kind in enumerate((R.SUM, R.AVG, R.MAX, R.MIN, R.PRODUCT)):
        if op == kind:
            return code
    raise ValueError(f"host backend: unsupported reduce op {op}")


def _done(result=None):
    from torch._C._distributed_c10d import _create_work_from_future
    from torch.futures import Future

    fut = Future()
    fut.set_result(result)
    return _create_work_from_future(fut)


def _local_addr() -> str:
    """Address peers use to reach this rank: ``TDS_HOST_ADDR`` if set, loopback
    for single-node rendezvous, else the interface that routes to MASTER_ADDR."""
    a = os.environ.get("TDS_HOST_ADDR")
    if a:
        return a
    master = os.environ.get("MASTER_ADDR", "127.0.0.1")
    if master in ("127.0.0.1", "localhost", "::1"):
        return "127.0.0.1"
    try:
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        s.connect((master, 1))
        ip = s.getsockname()[0]
        s.close()
        return ip
    except OSError:
        return "127.0.0.1"


class _Staged:
    """Contiguous CPU view of a tensor for the native ring (copy in/out when needed)."""

    def __init__(self, t: torch.Tensor):
        self.t = t
        self.direct = t.device.type == "cpu" and t.is_contiguous()
        self.buf = t if self.direct else t.detach().to("cpu", copy=True).contiguous()

    def finish(self):
        if not self.direct:
            self.t.copy_(self.buf)


class HostProcessGroup(dist.ProcessGroup):
    """torch ProcessGroup whose collectives run on the native ring communicator.

    Collectives execute synchronously on the calling thread and return completed
    works, so ``async_op=True`` is accepted (and already done on return)."""

    def __init__(self, store, rank: int, world_size: int, timeout: datetime.timedelta):
        super().__init__(rank, world_size)
        from .._ext import classes

        self._rank, self._world = rank, world_size
        ms = int(timeout.total_seconds() * 1000) if timeout is not None else 600_000
        self._comm = classes().HostComm(rank, world_size, ms)
        if world_size > 1:
            store.set(f"addr/{rank}", f"{_local_addr()}:{self._comm.port()}")
            peers = [store.get(f"addr/{r}").decode() for r in range(world_size)]
            self._comm.connect(peers)

    # ---- identity -------------------------------------------------------
    def size(self):
        return self._world

    def rank(self):
        return self._rank

    def getBackendName(self):
        return BACKEND_NAME

    def __repr__(self):
        return f"HostProcessGroup(rank={self._rank}, world_size={self._world})"

    # ---- collectives ----------------------------------------------------
    def allreduce(self, tensor_list, opts=None):
        op = _op_code(opts.reduceOp if opts is not None else dist.ReduceOp.SUM)
        for t in tensor_list:
            st = _Staged(t)
            self._comm.allreduce_(st.buf, op)
            st.finish()
        return _done(tensor_list)

    def allreduce_coalesced(self, tensor_list, opts=None):
        op = _op_code(opts.reduceOp if opts is not None else dist.ReduceOp.SUM)
        by_dtype = {}
        for t in tensor_list:
            by_dtype.setdefault(t.dtype, []).append(t)
        for ts in by_dtype.values():
            flat = torch.cat([t.detach().reshape(-1).cpu() for t in ts])
            self._comm.allreduce_(flat, op)
            o = 0
            for t in ts:
                t.copy_(flat[o:o + t.numel()].view_as(t))
                o += t.numel()
        return _done(tensor_list)

    def broadcast(self, tensor_list, opts=None):
        root = opts.rootRank if opts is not None else 0
        for t in tensor_list:
            st = _Staged(t)
            self._comm.broadcast_(st.buf, root)
            st.finish()
        return _done(tensor_list)

    def _allgather_base(self, output, input, opts=None):
        so = _Staged(output)
        self._comm.allgather(so.buf.view(-1), input.detach().cpu().contiguous().view(-1))
        so.finish()
        return _done(output)

    def allgather(self, output_tensors, input_tensor, opts=None):
        for outs, inp in zip(output_tensors, input_tensor):
            flat = torch.empty(self._world * inp.numel(), dtype=inp.dtype)
            self._comm.allgather(flat, inp.detach().cpu().contiguous().view(-1))
            for r, o in enumerate(outs):
                o.copy_(flat[r * inp.numel():(r + 1) * inp.numel()].view_as(o))
        return _done(output_tensors)

    def allgather_into_tensor_coalesced(self, outputs, inputs, opts=None):
        for o, i in zip(outputs, inputs):
            self._allgather_base(o, i)
        return _done(outputs)

    def _reduce_scatter_base(self, output, input, opts=None):
        op = _op_code(opts.reduceOp if opts is not None else dist.ReduceOp.SUM)
        so = _Staged(output)
        self._comm.reduce_scatter_(so.buf.view(-1), input.detach().cpu().contiguous().view(-1), op)
        so.finish()
        return _done(output)

    def reduce_scatter(self, output_tensors, input_tensors, opts=None):
        for out, ins in zip(output_tensors, input_tensors):
            flat = torch.cat([t.detach().reshape(-1).cpu() for t in ins])
            self._reduce_scatter_base(out, flat, opts)
        return _done(output_tensors)

    def reduce_scatter_tensor_coalesced(self, outputs, inputs, opts=None):
        for o, i in zip(outputs, inputs):
            self._reduce_scatter_base(o, i, opts)
        return _done(outputs)

    def reduce(self, tensor_list, opts=None):
        # all-reduce then non-roots restore their input: same traffic class as a ring reduce
        op = _op_code(opts.reduceOp if opts is not None else dist.ReduceOp.SUM)
        root = opts.rootRank if opts is not None else 0
        for t in tensor_list:
            st = _Staged(t)
            buf = st.buf if self._rank == root else st.buf.clone()
            self._comm.allreduce_(buf, op)
            if self._rank == root:
                st.finish()
        return _done(tensor_list)

    def gather(self, output_tensors, input_tensors, opts=None):
        root = opts.rootRank if opts is not None else 0
        inp = input_tensors[0]
        flat = torch.empty(self._world * inp.numel(), dtype=inp.dtype)
        self._comm.allgather(flat, inp.detach().cpu().contiguous().view(-1))
        if self._rank == root:
            for r, o in enumerate(output_tensors[0]):
                o.copy_(flat[r * inp.numel():(r + 1) * inp.numel()].view_as(o))
        return _done(output_tensors)

    def scatter(self, output_tensors, input_tensors, opts=None):
        root = opts.rootRank if opts is not None else 0
        out = output_tensors[0]
        flat = torch.empty(self._world * out.numel(), dtype=out.dtype)
        if self._rank == root:
            flat.copy_(torch.cat([t.detach().reshape(-1).cpu() for t in input_tensors[0]]))
        self._comm.broadcast_(flat, root)
        out.copy_(flat[self._rank * out.numel():(self._rank + 1) * out.numel()].view_as(out))
        return _done(output_tensors)

    def alltoall_base(self, output, input, output_split_sizes, input_split_sizes, opts=None):
        if output_split_sizes or input_split_sizes:
            raise NotImplementedError("host backend: uneven all_to_all_single is not supported")
        n = input.numel() // self._world
        flat = torch.empty(self._world * input.numel(), dtype=input.dtype)
        self._comm.allgather(flat, input.detach().cpu().contiguous().view(-1))
        parts = flat.view(self._world, self._world, n)[:, self._rank]  # [src][n]
        output.copy_(parts.reshape(output.shape))
        return _done(output)

    def barrier(self, opts=None):
        self._comm.barrier()
        return _done(None)

    def shutdown(self):
        self._comm.close()


def _create(store, rank, world_size, timeout):
    return HostProcessGroup(store, rank, world_size, timeout)


_registered = False


def register() -> str:
    global _registered
    if not _registered:
        if BACKEND_NAME not in dist.Backend.backend_list:
            dist.Backend.register_backend(BACKEND_NAME, _create, devices=["cpu", "cuda"])
        _registered = True
    return BACKEND_NAME
