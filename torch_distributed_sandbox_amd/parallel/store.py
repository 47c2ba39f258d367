"""Rendezvous key-value store backed by the native C++ TCP store
(``csrc/comm/tcp_store.cpp``, SURVEY.md §2.3 N1 — the role of c10d's TCPStore
behind ``MASTER_ADDR``/``MASTER_PORT`` in the reference's
mnist_distributed.py:124-125).

``NativeStore`` subclasses ``torch.distributed.Store``, so it can be handed to
``torch.distributed.init_process_group(store=...)`` and serves every backend's
rendezvous (RCCL unique-id exchange, gloo / host-ring address exchange).
Rank 0 runs the server thread in-process; every rank (including 0) is a client.
The server supports blocking GET/WAIT, ADD, CHECK, compare-and-set, DELETE and
NUM_KEYS; every wait is bounded by the store timeout.
"""
from __future__ import annotations

import datetime
from typing import List, Optional

import torch
import torch.distributed as dist


def _to_u8(v) -> torch.Tensor:
    if isinstance(v, str):
        v = v.encode()
    return torch.frombuffer(bytearray(v), dtype=torch.uint8) if len(v) else torch.empty(0, dtype=torch.uint8)


def _to_bytes(t: torch.Tensor) -> bytes:
    return t.numpy().tobytes()


class NativeStore(dist.Store):
    def __init__(self, host: str, port: int, world_size: int, is_server: bool,
                 timeout: datetime.timedelta = datetime.timedelta(minutes=5)):
        super().__init__()
        from .._ext import classes

        self._ms = int(timeout.total_seconds() * 1000)
        self._s = classes().TCPStore(host, int(port), int(world_size), bool(is_server), self._ms)
        self.host, self.world = host, world_size

    @property
    def port(self) -> int:
        return int(self._s.port())

    # --- dist.Store interface (called by c10d through the PythonStore trampoline) ---
    def set(self, key, value):
        self._s.set(key, _to_u8(value))

    def get(self, key):
        return _to_bytes(self._s.get(key))

    def add(self, key, value):
        return int(self._s.add(key, int(value)))

    def compare_set(self, key, expected, desired):
        return _to_bytes(self._s.compare_set(key, _to_u8(expected), _to_u8(desired)))

    def delete_key(self, key):
        return bool(self._s.delete_key(key))

    def num_keys(self):
        return int(self._s.num_keys())

    def check(self, keys: List[str]):
        return all(self._s.check(k) for k in keys)

    def wait(self, keys: List[str], timeout: Optional[datetime.timedelta] = None):
        ms = int(timeout.total_seconds() * 1000) if timeout is not None else self._ms
        for k in keys:
            self._s.wait(k, ms)

    def set_timeout(self, timeout: datetime.timedelta):
        self._ms = int(timeout.total_seconds() * 1000)
        self._s.set_timeout(self._ms)


def create_store(rank: int, world_size: int, host: Optional[str] = None, port: Optional[int] = None,
                 timeout: datetime.timedelta = datetime.timedelta(minutes=5)) -> NativeStore:
    """Store at ``host:port``; rank 0 serves.  Default port: ``TDS_STORE_PORT``, else
    ``MASTER_PORT`` — or ``MASTER_PORT + 1`` under torchrun, whose agent already
    serves c10d's store on ``MASTER_PORT``."""
    import os

    host = host or os.environ.get("MASTER_ADDR", "127.0.0.1")
    if port is None:
        if "TDS_STORE_PORT" in os.environ:
            port = int(os.environ["TDS_STORE_PORT"])
        else:
            port = int(os.environ.get("MASTER_PORT", "29500"))
            if os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True":
                port += 1
    return NativeStore(host, port, world_size, rank == 0, timeout)
