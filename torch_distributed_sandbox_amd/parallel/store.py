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

``rendezvous()`` is how every entry point gets its store (``init_process_group``'s
default, bench.py, the trainers, the toy): the native store carries the rendezvous --
process-group init, ``new_group``, the RCCL unique-id exchange, bench.py's fallback votes.
c10d's TCPStore at ``MASTER_ADDR:MASTER_PORT`` (rank 0's, or torchrun's agent store) is
only the locator -- rank 0 publishes the native server's ephemeral port there -- and the
fallback: if any rank cannot create or reach the native store, all ranks agree (through
c10d) to use c10d's store instead, and say so (``kind``).
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


def _c10d_store(host: str, port: int, rank: int, world_size: int, timeout: datetime.timedelta):
    """c10d's TCPStore at host:port: rank 0 serves it, unless torchrun's agent already does."""
    import os

    agent = os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True"
    return dist.TCPStore(host, port, world_size, is_master=(rank == 0 and not agent), timeout=timeout,
                         wait_for_workers=False)


def rendezvous(rank: int, world_size: int, host: Optional[str] = None, port: Optional[int] = None,
               timeout: datetime.timedelta = datetime.timedelta(minutes=5), prefer: Optional[str] = None):
    """The rendezvous store of this job and its kind: ``(store, "native")``, or c10d's store
    with ``"c10d"`` (asked for: ``prefer="c10d"`` / ``TDS_STORE=c10d``) or
    ``"c10d (fallback: <reason>)"`` (the native store failed on some rank; every rank takes the
    same decision).  ``host``/``port`` default to ``MASTER_ADDR``/``MASTER_PORT``."""
    import os

    host = host or os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(port if port is not None else os.environ.get("MASTER_PORT", "29500"))
    prefer = prefer or os.environ.get("TDS_STORE", "native") or "native"
    if prefer not in ("native", "c10d"):
        raise ValueError(f"TDS_STORE / prefer must be native or c10d, got {prefer!r}")
    loc = _c10d_store(host, port, rank, world_size, timeout)
    if prefer == "c10d":
        return loc, "c10d"
    gen = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
    key = f"tds/native_store/{gen}"
    native, err = None, None
    if rank == 0:
        try:
            native = NativeStore(host, 0, world_size, True, timeout)  # ephemeral port, published below
            loc.set(key, f"ok {native.port}")
        except Exception as e:  # noqa: BLE001 -- reported to every rank, c10d is used
            err = f"rank 0: {type(e).__name__}: {e}"
            loc.set(key, "fail " + err[:300])
    else:
        v = loc.get(key).decode()
        if v.startswith("ok "):
            try:
                native = NativeStore(host, int(v[3:]), world_size, False, timeout)
            except Exception as e:  # noqa: BLE001
                err = f"rank {rank}: {type(e).__name__}: {e}"
        else:
            err = v[5:]
    # every rank reports; all take the same decision
    loc.set(f"{key}/{rank}", "ok" if err is None else "fail " + err[:300])
    bad = [v for v in (loc.get(f"{key}/{r}").decode() for r in range(world_size)) if v != "ok"]
    if bad:
        return loc, f"c10d (fallback: {bad[0][5:]})"
    native._locator = loc  # rank 0 serves both; keep the locator alive with the store
    return native, "native"


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
