"""Process launching and rendezvous helpers.

* :func:`find_free_port` — the reference's helper (copied 3x there, e.g.
  allreduce_toy.py:10-18), fixed: ``SO_REUSEADDR`` is set *before* ``bind``
  and the socket is bound to the loopback address.
* :func:`spawn` — ``torch.multiprocessing.spawn`` semantics (child ``i`` runs
  ``fn(i, *args)``, spawn start method, fail-fast: the first failing child
  terminates the others and its traceback is re-raised in the parent), with an
  optional overall timeout so a hung rank cannot hang the job.
* :func:`setup_rendezvous_env` — ``MASTER_ADDR``/``MASTER_PORT`` from flags or
  env, so multi-node works (``--nodes/--nr`` + ``--master-addr``).
* :func:`env_rank_info` — RANK / LOCAL_RANK / WORLD_SIZE as set by torchrun.
"""
from __future__ import annotations

import multiprocessing as _mp
import os
import signal
import socket
import sys
import time
import traceback
from contextlib import closing
from typing import Callable, Optional


def find_free_port(host: str = "127.0.0.1") -> str:
    with closing(socket.socket(socket.AF_INET, socket.SOCK_STREAM)) as s:
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        s.bind((host, 0))
        return str(s.getsockname()[1])


def setup_rendezvous_env(master_addr: Optional[str] = None, master_port: Optional[str] = None) -> tuple:
    addr = master_addr or os.environ.get("MASTER_ADDR") or "127.0.0.1"
    port = master_port or os.environ.get("MASTER_PORT") or find_free_port()
    os.environ["MASTER_ADDR"] = addr
    os.environ["MASTER_PORT"] = str(port)
    return addr, str(port)


def env_rank_info() -> dict:
    return {
        "rank": int(os.environ.get("RANK", "0")),
        "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
        "world_size": int(os.environ.get("WORLD_SIZE", "1")),
        "local_world_size": int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1"))),
    }


class ProcessRaisedException(RuntimeError):
    def __init__(self, msg: str, error_index: int, pid: int):
        super().__init__(msg)
        self.error_index, self.pid = error_index, pid


class ProcessExitedException(RuntimeError):
    def __init__(self, msg: str, error_index: int, pid: int, exit_code: int):
        super().__init__(msg)
        self.error_index, self.pid, self.exit_code = error_index, pid, exit_code


def _child_entry(fn, i, args, err_q):
    try:
        fn(i, *args)
    except KeyboardInterrupt:
        pass
    except BaseException:
        err_q.put((i, traceback.format_exc()))
        sys.exit(1)


def spawn(fn: Callable, args=(), nprocs: int = 1, join: bool = True, timeout: Optional[float] = None,
          poll_interval: float = 0.05):
    """Start ``nprocs`` processes running ``fn(i, *args)``; fail fast."""
    ctx = _mp.get_context("spawn")
    err_q = ctx.SimpleQueue()
    procs = []
    for i in range(nprocs):
        p = ctx.Process(target=_child_entry, args=(fn, i, tuple(args), err_q), daemon=False)
        p.start()
        procs.append(p)
    if not join:
        return procs
    t0 = time.time()
    try:
        while True:
            alive = [p for p in procs if p.is_alive()]
            failed = [(i, p) for i, p in enumerate(procs) if not p.is_alive() and p.exitcode not in (0, None)]
            if failed:
                i, p = failed[0]
                _terminate(procs)
                msg = f"process {i} (pid {p.pid}) exited with code {p.exitcode}"
                tb = None
                while not err_q.empty():
                    ei, etb = err_q.get()
                    if tb is None or ei == i:
                        tb, i = etb, ei
                if tb is not None:
                    raise ProcessRaisedException(f"\n\n-- Process {i} terminated with the following error:\n{tb}", i,
                                                 procs[i].pid)
                code = p.exitcode
                if code is not None and code < 0:
                    msg += f" (signal {signal.Signals(-code).name})"
                raise ProcessExitedException(msg, i, p.pid, code)
            if not alive:
                return None
            if timeout is not None and time.time() - t0 > timeout:
                _terminate(procs)
                raise TimeoutError(f"spawn: ranks still running after {timeout:.0f}s; terminated")
            time.sleep(poll_interval)
    finally:
        for p in procs:
            p.join(timeout=0.1)


def _terminate(procs, grace: float = 5.0):
    for p in procs:
        if p.is_alive():
            p.terminate()
    deadline = time.time() + grace
    for p in procs:
        p.join(timeout=max(0.0, deadline - time.time()))
        if p.is_alive():
            p.kill()
            p.join(timeout=1.0)
