"""Environment-driven fault injection (SURVEY.md §5 "Failure detection").

The reference relies only on ``mp.spawn`` fail-fast and the NCCL watchdog.
To *test* those paths without a cluster, trainers call :func:`maybe_inject`
once per step:

    TDS_FAULT_RANK=1 TDS_FAULT_STEP=3 TDS_FAULT_MODE=raise|exit|hang|segv

``raise`` throws ``InjectedFault``; ``exit`` calls ``os._exit(17)``; ``hang``
sleeps (for the watchdog / launcher timeout to catch); ``segv`` sends SIGSEGV
to itself.  Nothing happens unless both rank and step match.
"""
from __future__ import annotations

import os
import signal
import time


class InjectedFault(RuntimeError):
    pass


def fault_config():
    r = os.environ.get("TDS_FAULT_RANK")
    s = os.environ.get("TDS_FAULT_STEP")
    if r is None or s is None:
        return None
    return int(r), int(s), os.environ.get("TDS_FAULT_MODE", "raise")


def maybe_inject(rank: int, step: int) -> None:
    cfg = fault_config()
    if cfg is None:
        return
    fr, fs, mode = cfg
    if rank != fr or step != fs:
        return
    if mode == "raise":
        raise InjectedFault(f"injected fault on rank {rank} at step {step}")
    if mode == "exit":
        os._exit(17)
    if mode == "hang":
        time.sleep(float(os.environ.get("TDS_FAULT_HANG_S", "3600")))
        return
    if mode == "segv":
        os.kill(os.getpid(), signal.SIGSEGV)
        return
    raise ValueError(f"unknown TDS_FAULT_MODE {mode!r}")


def maybe_inject_bench(rank: int, phase: str) -> None:
    """bench.py's failure rehearsal: ``TDS_BENCH_FAULT=<rank>:<phase>:<mode>[:<attempt-limit>]``
    with phase ``init`` (before the process group is joined: a rank that never joins) or
    ``step`` (every warmup step) and mode ``raise`` | ``exit`` | ``hang``.  With an attempt limit
    n the fault fires only in the first n calls of this process (so a fallback attempt can
    succeed)."""
    spec = os.environ.get("TDS_BENCH_FAULT")
    if not spec:
        return
    parts = spec.split(":")
    fr, fphase, mode = int(parts[0]), parts[1], parts[2]
    if rank != fr or phase != fphase:
        return
    if len(parts) > 3:
        key = f"_TDS_BENCH_FAULT_N_{phase}"
        n = int(os.environ.get(key, "0"))
        if n >= int(parts[3]):
            return
        os.environ[key] = str(n + 1)
    if mode == "raise":
        raise InjectedFault(f"injected bench fault on rank {rank} in phase {phase}")
    if mode == "exit":
        os._exit(17)
    if mode == "hang":
        time.sleep(float(os.environ.get("TDS_FAULT_HANG_S", "3600")))
        return
    raise ValueError(f"unknown TDS_BENCH_FAULT mode {mode!r}")
