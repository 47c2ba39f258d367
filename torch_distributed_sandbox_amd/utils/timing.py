"""Timing / profiling helpers (SURVEY.md §5 "Tracing / profiling", "Metrics / logging").

* :class:`StepTimer` — HIP-event timing of named phases per step (fwd / bwd /
  step), no host sync inside the step; summarised at the end.
* :func:`range_push` / :func:`range_pop` / :func:`nvtx_range` — roctx ranges
  (``torch.cuda.nvtx`` maps to roctx on ROCm) so ``rocprofv3 --marker-trace``
  or the kernel trace can be split by phase.
* :func:`rank_print` — print on selected ranks only, flushed.
"""
from __future__ import annotations

import contextlib
import os
import sys
import time
from collections import defaultdict

import torch


def rank_print(*args, rank: int = 0, only=(0,), **kw):
    if only is None or rank in only:
        print(*args, **kw)
        sys.stdout.flush()


def _roctx_enabled() -> bool:
    return os.environ.get("TDS_ROCTX", "0") == "1" and torch.cuda.is_available()


def range_push(name: str):
    if _roctx_enabled():
        torch.cuda.nvtx.range_push(name)


def range_pop():
    if _roctx_enabled():
        torch.cuda.nvtx.range_pop()


@contextlib.contextmanager
def nvtx_range(name: str):
    range_push(name)
    try:
        yield
    finally:
        range_pop()


class StepTimer:
    """Per-phase GPU timing with events (``trainer.py --phase-times``); call :meth:`summary`
    at the end.  Disabled, a phase only records host wall time (and still emits its roctx
    range when ``TDS_ROCTX=1``)."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self._events = defaultdict(list)
        self._wall = defaultdict(float)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            t0 = time.perf_counter()
            with nvtx_range(name):
                yield
            self._wall[name] += time.perf_counter() - t0
            return
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        with nvtx_range(name):
            yield
        e.record()
        self._events[name].append((s, e))

    def summary(self) -> dict:
        out = {}
        if self.enabled:
            torch.cuda.synchronize()
            for k, lst in self._events.items():
                ts = [s.elapsed_time(e) for s, e in lst]
                out[k] = {"n": len(ts), "mean_ms": sum(ts) / len(ts), "min_ms": min(ts)}
        for k, v in self._wall.items():
            out[k] = {"wall_s": v}
        return out
