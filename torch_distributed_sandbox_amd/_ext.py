"""Loader for the in-tree native extension ``_C.so`` (gfx950 kernels + C++ runtime).

Policy (no silent fallbacks on the GPU):

* GPU tensors always go through ``torch.ops.tdsa``; if the extension is
  missing or fails to load, :func:`ops` raises with the load error.
* CPU tensors (unit tests, ``gloo`` rehearsals) use the reference PyTorch
  implementation of each op; that is dispatch by device, not a fallback.

Set ``TDS_AUTOBUILD=1`` to build the extension on first use when it is absent.
"""
from __future__ import annotations

import os
import threading

import torch

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# TDS_SO_VARIANT=<name> loads the side build _C_<name>.so (_build.py --variant; A/B experiments)
_VARIANT = os.environ.get("TDS_SO_VARIANT", "")
SO_PATH = os.path.join(_PKG_DIR, f"_C_{_VARIANT}.so" if _VARIANT else "_C.so")

_lock = threading.Lock()
_loaded = False
_load_error: Exception | None = None


def load(autobuild: bool | None = None) -> bool:
    """Load ``_C.so`` once; returns True on success."""
    global _loaded, _load_error
    if _loaded:
        return True
    with _lock:
        if _loaded:
            return True
        if autobuild is None:
            autobuild = os.environ.get("TDS_AUTOBUILD", "0") == "1"
        if not os.path.exists(SO_PATH) and autobuild:
            from . import _build

            _build.build()
        try:
            torch.ops.load_library(SO_PATH)
            _loaded = True
            _load_error = None
        except Exception as e:  # pragma: no cover - depends on build state
            _load_error = e
    return _loaded


def available() -> bool:
    return load()


def ops():
    """``torch.ops.tdsa`` — raises loudly if the native extension is unusable."""
    if not load():
        raise RuntimeError(
            f"torch_distributed_sandbox_amd native extension not loaded from {SO_PATH}: {_load_error!r}. "
            "Build it with `python -m torch_distributed_sandbox_amd._build` (hipcc --offload-arch=gfx950)."
        )
    return torch.ops.tdsa


def classes():
    """``torch.classes.tdsa`` (C++ store / host backend / RCCL communicator / reducer)."""
    ops()
    return torch.classes.tdsa


def on_gpu(*tensors) -> bool:
    return any(isinstance(t, torch.Tensor) and t.is_cuda for t in tensors)
