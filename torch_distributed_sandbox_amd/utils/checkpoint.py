"""Checkpoint / resume (absent in the reference).

Rank 0 writes ``{model, optimizer, step, epoch, rng}`` with ``torch.save``;
every rank loads with ``weights_only=True`` (no pickle execution), and under
DDP the rank-0 values are broadcast so all replicas resume bit-identical.
Writes are atomic (tmp file + rename).
"""
from __future__ import annotations

import os

import torch


def _unwrap(model):
    return getattr(model, "module", model)


def save(path: str, model, optimizer=None, step: int = 0, epoch: int = 0, rank: int = 0, extra=None) -> None:
    if hasattr(model, "wait_pending_updates"):
        model.wait_pending_updates()  # DDP(overlap_optimizer=True) side-stream updates land first
    if rank != 0:
        return
    state = {
        "model": _unwrap(model).state_dict(),
        "optimizer": optimizer.state_dict() if optimizer is not None else None,
        "step": int(step),
        "epoch": int(epoch),
        "torch_rng": torch.get_rng_state(),
        "extra": extra or {},
    }
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, path)


def load(path: str, model, optimizer=None, map_location=None, broadcast: bool = True):
    state = torch.load(path, map_location=map_location or "cpu", weights_only=True)
    m = _unwrap(model)
    m.load_state_dict(state["model"])
    if optimizer is not None and state.get("optimizer") is not None:
        optimizer.load_state_dict(state["optimizer"])
    if broadcast:
        from ..parallel import distributed as tdist

        if tdist.is_initialized() and tdist.get_world_size() > 1:
            with torch.no_grad():
                for t in list(m.parameters()) + [b for b in m.buffers() if b is not None]:
                    tdist.broadcast(t.data, 0)
    if state.get("torch_rng") is not None:
        torch.set_rng_state(state["torch_rng"])
    return int(state.get("step", 0)), int(state.get("epoch", 0)), state.get("extra", {})
