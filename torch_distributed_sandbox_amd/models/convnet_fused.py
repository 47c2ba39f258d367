"""Fused gfx950 execution plan for the ConvNet (filled in by the fused-kernel milestone)."""
from __future__ import annotations


def supported(model, x) -> bool:
    return False


def forward(model, x):  # pragma: no cover - not yet available
    raise NotImplementedError
