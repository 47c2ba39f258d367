"""Host-side views of the fused plan's blocked pooled layouts (csrc/kernels/pooled_layout.h), for
tests and tools: plane sizes and conversions to / from the planar [B, 32, Q, Q] form.

* ya, pooled-blocked: blocks of 4 pooled rows x 8 pooled columns (128 B), block row R = py // 4.
* g2m, row-shifted pooled-blocked: the same blocks with block row R = (py + 3) // 4 (it holds
  pooled rows 4R - 3 .. 4R), so a conv2 backward tile's staged windows are one block per channel.
"""
from __future__ import annotations

import torch


def pb_plane(Q: int) -> int:
    """ya floats per (image, channel) plane."""
    return ((Q + 3) // 4) * ((Q + 7) // 8) * 32


def g2m_plane(Q: int) -> int:
    """g2m floats per (image, channel) plane."""
    return ((Q + 2) // 4 + 1) * ((Q + 7) // 8) * 32


def _g2m_index(Q: int, device) -> torch.Tensor:
    """[Q, Q] int64: each pooled position's offset inside a g2m plane."""
    py = torch.arange(Q, device=device).view(Q, 1)
    px = torch.arange(Q, device=device).view(1, Q)
    q8 = (Q + 7) // 8
    return ((((py + 3) // 4) * q8 + px // 8) * 32 + ((py + 3) % 4) * 8 + px % 8).to(torch.int64)


def g2m_to_planar(g2m: torch.Tensor, Q: int) -> torch.Tensor:
    """[B, 32, g2m_plane(Q)] -> [B, 32, Q, Q] (the positions inside the image)."""
    B = g2m.shape[0]
    idx = _g2m_index(Q, g2m.device).view(-1)
    return g2m.reshape(B, 32, -1).index_select(2, idx).view(B, 32, Q, Q)


def planar_to_g2m(x: torch.Tensor) -> torch.Tensor:
    """[B, 32, Q, Q] -> [B, 32, g2m_plane(Q)] (slots outside the image: 0)."""
    B, C, Q, _ = x.shape
    out = torch.zeros(B, C, g2m_plane(Q), device=x.device, dtype=x.dtype)
    out.index_copy_(2, _g2m_index(Q, x.device).view(-1), x.reshape(B, C, Q * Q))
    return out
