"""Lossless zero-suppressed encoding of the fc input rows X for the fc-gradient exchanges.

The activation and sharded exchanges (parallel/factored.py) put X -- the fc layer's input,
``maxpool(ReLU(BN2(conv2)))`` flattened, 360 MB per rank per step at the 3000^2 bench shape --
on the xGMI links.  X is a ReLU output: a large share of it is exact zeros.  This module sends
the non-zero values only, plus a bitmask, and rebuilds X bit for bit on the receiver, so the
exchanged gradient (and every parameter after the step) is bitwise the one the dense exchange
gives.

Format of an encoded tensor x (any shape, fp32, n elements, read flat):

* pages of ``PAGE`` = 2048 consecutive elements, ``npages = ceil(n / PAGE)``;
* ``meta`` int32 ``[npages * (1 + PAGE // 32)]``: per page its value offset (the exclusive
  prefix sum of the non-zero counts: where its values start) followed by its 64 mask words;
  bit i of mask word j of page p <-> element ``p*PAGE + 32*j + i`` is non-zero -- "non-zero"
  means any bit set, so -0.0 and NaN payloads survive exactly;
* ``values`` fp32 ``[nnz]``: the non-zero elements in element order.

``meta`` has a fixed size (3.2 % of the dense bytes), ``values`` does not: a transfer sends a
capacity ``cap >= nnz`` (parallel/factored.py keeps it from the previous steps' counts and
falls back to the dense rows when a step overflows it).

GPU: the encode / decode kernels of csrc/kernels/zs_exchange.hip (``ops.zs_encode`` /
``ops.zs_decode``).  CPU: the torch reference below (tests, gloo rehearsals).
"""
from __future__ import annotations

from typing import Tuple

import torch

PAGE = 2048
WORDS = PAGE // 32  # mask words per page
META = 1 + WORDS     # int32 per page


def npages(n: int) -> int:
    return (n + PAGE - 1) // PAGE


def meta_numel(n: int) -> int:
    return npages(n) * META


def _bits(x: torch.Tensor) -> torch.Tensor:
    return x.reshape(-1).view(torch.int32)


def encode_ref(x: torch.Tensor, values_out: torch.Tensor = None) -> Tuple[torch.Tensor, torch.Tensor, int]:
    """(meta, values, nnz) of x (torch reference, any device).  With ``values_out`` the values
    are written into its first nnz elements (it must hold them)."""
    b = _bits(x)
    n = b.numel()
    P = npages(n)
    nz = b != 0
    pad = P * PAGE - n
    nzp = torch.cat([nz, nz.new_zeros(pad)]) if pad else nz
    counts = nzp.view(P, PAGE).sum(1, dtype=torch.int64)
    offs = torch.cumsum(counts, 0) - counts
    # mask words: bit i of word j <- element 32j + i
    w = nzp.view(P, WORDS, 32).to(torch.int64)
    shifts = torch.arange(32, device=x.device, dtype=torch.int64)
    words = (w << shifts).sum(-1)
    words = torch.where(words >= 2 ** 31, words - 2 ** 32, words).to(torch.int32)  # uint32 bits as int32
    meta = torch.cat([offs.to(torch.int32).view(P, 1), words], dim=1).reshape(-1)
    vals = x.reshape(-1)[nz]
    nnz = int(vals.numel())
    if values_out is not None:
        if values_out.numel() < nnz:
            raise ValueError(f"zs.encode: values_out holds {values_out.numel()} < nnz {nnz}")
        values_out[:nnz].copy_(vals)
        vals = values_out
    return meta, vals, nnz


def nnz_of(meta: torch.Tensor, n: int) -> torch.Tensor:
    """Number of non-zero elements of an encoded tensor of n elements, as a 0-d int64 tensor
    on meta's device (no host sync): the last page's offset + its popcount."""
    P = npages(n)
    last = meta.view(P, META)[P - 1]
    words = last[1:].to(torch.int64) & 0xFFFFFFFF
    return last[0].to(torch.int64) + _popcount64(words).sum()


def _popcount64(v: torch.Tensor) -> torch.Tensor:
    v = v - ((v >> 1) & 0x5555555555555555)
    v = (v & 0x3333333333333333) + ((v >> 2) & 0x3333333333333333)
    v = (v + (v >> 4)) & 0x0F0F0F0F0F0F0F0F
    return ((v * 0x0101010101010101) & 0xFFFFFFFFFFFFFFFF) >> 56


def decode_ref(meta: torch.Tensor, values: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """Rebuild the dense tensor into ``out`` (its shape defines n) -- torch reference."""
    n = out.numel()
    P = npages(n)
    m = meta.view(P, META)
    words = m[:, 1:].to(torch.int64) & 0xFFFFFFFF
    shifts = torch.arange(32, device=meta.device, dtype=torch.int64)
    nz = ((words.unsqueeze(-1) >> shifts) & 1).bool().reshape(-1)[:n]
    flat = torch.zeros(n, dtype=torch.int32, device=out.device)
    k = int(nz.sum())
    flat[nz] = values.reshape(-1)[:k].view(torch.int32)
    out.reshape(-1).view(torch.int32).copy_(flat)
    return out


def encode(x: torch.Tensor, meta_out: torch.Tensor, values_out: torch.Tensor) -> torch.Tensor:
    """Encode x into meta_out [meta_numel(n)] and values_out [cap]; returns the 0-d int64 nnz
    (device tensor, no host sync).  Values beyond cap are dropped (the caller checks nnz <=
    cap before decoding)."""
    n = x.numel()
    if meta_out.numel() != meta_numel(n) or meta_out.dtype != torch.int32:
        raise ValueError("zs.encode: meta_out must be int32 [meta_numel(n)]")
    if x.is_cuda:
        from .. import _ext

        return _ext.ops().zs_encode(x.contiguous(), meta_out, values_out)
    meta, vals, nnz = encode_ref(x)
    meta_out.copy_(meta)
    k = min(nnz, values_out.numel())
    values_out[:k].copy_(vals[:k])
    return torch.tensor(nnz, dtype=torch.int64)


def decode(meta: torch.Tensor, values: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    if out.is_cuda:
        from .. import _ext

        _ext.ops().zs_decode(meta, values, out)
        return out
    return decode_ref(meta, values, out)
