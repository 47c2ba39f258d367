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


# ---------------------------------------------------------------------------- segmented form
class SegLayout:
    """Segments = flat element ranges ``(start, length)`` of one tensor, in order; each is cut
    into pages of ``PAGE`` (its last page partial), page g's record at ``meta[g * META]`` with
    offsets restarting per segment and its values in slot ``seg`` (a fixed capacity each).  The
    sharded exchange lays out (destination shard, row) segments of X this way, so one
    destination's share is one contiguous meta range and one run of slots
    (csrc/kernels/zs_exchange.hip, zs_seg_*)."""

    def __init__(self, segments, device):
        self.segments = [(int(a), int(n)) for a, n in segments]
        starts, cnts, segs, first, npg = [], [], [], [], []
        for s, (a, n) in enumerate(self.segments):
            first.append(len(starts))
            k = npages(n) if n > 0 else 0
            npg.append(k)
            for p in range(k):
                starts.append(a + p * PAGE)
                cnts.append(min(PAGE, n - p * PAGE))
                segs.append(s)
        self.first, self.npg = first, npg
        self.npages = len(starts)
        dev = torch.device(device)
        self.pg_start = torch.tensor(starts, dtype=torch.int64, device=dev)
        self.pg_cnt = torch.tensor(cnts, dtype=torch.int32, device=dev)
        self.pg_seg = torch.tensor(segs, dtype=torch.int32, device=dev)
        self.seg_first = torch.tensor(first, dtype=torch.int32, device=dev)
        self.seg_npg = torch.tensor(npg, dtype=torch.int32, device=dev)

    @property
    def nseg(self) -> int:
        return len(self.segments)

    @property
    def meta_numel(self) -> int:
        return self.npages * META

    def meta_range(self, s0: int, s1: int) -> Tuple[int, int]:
        """[begin, end) of segments s0 .. s1-1 in the meta buffer (consecutive segments)."""
        g0 = self.first[s0] if s0 < self.nseg else self.npages
        g1 = self.first[s1] if s1 < self.nseg else self.npages
        return g0 * META, g1 * META


def seg_encode(x: torch.Tensor, lay: SegLayout, meta_out: torch.Tensor, vals_out: torch.Tensor,
               cap: int) -> torch.Tensor:
    """Encode the segments of x (flat) into meta_out [lay.meta_numel] and vals_out [nseg * cap];
    returns the per-segment counts, int64 [nseg] on x's device (no host sync)."""
    if x.is_cuda:
        from .. import _ext

        return _ext.ops().zs_seg_encode(x.contiguous(), lay.pg_start, lay.pg_cnt, lay.pg_seg, lay.seg_first,
                                        lay.seg_npg, meta_out, vals_out, int(cap))
    flat = x.reshape(-1)
    slots = vals_out.view(lay.nseg, cap) if lay.nseg else vals_out
    counts = torch.zeros(lay.nseg, dtype=torch.int64)
    for s, (a, n) in enumerate(lay.segments):
        if n == 0:
            continue
        m0, m1 = lay.meta_range(s, s + 1)
        meta, vals, nnz = encode_ref(flat[a:a + n])
        meta_out[m0:m1].copy_(meta)
        k = min(nnz, cap)
        slots[s, :k].copy_(vals[:k])
        counts[s] = nnz
    return counts


def seg_decode(meta: torch.Tensor, lay: SegLayout, vals: torch.Tensor, cap: int, out: torch.Tensor) -> torch.Tensor:
    """Rebuild the segments of ``out`` (flat ranges of ``lay``) from ``meta`` [lay.meta_numel] and
    the value slots ``vals`` [nseg * cap]; the counts must not exceed ``cap``."""
    if out.is_cuda:
        from .. import _ext

        _ext.ops().zs_seg_decode(meta, lay.pg_start, lay.pg_cnt, lay.pg_seg, vals, int(cap), out)
        return out
    flat = out.reshape(-1)
    slots = vals.view(lay.nseg, cap) if lay.nseg else vals
    for s, (a, n) in enumerate(lay.segments):
        if n == 0:
            continue
        m0, m1 = lay.meta_range(s, s + 1)
        decode_ref(meta[m0:m1], slots[s], flat[a:a + n])
    return out
