"""Host-side pieces of the native kernels that run without a GPU: the conv2 backward walk
table (tds_conv2_bwd_walk, conv2_bwd.hip) that every rolling-window workgroup follows."""
import collections

import pytest
import torch

from torch_distributed_sandbox_amd import _ext

START, END = 1 << 31, 1 << 30


def _table(B, tr, tc, nwg, seg=24):
    t = _ext.ops().conv2_bwd_walk_table(B, tr, tc, nwg, seg)
    assert t.dtype == torch.int32 and t.dim() == 2 and t.shape[1] == nwg
    return t.to(torch.int64) & 0xFFFFFFFF


def _decode(v):
    return bool(v & START), bool(v & END), (v >> 24) & 63, (v >> 12) & 4095, v & 4095


@pytest.mark.parametrize("B,tr,tc,nwg", [(5, 188, 94, 256), (5, 188, 94, 248), (1, 3, 2, 7), (2, 50, 1, 4),
                                         (3, 25, 9, 512), (2, 16, 8, 256), (1, 7, 1, 7)])
def test_walk_covers_every_tile_once_in_vertical_segments(B, tr, tc, nwg):
    t = _table(B, tr, tc, nwg)
    seen = collections.Counter()
    lens = []
    for w in range(nwg):
        col = [int(v) for v in t[:, w]]
        n = 0
        while n < len(col) and not (col[n] & END):
            n += 1
        lens.append(n)
        # after the list: end-marked copies of the last tile, as many as the staging's look-ahead
        # reads past a list (tile k + 6 at its last iteration with three register sets; (2, 16, 8,
        # 256): one tile per workgroup, every list the longest -- with too few the last workgroup
        # read past the table)
        assert len(col) - n >= 6
        for v in col[n:]:
            assert v & END and (v & ~(START | END)) == ((col[n - 1] & ~START) if n else 0)
        prev = None
        for k in range(n):
            start, _, b, r, c = _decode(col[k])
            seen[(b, r, c)] += 1
            if not start:  # inside a segment: the tile right below the previous one
                pb, pr, pc = prev
                assert (b, r, c) == (pb, pr + 1, pc)
            prev = (b, r, c)
    assert set(seen) == {(b, r, c) for b in range(B) for r in range(tr) for c in range(tc)}
    assert max(seen.values()) == 1
    # balanced: the last partial round is cut into near-equal runs, so the longest list (the
    # kernel's critical path) is within 2 tiles of the ideal share
    total = B * tr * tc
    assert max(lens) <= -(-total // nwg) + 2


def test_walk_rejects_unsupported_sizes():
    with pytest.raises(RuntimeError, match="unsupported"):
        _ext.ops().conv2_bwd_walk_table(64, 10, 10, 8, 24)  # B > 63 (6-bit image field)
    with pytest.raises(RuntimeError, match="unsupported"):
        _ext.ops().conv2_bwd_walk_table(1, 5000, 10, 8, 24)  # > 4095 tile rows
