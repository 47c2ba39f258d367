"""Streaming head backward (head_bwd_stream_kernel, TDS_HEAD_BWD_NW=0) and the lane-per-column
forms (4 / 8): dW / g2m / BN2 grads / the fused W update against the y2 path, and timing."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timeit(fn, n=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / n, 4)


def run(P, B=5, NC=10, timing=False):
    import torch_distributed_sandbox_amd as tds
    ops = tds._ext.ops()
    dev = torch.device("cuda", 0)
    Q = P // 2
    torch.manual_seed(P)
    y2 = torch.randn(B, P, P, 32, device=dev)
    b2 = torch.zeros(32, device=dev)
    g2 = torch.rand(32, device=dev) + 0.5
    be2 = torch.randn(32, device=dev) * 0.1
    wfc = torch.randn(NC, 32 * Q * Q, device=dev) * 0.01
    bfc = torch.randn(NC, device=dev)
    partial2 = torch.stack([y2.double().sum((0, 1, 2)), (y2.double() ** 2).sum((0, 1, 2))], 1).contiguous()
    ya = torch.empty(B, 32 * Q * Q, device=dev)
    _, stats2, aff2 = ops.fused_head_forward(y2, partial2, b2, g2, be2, None, None, None, 0.1, 1e-5, wfc, bfc, None, ya)
    fw = {}
    for f in ("1", "0"):
        os.environ["TDS_HEAD_FWD"] = f
        ya_f = torch.empty_like(ya)
        xo = torch.empty_like(ya)
        r = ops.fused_head_forward(y2, partial2, b2, g2, be2, None, None, None, 0.1, 1e-5, wfc, bfc, xo, ya_f)
        fw[f] = [t.clone() for t in r] + [ya_f, xo]
        if timing:
            fw["ms" + f] = timeit(lambda: ops.fused_head_forward(y2, partial2, b2, g2, be2, None, None, None, 0.1, 1e-5,
                                                                 wfc, bfc, None, ya_f))
    os.environ.pop("TDS_HEAD_FWD")
    print(P, "fwd wide vs narrow maxdiff", [float((u - v).abs().max()) for u, v in zip(fw["0"], fw["1"])],
          {k: v for k, v in fw.items() if k.startswith("ms")}, flush=True)
    dl = torch.randn(B, NC, device=dev)
    ref = [t.clone() for t in ops.fused_head_backward_g2m(dl, y2, stats2, aff2, g2, wfc, None, 1.0, True)]
    out = {}
    for nw in ("0", "4", "8"):
        os.environ["TDS_HEAD_BWD_NW"] = nw
        dW = torch.full_like(wfc, 7.0)
        r = ops.fused_head_backward_g2m(dl, y2, stats2, aff2, g2, wfc, dW, 1.0, True, ya)
        res = {"dW": float((r[0] - ref[0]).abs().max()), "g2m": float((r[4] - ref[4]).abs().max()),
               "dg": float((r[2] - ref[2]).abs().max()), "db": float((r[3] - ref[3]).abs().max()),
               "kbuf": float((r[5] - ref[5]).abs().max())}
        w0 = wfc.clone()
        r = ops.fused_head_backward_g2m(dl, y2, stats2, aff2, g2, wfc, dW, 1.0, True, ya, 0.5)
        res["upd"] = float((wfc - (w0 - 0.5 * ref[0])).abs().max())
        wfc.copy_(w0)
        if timing:
            res["ms"] = timeit(lambda: ops.fused_head_backward_g2m(dl, y2, stats2, aff2, g2, wfc, dW, 1.0, True, ya))
            res["ms_upd"] = timeit(lambda: ops.fused_head_backward_g2m(dl, y2, stats2, aff2, g2, wfc, dW, 1.0, True,
                                                                       ya, 1e-12))
            wfc.copy_(w0)
        out[nw] = res
    os.environ.pop("TDS_HEAD_BWD_NW")
    print(P, out, flush=True)


if __name__ == "__main__":
    run(64)
    run(1500, timing=True)
