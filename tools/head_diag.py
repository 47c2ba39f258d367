"""A/B timing of the fused head kernels at the bench shape (B=5, P=1500): forward, backward
from y2 (LDS transpose) and backward from the saved argmax values ya (TDS_HEAD_BWD_NW=8|4 lane-per-column, 0 streaming)."""
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


def main():
    import torch_distributed_sandbox_amd as tds
    ops = tds._ext.ops()
    dev = torch.device("cuda", 0)
    B, P, NC = 5, int(os.environ.get("P", 1500)), 10
    Q = P // 2
    torch.manual_seed(0)
    y2 = torch.randn(B, P, P, 32, device=dev)
    b2 = torch.zeros(32, device=dev)
    g2 = torch.rand(32, device=dev) + 0.5
    be2 = torch.randn(32, device=dev) * 0.1
    wfc = torch.randn(NC, 32 * Q * Q, device=dev) * 0.01
    bfc = torch.randn(NC, device=dev)
    partial2 = torch.stack([y2.double().sum((0, 1, 2)), (y2.double() ** 2).sum((0, 1, 2))], 1).contiguous()
    ya = torch.empty(B, 32 * Q * Q, device=dev)
    dW = torch.empty_like(wfc)
    dl = torch.randn(B, NC, device=dev)
    res = {}
    res["fwd"] = timeit(lambda: ops.fused_head_forward(y2, partial2, b2, g2, be2, None, None, None, 0.1, 1e-5, wfc,
                                                       bfc, None, ya))
    fo = {}
    for mode in ("2", "1"):
        os.environ["TDS_HEAD_FWD"] = mode
        res[f"fwd_mode{mode}"] = timeit(lambda: ops.fused_head_forward(y2, partial2, b2, g2, be2, None, None, None, 0.1,
                                                                       1e-5, wfc, bfc, None, ya))
        lg = ops.fused_head_forward(y2, partial2, b2, g2, be2, None, None, None, 0.1, 1e-5, wfc, bfc, None, ya)[0]
        fo[mode] = (lg.clone(), ya.clone())
    os.environ.pop("TDS_HEAD_FWD")
    for mode in ("1",):
        res[f"fwd_mode{mode}_vs_2"] = {"logits_rel": float((fo[mode][0] - fo["2"][0]).norm() / fo["2"][0].norm()),
                                       "ya_maxdiff": float((fo[mode][1] - fo["2"][1]).abs().max())}
    _, stats2, aff2 = ops.fused_head_forward(y2, partial2, b2, g2, be2, None, None, None, 0.1, 1e-5, wfc, bfc, None, ya)
    res["bwd_y2"] = timeit(lambda: ops.fused_head_backward_g2m(dl, y2, stats2, aff2, g2, wfc, dW, 1.0, True))
    outs = {}
    for nw in ("8", "4", "0"):
        os.environ["TDS_HEAD_BWD_NW"] = nw
        res[f"bwd_ya_nw{nw}"] = timeit(lambda: ops.fused_head_backward_g2m(dl, y2, stats2, aff2, g2, wfc, dW, 1.0, True,
                                                                           ya))
        r = ops.fused_head_backward_g2m(dl, y2, stats2, aff2, g2, wfc, dW, 1.0, True, ya)
        outs[nw] = [t.clone() for t in r]
        w0 = wfc.clone()
        res[f"bwd_ya_upd_nw{nw}"] = timeit(lambda: ops.fused_head_backward_g2m(dl, y2, stats2, aff2, g2, wfc, dW, 1.0,
                                                                               True, ya, 1e-12))
        wfc.copy_(w0)
    os.environ.pop("TDS_HEAD_BWD_NW")
    names = ["dW", "dbfc", "dg2", "dbe2", "g2m", "kbuf"]
    for nw in ("4", "0"):
        res[f"maxdiff_nw{nw}_vs_nw8"] = {n: float((a - b).abs().max()) for n, a, b in zip(names, outs[nw], outs["8"])}
    # update path: W - lr*dW once, compare against the unfused result
    os.environ["TDS_HEAD_BWD_NW"] = "0"
    w0 = wfc.clone()
    r = ops.fused_head_backward_g2m(dl, y2, stats2, aff2, g2, wfc, dW, 1.0, True, ya, 0.5)
    res["upd_maxdiff"] = float((wfc - (w0 - 0.5 * r[0])).abs().max())
    wfc.copy_(w0)
    os.environ.pop("TDS_HEAD_BWD_NW")
    gb_fwd = (y2.numel() + wfc.numel() + ya.numel()) * 4 / 1e9
    gb_bwd = (ya.numel() + 2 * wfc.numel() + B * Q * Q * 32) * 4 / 1e9
    res["fwd_TBps"] = round(gb_fwd / res["fwd"], 3)
    res["bwd_ya_TBps"] = {nw: round(gb_bwd / res[f"bwd_ya_nw{nw}"], 3) for nw in ("8", "4", "0")}
    res["bwd_ya_upd_TBps"] = {nw: round((gb_bwd + wfc.numel() * 4 / 1e9) / res[f"bwd_ya_upd_nw{nw}"], 3)
                              for nw in ("8", "4", "0")}
    print(res, flush=True)


if __name__ == "__main__":
    main()
