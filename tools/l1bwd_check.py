"""Layer-1 backward: MFMA kernel vs the sparse VALU kernel on the forward's own p1/idx1 at
several shapes; per-output relative errors."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    import torch_distributed_sandbox_amd as tds
    ops = tds._ext.ops()
    dev = torch.device("cuda", 0)
    for B, H in ((2, 128), (3, 64), (2, 76), (1, 256)):
        torch.manual_seed(H)
        x = torch.rand(B, 1, H, H, device=dev)
        w1 = torch.randn(16, 1, 5, 5, device=dev) * 0.2
        b1 = torch.randn(16, device=dev) * 0.1
        g1 = torch.rand(16, device=dev) + 0.5
        be1 = torch.randn(16, device=dev) * 0.1
        p1, idx1, stats1, gram = ops.fused_l1_forward(x, w1, b1, g1, be1, None, None, None, 0.1, 1e-5)
        dp1 = torch.randn(B, H // 2, H // 2, 16, device=dev) * 1e-3
        outs = {}
        for ver in ("1", "0"):
            os.environ["TDS_L1_BWD"] = ver
            outs[ver] = [t.clone() for t in ops.fused_l1_backward(dp1, x, p1, idx1, w1, b1, g1, stats1, gram, 1.0)]
        os.environ.pop("TDS_L1_BWD")
        dw_s, dw_m = outs["1"][0].view(16, 25), outs["0"][0].view(16, 25)
        rel = float((dw_m - dw_s).norm() / dw_s.norm())
        per_tap = ((dw_m - dw_s).abs().max(0).values / dw_s.abs().max()).tolist()
        print({"B": B, "H": H, "dw1_rel": rel, "dg_rel": float((outs["0"][2] - outs["1"][2]).norm() / outs["1"][2].norm()),
               "dbe_rel": float((outs["0"][3] - outs["1"][3]).norm() / outs["1"][3].norm()),
               "worst_taps": sorted(range(25), key=lambda t: -per_tap[t])[:5]}, flush=True)


if __name__ == "__main__":
    main()
