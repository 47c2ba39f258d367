"""Timing-only variants of the conv2 kernels (conv2_bf16x3.hip, TDS_CONV2_DIAG):
0 real, 1 no MFMA, 2 no LDS operand reads, 3 no global tile loads, 4 (forward v2 only) no y2 stores.
Tells which resource bounds each kernel at the bench shape (B=5, P=1500).
Outputs of variants 1-3 are garbage by design."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    import torch_distributed_sandbox_amd as tds

    ops = tds._ext.ops()
    B, P = int(os.environ.get("B", 5)), int(os.environ.get("P", 1500))
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    p1 = torch.randn(B, P, P, 16, device=dev)  # carrier bytes (values irrelevant for timing)
    dy2 = torch.randn(B, P, P, 32, device=dev)
    w2 = torch.randn(32, 16, 5, 5, device=dev) * 0.05
    b2 = torch.zeros(32, device=dev)
    wp, wd = ops.conv2_pack(w2)
    Q = P // 2
    g2m = torch.randn(B, 32, Q, Q, device=dev)
    aff2 = torch.cat([torch.rand(32, device=dev) + 0.5, torch.randn(32, device=dev)])
    kbuf = torch.randn(96, device=dev)
    res = {}
    for diag in (0, 1, 2, 3, 4):
        os.environ["TDS_CONV2_DIAG"] = str(diag)
        times = {}
        for name, fn in (("fwd", lambda: ops.fused_conv2_forward(p1, wp, b2)),
                         ("bwd(dgrad+wgrad)", lambda: ops.fused_conv2_backward(dy2, p1, wd, True, 1.0)),
                         ("wgrad_only", lambda: ops.fused_conv2_backward(dy2, p1, wd, False, 1.0)),
                         ("bwd_fused_y2", lambda: ops.fused_conv2_backward_y2(dy2, g2m, aff2, kbuf, p1, wd, 1.0))):
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            n = 10
            for _ in range(n):
                fn()
            e.record()
            torch.cuda.synchronize()
            times[name] = round(s.elapsed_time(e) / n, 4)
        times["dgrad_only"] = round(times["bwd(dgrad+wgrad)"] - times["wgrad_only"], 4)
        res[f"diag{diag}"] = times
        print(diag, times, flush=True)
    os.environ["TDS_CONV2_DIAG"] = "0"
    # A/B of the fused backward designs (TDS_CONV2_BWD: 1 = one 8-wave WG per CU, 2 = two 4-wave WGs)
    fn = lambda: ops.fused_conv2_backward_y2(dy2, g2m, aff2, kbuf, p1, wd, 1.0)  # noqa: E731
    ab = {}
    for rep in range(3):
        for ver in ("1", "2"):
            os.environ["TDS_CONV2_BWD"] = ver
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                fn()
            e.record()
            torch.cuda.synchronize()
            ab.setdefault(f"bwd_v{ver}", []).append(round(s.elapsed_time(e) / 10, 4))
    os.environ.pop("TDS_CONV2_BWD")
    print("fused backward A/B (ms):", ab, flush=True)
    fab = {}
    fwd = lambda: ops.fused_conv2_forward(p1, wp, b2)  # noqa: E731
    for rep in range(3):
        for ver in ("1", "2"):
            os.environ["TDS_CONV2_FWD"] = ver
            for _ in range(2):
                fwd()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                fwd()
            e.record()
            torch.cuda.synchronize()
            fab.setdefault(f"fwd_v{ver}", []).append(round(s.elapsed_time(e) / 10, 4))
    os.environ.pop("TDS_CONV2_FWD")
    print("forward A/B (ms):", fab, flush=True)
    ab.update(fab)
    print(json.dumps({"B": B, "P": P, "ms": res, "bwd_ab": ab}))


if __name__ == "__main__":
    main()
