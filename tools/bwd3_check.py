"""conv2 backward v3 (producer/consumer waves, TDS_CONV2_BWD=3) against v2: dp1 must match
bit for bit (same per-tile arithmetic), dw2/db2 to fp32 rounding (the per-workgroup tile sets
differ, so the wgrad partial sums are added in another order); then timing at the bench shape."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def pack_hilo(p):
    hi = p.to(torch.bfloat16)
    lo = (p - hi.float()).to(torch.bfloat16)
    return torch.cat([hi, lo], dim=-1).contiguous().view(torch.float32)


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


def case(ops, dev, B, P, timing=False):
    Q = P // 2
    torch.manual_seed(P)
    y2 = torch.randn(B, P, P, 32, device=dev)
    g2m = torch.randn(B, 32, Q, Q, device=dev)
    aff2 = torch.cat([torch.rand(32, device=dev) + 0.5, torch.randn(32, device=dev)])
    kbuf = torch.randn(96, device=dev) * 0.01
    p1 = pack_hilo(torch.relu(torch.randn(B, P, P, 16, device=dev)))
    w2 = torch.randn(32, 16, 5, 5, device=dev) * 0.05
    _, wd = ops.conv2_pack(w2)
    out = {}
    for v in ("2", "3"):
        os.environ["TDS_CONV2_BWD"] = v
        out[v] = [t.clone() for t in ops.fused_conv2_backward_y2(y2, g2m, aff2, kbuf, p1, wd, 1.0)]
        if timing:
            out["ms" + v] = timeit(lambda: ops.fused_conv2_backward_y2(y2, g2m, aff2, kbuf, p1, wd, 1.0))
    os.environ.pop("TDS_CONV2_BWD")
    r = {"P": P, "dp1_maxdiff": float((out["3"][0] - out["2"][0]).abs().max()),
         "dw2_rel": float((out["3"][1] - out["2"][1]).norm() / out["2"][1].norm()),
         "db2_rel": float((out["3"][2] - out["2"][2]).norm() / out["2"][2].norm())}
    if timing:
        r["ms_v2"], r["ms_v3"] = out["ms2"], out["ms3"]
    print(r, flush=True)


def main():
    import torch_distributed_sandbox_amd as tds
    ops = tds._ext.ops()
    dev = torch.device("cuda", 0)
    for B, P in ((2, 37), (2, 40), (1, 128), (3, 200)):
        case(ops, dev, B, P)
    case(ops, dev, 5, 1500, timing=True)
    # where v3's time goes (timing-only builds): 1 = no MFMAs, 3 = no global loads, 5 = no staging,
    # 6 = no g2m loads, 7 = no y2 loads
    B, P = 5, 1500
    Q = P // 2
    y2 = torch.randn(B, P, P, 32, device=dev)
    g2m = torch.randn(B, 32, Q, Q, device=dev)
    aff2 = torch.cat([torch.rand(32, device=dev) + 0.5, torch.randn(32, device=dev)])
    kbuf = torch.randn(96, device=dev) * 0.01
    p1 = pack_hilo(torch.relu(torch.randn(B, P, P, 16, device=dev)))
    _, wd = ops.conv2_pack(torch.randn(32, 16, 5, 5, device=dev) * 0.05)
    os.environ["TDS_CONV2_BWD"] = "3"
    res = {}
    for d in ("0", "1", "3", "5", "6", "7"):
        os.environ["TDS_CONV2_DIAG"] = d
        res["diag" + d] = timeit(lambda: ops.fused_conv2_backward_y2(y2, g2m, aff2, kbuf, p1, wd, 1.0))
    os.environ.pop("TDS_CONV2_DIAG")
    os.environ.pop("TDS_CONV2_BWD")
    print("v3 diag ms", res, flush=True)


if __name__ == "__main__":
    main()
