"""A/B timing of the layer-1 forward (conv1 + BN1 + ReLU + pool) at the bench shape:
TDS_L1_CONV=1 (exact fp32 MFMA) vs the default bf16x3 kernel; also the sparse backward."""
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
    from torch_distributed_sandbox_amd.ops import functional as TF
    ops = tds._ext.ops()
    dev = torch.device("cuda", 0)
    B, H = 5, int(os.environ.get("H", 3000))
    torch.manual_seed(0)
    src = torch.randint(0, 256, (B, 28, 28), dtype=torch.uint8, device=dev)
    x = TF.upsample_bilinear_u8(src, H, H)
    w1 = torch.randn(16, 1, 5, 5, device=dev) * 0.2
    b1 = torch.randn(16, device=dev) * 0.1
    g1 = torch.rand(16, device=dev) + 0.5
    be1 = torch.randn(16, device=dev) * 0.1
    res = {}
    for rep in range(2):
        for ver in ("1", "2"):
            os.environ["TDS_L1_CONV"] = ver
            res.setdefault(f"l1_fwd_v{ver}", []).append(
                timeit(lambda: ops.fused_l1_forward(x, w1, b1, g1, be1, None, None, None, 0.1, 1e-5)))
    os.environ.pop("TDS_L1_CONV")
    # backward: sparse VALU (TDS_L1_BWD=1) vs MFMA (default) on the forward's saved tensors
    p1, idx1, stats1, gram = ops.fused_l1_forward(x, w1, b1, g1, be1, None, None, None, 0.1, 1e-5)
    dp1 = torch.randn(B, H // 2, H // 2, 16, device=dev) * 1e-3
    outs = {}
    for ver in ("1", "0"):
        os.environ["TDS_L1_BWD"] = ver
        outs[ver] = [t.clone() for t in ops.fused_l1_backward(dp1, x, p1, idx1, w1, b1, g1, stats1, gram, 1.0)]
        res[f"l1_bwd_{'sparse' if ver == '1' else 'mfma'}"] = timeit(
            lambda: ops.fused_l1_backward(dp1, x, p1, idx1, w1, b1, g1, stats1, gram, 1.0))
    os.environ.pop("TDS_L1_BWD")
    res["l1_bwd_rel_err"] = [float((u - v).norm() / v.norm().clamp_min(1e-30)) for u, v in zip(outs["0"], outs["1"])]
    print(res, flush=True)


if __name__ == "__main__":
    main()
