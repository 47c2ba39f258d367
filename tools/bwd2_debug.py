"""Compare the two fused conv2 backward kernels (TDS_CONV2_BWD=1 vs 2) on random inputs:
run-to-run determinism of v2 and where dp1 / dw2 differ (debug aid for conv2_bwd2.hip)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def pack_hilo(p):
    hi = p.to(torch.bfloat16)
    lo = (p - hi.float()).to(torch.bfloat16)
    return torch.cat([hi, lo], dim=-1).contiguous().view(torch.float32)


def main():
    import torch_distributed_sandbox_amd as tds
    ops = tds._ext.ops()
    dev = torch.device("cuda", 0)
    reps = int(os.environ.get("REPS", "6"))
    for P in [int(v) for v in (sys.argv[1:] or ["37", "64", "130", "200"])]:
        torch.manual_seed(P)
        B, Q = 2, P // 2
        y2 = torch.randn(B, P, P, 32, device=dev)
        g2m = torch.randn(B, 32, Q, Q, device=dev)
        aff2 = torch.cat([torch.rand(32, device=dev) + 0.5, torch.randn(32, device=dev)])
        kbuf = torch.randn(96, device=dev)
        p1 = pack_hilo(torch.relu(torch.randn(B, P, P, 16, device=dev)))
        w2 = torch.randn(32, 16, 5, 5, device=dev) * 0.05
        _, wd = ops.conv2_pack(w2)
        os.environ["TDS_CONV2_BWD"] = "1"
        r1 = [t.clone() for t in ops.fused_conv2_backward_y2(y2, g2m, aff2, kbuf, p1, wd, 1.0)]
        os.environ["TDS_CONV2_BWD"] = "2"
        nbad_runs = 0
        msgs = []
        for k in range(reps):
            junk = torch.full((B, P, P, 16), float("nan"), device=dev)  # poison the allocator's free list
            del junk
            r2 = ops.fused_conv2_backward_y2(y2, g2m, aff2, kbuf, p1, wd, 1.0)
            torch.cuda.synchronize()
            d = (r2[0] - r1[0]).abs()
            d = torch.nan_to_num(d, nan=1e30)
            bad = (d > 1e-4 * r1[0].abs().max().item()).nonzero()
            dw = ((r2[1] - r1[1]).abs().max() / r1[1].abs().max()).item()
            if bad.shape[0] or not dw < 1e-4:
                nbad_runs += 1
                rows = bad[:, 1].unique().tolist()
                cols = bad[:, 2].unique().tolist()
                msgs.append(f"  run{k}: nbad {bad.shape[0]} rows {rows[:10]} cols {cols[:16]} b {bad[:, 0].unique().tolist()} dw2 rel {dw:.2e}")
        print(f"P={P} pad={os.environ.get('TDS_B2_LDS_PAD', '0')}: {nbad_runs}/{reps} runs differ from v1", flush=True)
        for m in msgs[:4]:
            print(m, flush=True)
    os.environ.pop("TDS_CONV2_BWD", None)


if __name__ == "__main__":
    main()
