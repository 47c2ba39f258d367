"""Time the fused head forward/backward ops in isolation at the bench shape (ya, fc weight
random or zero) to separate kernel cost from in-step effects.  Usage: python tools/micro/head_op_timing.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import torch_distributed_sandbox_amd as tds  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ops = tds._ext.ops()
    dev = torch.device("cuda", 0)
    B, P = 5, 1500
    Q = P // 2
    Q4, Q8 = (Q + 3) // 4, (Q + 7) // 8
    for fill in ("random", "zero"):
        g = torch.Generator(device=dev).manual_seed(0)
        mk = (lambda *s: torch.randn(*s, device=dev, generator=g)) if fill == "random" else \
            (lambda *s: torch.zeros(*s, device=dev))
        ya = mk(B, 32, Q4 * Q8 * 32).half()  # fp16 as the conv2 forward stores it (d = 1: no mag)
        wfc = mk(10, 32 * Q * Q) * 0.01
        bfc = torch.zeros(10, device=dev)
        b2, g2, be2 = torch.zeros(32, device=dev), torch.ones(32, device=dev), torch.zeros(32, device=dev)
        partial2 = torch.ones(32, 1, 2, device=dev, dtype=torch.float64)
        out = ops.fused_head_forward(ya, partial2, b2, g2, be2, None, None, None, 0.1, 1e-5, wfc, bfc, P)
        stats2, aff2 = out[1], out[2]
        dl = torch.randn(B, 10, device=dev)
        dw = torch.empty_like(wfc)
        tf = timeit(lambda: ops.fused_head_forward(ya, partial2, b2, g2, be2, None, None, None, 0.1, 1e-5, wfc, bfc, P))
        tb = timeit(lambda: ops.fused_head_backward(dl, ya, stats2, aff2, b2, g2, wfc, P, dw, 1.0, True))
        tu = timeit(lambda: ops.fused_head_backward(dl, ya, stats2, aff2, b2, g2, wfc, P, dw, 1.0, True, 1e-9))
        tn = timeit(lambda: ops.fused_head_backward(dl, ya, stats2, aff2, b2, g2, wfc, P, None, 1.0, False))
        gb_f = (ya.numel() * 2 + wfc.numel() * 4) / 1e9
        print(f"{fill:6s} head fwd op {tf:.3f} ms ({gb_f / tf:.2f} TB/s incl. small kernels) | bwd dW {tb:.3f} ms | "
              f"bwd dW+update {tu:.3f} ms | bwd no-dW {tn:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
