"""Time the pooled activation exchange's fc step (ops.head_update_pooled, mode 0) at the bench shape
for 1, 2 and 4 source ranks' gathered pooled inputs on one GPU (the W = 2 / 4 update of the default
exchange, parallel/factored.py "pooled"), with the bytes it moves and the rate.

  python tools/micro/pooled_update_timing.py [--ranks 1,2,4] [--iters 10]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import torch_distributed_sandbox_amd as tds  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="1,2,4")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    ops = tds._ext.ops()
    dev = torch.device("cuda", 0)
    B, P, NC = 5, 1500, 10
    Q = P // 2
    pb = ((Q + 3) // 4 * 4) * ((Q + 7) // 8 * 8)
    w = torch.randn(NC, 32 * Q * Q, device=dev) * 0.01
    b2 = torch.zeros(32, device=dev)
    for nr in [int(v) for v in a.ranks.split(",")]:
        ya_all = torch.randn(nr, B, 32, pb, device=dev).half()
        aff2 = torch.cat([torch.ones(32, device=dev), torch.zeros(32, device=dev)])
        rec = ops.head_pooled_record(aff2, b2, None)
        rec_all = rec.expand(nr, 128).contiguous()
        dl = torch.randn(nr * B, NC, device=dev) * 1e-3
        for _ in range(3):
            ops.head_update_pooled(dl, ya_all, rec_all, w, None, P, 1.0 / nr, 1e-6, 0)
        torch.cuda.synchronize()
        t = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                ops.head_update_pooled(dl, ya_all, rec_all, w, None, P, 1.0 / nr, 1e-6, 0)
            e1.record()
            torch.cuda.synchronize()
            t.append(e0.elapsed_time(e1) / a.iters)
        ms = sorted(t)[len(t) // 2]
        gb = (2 * w.numel() * 4 + ya_all.numel() * 2) / 1e9
        print(f"ranks {nr}: {ms:.4f} ms  {gb:.2f} GB  {gb / ms:.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
