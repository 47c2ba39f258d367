"""How compressible is the fc input X on the bench data?  

X = maxpool2(ReLU(BN2(conv2(...)))) flattened: the rows the activation / sharded fc-gradient
exchanges (parallel/factored.py) put on the xGMI links, 360 MB per rank per step at 3000^2,
batch 5.  This runs the bench's model and data (same seeds, the fused plan), takes X from the
head-forward kernel's x_out and reports, after 0 and after --train-steps SGD steps:

* the fraction of exact zeros (overall and per channel),
* the bytes of a lossless zero-suppressed encoding (1 mask bit per value + the non-zero
  values, per 32-value group), relative to the dense fp32 rows.

    python tools/x_sparsity.py [--image-size 3000] [--batch-size 5] [--train-steps 20] [--data noise|mnist]

``--data noise``: the bench's sources (uniform random 28x28 levels); ``--data mnist``: the
trainer's SyntheticMNIST digits (dark background, bright strokes: data/synthetic.py).  Both go
through the bench's input path (uint8 levels upsampled on device).  The JSON also carries the
ratio of the exchange's real page format (parallel/zs.py: 2048-value pages, 64 mask words each
+ the non-zero values + the count slot) and the path ``choose_path`` picks with it at W = 2, 4, 8.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def fc_input(model, x):
    """X [B, 32*Q*Q] of one forward of the fused plan (no autograd, no state change except the
    BN running statistics)."""
    from torch_distributed_sandbox_amd import _ext

    ops = _ext.ops()
    conv1, bn1 = model.layer1[0], model.layer1[1]
    conv2, bn2 = model.layer2[0], model.layer2[1]
    fc = model.fc
    with torch.no_grad():
        p1, _, _, _, p1s = ops.fused_l1_forward(x, conv1.weight, conv1.bias, bn1.weight, bn1.bias, None, None, None,
                                           float(bn1.momentum), float(bn1.eps), None, None)
        wp, _ = ops.conv2_pack(conv2.weight)
        y2, partial2, ya, _ = ops.fused_conv2_forward(p1, wp, conv2.bias, bn2.weight)
        P = y2.shape[1]
        xo = torch.empty((x.shape[0], fc.weight.shape[1]), device=x.device, dtype=torch.float32)
        ops.fused_head_forward(ya, partial2, conv2.bias, bn2.weight, bn2.bias, None, None, None, float(bn2.momentum),
                               float(bn2.eps), fc.weight, fc.bias, P, xo)
    return xo


def stats(X, group=32):
    from torch_distributed_sandbox_amd.parallel import factored, zs

    zero = X == 0
    B, K = X.shape
    C = 32
    per_ch = zero.view(B, C, -1).float().mean(dim=(0, 2)).tolist()
    nz = int((~zero).sum())
    n = X.numel()
    mask_bytes = n / 8
    # per-group counts (one byte per group of 32 is enough to locate the compacted values)
    enc = mask_bytes + nz * 4 + n / group
    # the exchange's own format (factored._meta_row: records + count slot), per rank = per batch
    page_ratio = (nz + factored._meta_row(zs.meta_numel(n))) / n
    return {"zero_frac": round(1 - nz / n, 4), "zero_frac_per_channel": [round(v, 3) for v in per_ch],
            "dense_MB": round(n * 4 / 1e6, 1), "zero_suppressed_MB": round(enc / 1e6, 1),
            "ratio": round(enc / (n * 4), 4), "page_format_ratio": round(page_ratio, 4),
            "choose_path": {w: factored.choose_path(B, 10, K, w, x_ratio=page_ratio) for w in (2, 4, 8)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--image-size", type=int, default=3000)
    ap.add_argument("--batch-size", type=int, default=5)
    ap.add_argument("--train-steps", type=int, default=20)
    ap.add_argument("--data", default="noise", choices=["noise", "mnist"])
    args = ap.parse_args()
    from torch_distributed_sandbox_amd.data import synthetic_batch
    from torch_distributed_sandbox_amd.models import ConvNet
    from torch_distributed_sandbox_amd.ops import SGD, CrossEntropyLoss
    from torch_distributed_sandbox_amd.ops import functional as TF

    dev = torch.device("cuda", 0)
    H, B = args.image_size, args.batch_size
    torch.manual_seed(0)
    model = ConvNet(image_shape=(H, H), device=dev)
    opt = SGD(model.parameters(), 1e-4)
    crit = CrossEntropyLoss()
    pool = 16
    if args.data == "mnist":
        from torch_distributed_sandbox_amd.data import SyntheticMNIST

        ds = SyntheticMNIST(size=B * pool)
        s_, l_ = ds.batch(list(range(B * pool)))
        src, lab = s_.to(dev), l_.to(dev)
    else:
        src, lab = synthetic_batch(B * pool, (H, H), dev, seed=1234)
    src, lab = src.view(pool, B, 28, 28), lab.view(pool, B)
    out = {"image_size": H, "batch": B, "data": args.data}
    x = TF.upsample_bilinear_u8(src[0], H, H, levels=True)
    out["step0"] = stats(fc_input(model, x))
    for i in range(args.train_steps):
        x = TF.upsample_bilinear_u8(src[i % pool], H, H, levels=True)
        loss = crit(model(x), lab[i % pool])
        opt.zero_grad()
        loss.backward()
        opt.step()
    x = TF.upsample_bilinear_u8(src[args.train_steps % pool], H, H, levels=True)
    out[f"step{args.train_steps}"] = stats(fc_input(model, x))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
