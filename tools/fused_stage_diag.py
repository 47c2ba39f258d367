"""Stage-by-stage check of the fused plan vs fp64 autograd at one size (intermediates + grads)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
import torch_distributed_sandbox_amd as tds

ops = tds._ext.ops()
dev = torch.device("cuda", 0)


def unpack(c, C):
    b = c.contiguous().view(torch.bfloat16)
    return b[..., :C].float() + b[..., C:2 * C].float()


def rel(a, b):
    a = a.detach().double().cpu(); b = b.detach().double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


def main(H, B):
    torch.manual_seed(0)
    x = torch.rand(B, 1, H, H, device=dev)
    w1 = torch.randn(16, 1, 5, 5, device=dev) * 0.2; b1 = torch.randn(16, device=dev) * 0.1
    g1 = torch.rand(16, device=dev) + 0.5; be1 = torch.randn(16, device=dev) * 0.1
    w2 = torch.randn(32, 16, 5, 5, device=dev) * 0.05; b2 = torch.randn(32, device=dev) * 0.1
    g2 = torch.rand(32, device=dev) + 0.5; be2 = torch.randn(32, device=dev) * 0.1
    Q = H // 4
    wfc = torch.randn(10, 32 * Q * Q, device=dev) * 0.01; bfc = torch.randn(10, device=dev)
    # fp64 reference with autograd on every stage
    P = [t.double().cpu().requires_grad_(True) for t in (w1, b1, g1, be1, w2, b2, g2, be2, wfc, bfc)]
    xr = x.double().cpu()
    y1 = F.conv2d(xr, P[0], P[1], padding=2)
    p1r = F.max_pool2d(F.relu(F.batch_norm(y1, None, None, P[2], P[3], True, 0.1, 1e-5)), 2, 2)
    p1r.retain_grad()
    y2r = F.conv2d(p1r, P[4], P[5], padding=2)
    y2r.retain_grad()
    p2 = F.max_pool2d(F.relu(F.batch_norm(y2r, None, None, P[6], P[7], True, 0.1, 1e-5)), 2, 2)
    logits_r = F.linear(p2.reshape(B, -1), P[8], P[9])
    dl = torch.randn(B, 10, device=dev)
    logits_r.backward(dl.double().cpu())
    # fused
    p1, idx1, st1, gram = ops.fused_l1_forward(x, w1, b1, g1, be1, None, None, None, 0.1, 1e-5)
    print(f"H={H} B={B}")
    print("  p1      ", rel(unpack(p1, 16).permute(0, 3, 1, 2), p1r))
    wp, wd = ops.conv2_pack(w2)
    y2, part2 = ops.fused_conv2_forward(p1, wp, b2)
    print("  y2      ", rel(y2.permute(0, 3, 1, 2), y2r))
    logits, st2, aff2 = ops.fused_head_forward(y2, part2, b2, g2, be2, None, None, None, 0.1, 1e-5, wfc, bfc)
    print("  logits  ", rel(logits, logits_r))
    dW, dbfc, dg2, dbe2, dy2 = ops.fused_head_backward(dl, y2, st2, aff2, g2, wfc, None, 1.0)
    print("  dW      ", rel(dW, P[8].grad), " dg2", rel(dg2, P[6].grad), " dbe2", rel(dbe2, P[7].grad))
    print("  dy2     ", rel(unpack(dy2, 32).permute(0, 3, 1, 2), y2r.grad))
    dp1, dw2, db2 = ops.fused_conv2_backward(dy2, p1, wd, True, 1.0)
    print("  dp1     ", rel(dp1.permute(0, 3, 1, 2), p1r.grad))
    print("  dw2     ", rel(dw2, P[4].grad))
    dw1, db1, dg1, dbe1 = ops.fused_l1_backward(dp1, x, p1, idx1, w1, b1, g1, st1, gram, 1.0)
    print("  dw1     ", rel(dw1, P[0].grad), " dg1", rel(dg1, P[2].grad), " dbe1", rel(dbe1, P[3].grad))
    # conv2 backward fed with the exact fp64 dy2 / p1 (isolates the kernels from upstream error)
    def pack(t):
        hi = t.to(torch.bfloat16); lo = (t - hi.float()).to(torch.bfloat16)
        return torch.cat([hi, lo], -1).contiguous().view(torch.float32)
    dy2x = y2r.grad.permute(0, 2, 3, 1).float().to(dev)
    p1x = p1r.detach().permute(0, 2, 3, 1).float().to(dev)
    dp1b, dw2b, _ = ops.fused_conv2_backward(pack(dy2x), pack(p1x), wd, True, 1.0)
    print("  [exact inputs] dp1", rel(dp1b.permute(0, 3, 1, 2), p1r.grad), " dw2", rel(dw2b, P[4].grad))


if __name__ == "__main__":
    for H, B in ((128, 2), (256, 2), (512, 2)):
        main(H, B)
