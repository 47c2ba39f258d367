import os, sys
sys.path.insert(0, '/root/repo')
import torch
import torch_distributed_sandbox_amd as tds
ops = tds._ext.ops()
gpu = torch.device('cuda', 0)
for P in (64, 130):
    torch.manual_seed(P + 1)
    B, NC = 5, 10
    Q = P // 2
    y2 = torch.randn(B, P, P, 32, device=gpu)
    b2 = torch.randn(32, device=gpu) * 0.1
    g2 = torch.rand(32, device=gpu) + 0.5
    be2 = torch.randn(32, device=gpu) * 0.1
    wfc = torch.randn(NC, 32 * Q * Q, device=gpu) * 0.01
    bfc = torch.randn(NC, device=gpu)
    yc = (y2 - b2).double()
    partial2 = torch.stack([yc.sum((0, 1, 2)), (yc * yc).sum((0, 1, 2))], dim=1).contiguous()
    ya = torch.empty(B, 32 * Q * Q, device=gpu)
    logits, stats2, aff2 = ops.fused_head_forward(y2, partial2, b2, g2, be2, None, None, None, 0.1, 1e-5, wfc, bfc, None, ya)
    dl = torch.randn(B, NC, device=gpu)
    r_y2 = ops.fused_head_backward_g2m(dl, y2, stats2, aff2, g2, wfc, None, 1.0, True)
    r_ya = ops.fused_head_backward_g2m(dl, y2, stats2, aff2, g2, wfc, None, 1.0, True, ya)
    torch.cuda.synchronize()
    d = (r_ya[4] - r_y2[4]).abs()
    bad = (d > 1e-5).nonzero()
    print(P, 'g2m nbad', bad.shape[0], 'of', d.numel())
    if bad.shape[0]:
        print(' b', bad[:, 0].unique().tolist()[:10], 'py', bad[:, 1].unique().tolist()[:10], 'px', bad[:, 2].unique().tolist()[:40], 'c', bad[:, 3].unique().tolist())
        print(' sample ya', r_ya[4][tuple(bad[0].tolist())].item(), 'y2', r_y2[4][tuple(bad[0].tolist())].item())
    for k, nm in enumerate(("dW", "dbfc", "dg2", "dbe2", "g2m", "kbuf")):
        print('  ', nm, (r_ya[k] - r_y2[k]).abs().max().item(), r_y2[k].abs().max().item())
