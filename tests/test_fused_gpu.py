"""Numerics of the fused ConvNet plan (NHWC, bf16x3 conv2) vs fp64 PyTorch references."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ops():
    import torch_distributed_sandbox_amd as tds

    return tds._ext.ops()


def _err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return (a - b).abs().max().item(), b.abs().max().item()


def _check(a, b, rel, name=""):
    e, s = _err(a, b)
    assert e <= rel * s + 1e-12, f"{name}: max err {e:.3e} vs scale {s:.3e} (rel {e / max(s, 1e-30):.2e})"


def pack_hilo(x_nhwc):
    """fp32 [..., C] -> carrier fp32 [..., C/2... ] bytes = bf16 hi[C] | lo[C]."""
    hi = x_nhwc.to(torch.bfloat16)
    lo = (x_nhwc - hi.float()).to(torch.bfloat16)
    packed = torch.cat([hi, lo], dim=-1).contiguous()
    return packed.view(torch.float32)


def unpack_hilo(carrier, C):
    b = carrier.contiguous().view(torch.bfloat16)
    return b[..., :C].float() + b[..., C:2 * C].float()


@pytest.mark.parametrize("H", [68, 256, 264])
def test_layer1_forward(gpu, H):
    torch.manual_seed(0)
    B = 3
    x = torch.rand(B, 1, H, H, device=gpu)
    w1 = torch.randn(16, 1, 5, 5, device=gpu) * 0.2
    b1 = torch.randn(16, device=gpu) * 0.1
    g1 = torch.rand(16, device=gpu) + 0.5
    be1 = torch.randn(16, device=gpu) * 0.1
    rm, rv = torch.zeros(16, device=gpu), torch.ones(16, device=gpu)
    nbt = torch.zeros((), dtype=torch.long, device=gpu)
    p1, idx1, stats, gram = _ops().fused_l1_forward(x, w1, b1, g1, be1, rm, rv, nbt, 0.1, 1e-5)
    xd = x.double().cpu()
    y = F.conv2d(xd, w1.double().cpu(), b1.double().cpu(), padding=2)
    rmr, rvr = torch.zeros(16, dtype=torch.float64), torch.ones(16, dtype=torch.float64)
    z = F.batch_norm(y, rmr, rvr, g1.double().cpu(), be1.double().cpu(), True, 0.1, 1e-5)
    ref, ridx = F.max_pool2d(F.relu(z), 2, 2, return_indices=True)
    got = unpack_hilo(p1, 16).permute(0, 3, 1, 2)
    # p1 is stored as bf16 hi+lo (16 significant bits): <= 2^-16 relative representation error
    _check(got, ref, 2e-5, "p1")
    _check(rm, rmr, 1e-5, "running_mean")
    _check(rv, rvr, 1e-5, "running_var")
    assert int(nbt.item()) == 1
    # argmax: where pooled value > 0 the index must match the reference window position
    P = H // 2
    ri = ridx.view(B, 16, P, P)
    rr = (ri // H) % 2 * 2 + (ri % H) % 2
    mine = idx1.permute(0, 3, 1, 2).long().cpu()
    pos = ref > 1e-6
    assert ((mine & 3)[pos] == rr[pos]).float().mean().item() > 0.999
    # bit 2 of the argmax byte is the ReLU mask the backward uses (pooled value > 0)
    assert (((mine & 4) != 0) == (ref > 0)).float().mean().item() > 0.999
    # Gram of the zero-padded 5x5 patches and the patch sums (fp64 reference)
    pat = F.unfold(xd, 5, padding=2)  # [B, 25, H*W]
    G = torch.einsum("bkp,bjp->kj", pat, pat)
    S = pat.sum((0, 2))
    _check(gram[:625].view(25, 25), G, 2e-6, "G")
    _check(gram[625:], S, 2e-6, "S")


def test_conv2_forward(gpu):
    torch.manual_seed(0)
    B, P = 2, 40
    p = torch.relu(torch.randn(B, P, P, 16, device=gpu))
    w2 = torch.randn(32, 16, 5, 5, device=gpu) * 0.05
    b2 = torch.randn(32, device=gpu)
    wp, wd = _ops().conv2_pack(w2)
    y2, partial = _ops().fused_conv2_forward(pack_hilo(p), wp, b2)
    ref = F.conv2d(p.permute(0, 3, 1, 2).double().cpu(), w2.double().cpu(), b2.double().cpu(), padding=2)
    _check(y2.permute(0, 3, 1, 2), ref, 5e-5, "y2")
    # BN2 partials: sum over workgroups of (sum, sumsq) of y2 - b2
    s = partial.view(32, -1, 2).sum(1).cpu()
    yc = ref - b2.double().cpu().view(1, 32, 1, 1)
    _check(s[:, 0], yc.sum((0, 2, 3)), 1e-4, "sum")
    _check(s[:, 1], (yc * yc).sum((0, 2, 3)), 1e-4, "sumsq")


@pytest.mark.parametrize("P", [64, 128, 200])
def test_head_fwd_bwd(gpu, P):
    """BN2(batch stats) + ReLU + pool + fc forward/backward, incl. the dy2 build, vs fp64 autograd."""
    torch.manual_seed(P)
    B, NC = 3, 10
    Q = P // 2
    y2 = torch.randn(B, P, P, 32, device=gpu)
    b2 = torch.randn(32, device=gpu) * 0.1
    g2 = torch.rand(32, device=gpu) + 0.5
    be2 = torch.randn(32, device=gpu) * 0.1
    wfc = torch.randn(NC, 32 * Q * Q, device=gpu) * 0.01
    bfc = torch.randn(NC, device=gpu)
    yc = (y2 - b2).double()
    partial2 = torch.stack([yc.sum((0, 1, 2)), (yc * yc).sum((0, 1, 2))], dim=1).contiguous()  # [32][1][2]
    logits, stats2, aff2 = _ops().fused_head_forward(y2, partial2, b2, g2, be2, None, None, None, 0.1, 1e-5, wfc, bfc)
    yr = y2.permute(0, 3, 1, 2).double().cpu().requires_grad_(True)
    gr = g2.double().cpu().requires_grad_(True)
    ber = be2.double().cpu().requires_grad_(True)
    wr = wfc.double().cpu().requires_grad_(True)
    z = F.batch_norm(yr, None, None, gr, ber, True, 0.1, 1e-5)
    pz = F.max_pool2d(F.relu(z), 2, 2)
    ref = F.linear(pz.reshape(B, -1), wr, bfc.double().cpu())
    _check(logits, ref, 1e-5, "logits")
    dl = torch.randn(B, NC, device=gpu)
    ref.backward(dl.double().cpu())
    dW, dbfc, dg2, dbe2, dy2 = _ops().fused_head_backward(dl, y2, stats2, aff2, g2, wfc, None, 1.0)
    _check(dW, wr.grad, 1e-5, "dW")
    _check(dg2, gr.grad, 1e-5, "dgamma2")
    _check(dbe2, ber.grad, 1e-5, "dbeta2")
    _check(unpack_hilo(dy2, 32).permute(0, 3, 1, 2), yr.grad, 1e-4, "dy2")


@pytest.mark.parametrize("P", [64, 130])
def test_head_backward_from_saved_argmax(gpu, P):
    """head backward from the saved argmax values ya (head_bwd_ya_kernel) == the y2 path,
    and dW / dgamma / dbeta vs fp64 autograd."""
    torch.manual_seed(P + 1)
    B, NC = 5, 10
    Q = P // 2
    ops = _ops()
    y2 = torch.randn(B, P, P, 32, device=gpu)
    b2 = torch.randn(32, device=gpu) * 0.1
    g2 = torch.rand(32, device=gpu) + 0.5
    be2 = torch.randn(32, device=gpu) * 0.1
    wfc = torch.randn(NC, 32 * Q * Q, device=gpu) * 0.01
    bfc = torch.randn(NC, device=gpu)
    yc = (y2 - b2).double()
    partial2 = torch.stack([yc.sum((0, 1, 2)), (yc * yc).sum((0, 1, 2))], dim=1).contiguous()
    ya = torch.empty(B, 32 * Q * Q, device=gpu)
    logits, stats2, aff2 = ops.fused_head_forward(y2, partial2, b2, g2, be2, None, None, None, 0.1, 1e-5, wfc, bfc,
                                                  None, ya)
    # ya is y2 at the window argmax of the BN2 output: relu(a*ya + b) is the pooled activation
    yr = y2.permute(0, 3, 1, 2).double().cpu().requires_grad_(True)
    gr = g2.double().cpu().requires_grad_(True)
    ber = be2.double().cpu().requires_grad_(True)
    wr = wfc.double().cpu().requires_grad_(True)
    z = F.batch_norm(yr, None, None, gr, ber, True, 0.1, 1e-5)
    pz = F.max_pool2d(F.relu(z), 2, 2)
    a, b = aff2[:32].double().cpu(), aff2[32:].double().cpu()
    p_from_ya = torch.relu(a.view(1, 32, 1, 1) * ya.view(B, 32, Q, Q).double().cpu() + b.view(1, 32, 1, 1))
    _check(p_from_ya, pz, 1e-5, "relu(a*ya+b) vs pooled")
    ref = F.linear(pz.reshape(B, -1), wr, bfc.double().cpu())
    dl = torch.randn(B, NC, device=gpu)
    ref.backward(dl.double().cpu())
    r_y2 = ops.fused_head_backward_g2m(dl, y2, stats2, aff2, g2, wfc, None, 1.0, True)
    r_ya = ops.fused_head_backward_g2m(dl, y2, stats2, aff2, g2, wfc, None, 1.0, True, ya)
    for name, u, v in zip(("dW", "dbfc", "dgamma2", "dbeta2", "g2m", "kbuf"), r_ya, r_y2):
        _check(u, v, 1e-6, name + " (ya vs y2 path)")
    _check(r_ya[0], wr.grad, 1e-5, "dW")
    _check(r_ya[2], gr.grad, 1e-5, "dgamma2")
    _check(r_ya[3], ber.grad, 1e-5, "dbeta2")


@pytest.mark.parametrize("P", [40, 37, 128, 200])
def test_conv2_backward(gpu, P):
    torch.manual_seed(0)
    B = 2
    p = torch.relu(torch.randn(B, P, P, 16, device=gpu))
    w2 = torch.randn(32, 16, 5, 5, device=gpu) * 0.05
    dy = torch.randn(B, P, P, 32, device=gpu)
    wp, wd = _ops().conv2_pack(w2)
    dp1, dw2, db2 = _ops().fused_conv2_backward(pack_hilo(dy), pack_hilo(p), wd, True, 1.0)
    pr = p.permute(0, 3, 1, 2).double().cpu().requires_grad_(True)
    wr = w2.double().cpu().requires_grad_(True)
    br = torch.zeros(32, dtype=torch.float64, requires_grad=True)
    F.conv2d(pr, wr, br, padding=2).backward(dy.permute(0, 3, 1, 2).double().cpu())
    _check(dp1.permute(0, 3, 1, 2), pr.grad, 5e-5, "dp1")
    _check(dw2, wr.grad, 5e-5, "dw2")
    _check(db2, br.grad, 5e-5, "db2")


def _fused_vs_ref(gpu, B, H, steps=2, lr=0.05):
    import torch.nn as nn

    from torch_distributed_sandbox_amd.models import ConvNet, fc_in_features
    from torch_distributed_sandbox_amd.ops import SGD, CrossEntropyLoss

    class Ref(nn.Module):
        def __init__(self, inf):
            super().__init__()
            self.layer1 = nn.Sequential(nn.Conv2d(1, 16, 5, 1, 2), nn.BatchNorm2d(16), nn.ReLU(), nn.MaxPool2d(2, 2))
            self.layer2 = nn.Sequential(nn.Conv2d(16, 32, 5, 1, 2), nn.BatchNorm2d(32), nn.ReLU(), nn.MaxPool2d(2, 2))
            self.fc = nn.Linear(inf, 10)

        def forward(self, x):
            o = self.layer2(self.layer1(x))
            return self.fc(o.reshape(o.size(0), -1))

    torch.manual_seed(0)
    ours = ConvNet(image_shape=(H, H), mode="fused")
    ref = Ref(fc_in_features((H, H))).double()
    ref.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in ours.state_dict().items()})
    ours = ours.to(gpu)
    opt = SGD(ours.parameters(), lr)
    ropt = torch.optim.SGD(ref.parameters(), lr)
    crit = CrossEntropyLoss()
    for s in range(steps):
        x = torch.rand(B, 1, H, H, device=gpu)
        y = torch.randint(0, 10, (B,), device=gpu)
        loss = crit(ours(x), y)
        opt.zero_grad()
        loss.backward()
        rl = F.cross_entropy(ref(x.double().cpu()), y.cpu())
        ropt.zero_grad()
        rl.backward()
        assert abs(loss.item() - rl.item()) <= 2e-4 * max(1.0, abs(rl.item())), (loss.item(), rl.item())
        rp = dict(ref.named_parameters())
        for n, p in ours.named_parameters():
            g, rg = p.grad.double().cpu(), rp[n].grad
            if n.endswith("0.bias"):  # analytically zero (bias before BN): rounding noise both sides
                wsc = rp[n.replace("bias", "weight")].grad.abs().max().item()
                assert (g - rg).abs().max().item() <= 1e-3 * wsc + 1e-6, f"step {s} {n}"
                continue
            # relative L2 (robust to rare argmax flips on near-tied pool windows)
            rel = ((g - rg).norm() / rg.norm().clamp_min(1e-30)).item()
            assert rel <= 1e-3, f"step {s} {n}: rel L2 err {rel:.3e}"
        opt.step()
        ropt.step()
    rb = dict(ref.named_buffers())
    for n, b in ours.named_buffers():
        if b.is_floating_point():
            e, sc = _err(b, rb[n])
            assert e <= 1e-4 * max(sc, 1.0), n
        else:
            assert int(b.item()) == int(rb[n].item()), n


def test_fused_model_matches_reference(gpu):
    _fused_vs_ref(gpu, B=3, H=64)


def test_fused_model_matches_reference_odd_pool(gpu):
    # P = 38 (not a multiple of the 32-column conv2 tile), Q = 19
    _fused_vs_ref(gpu, B=2, H=76, steps=1)


def test_fused_grads_land_in_ddp_bucket(gpu):
    from torch_distributed_sandbox_amd.models import ConvNet
    from torch_distributed_sandbox_amd.ops import CrossEntropyLoss
    from torch_distributed_sandbox_amd.parallel import DistributedDataParallel

    m = ConvNet(image_shape=(64, 64), device=gpu, mode="fused")
    d = DistributedDataParallel(m)
    x = torch.rand(2, 1, 64, 64, device=gpu)
    loss = CrossEntropyLoss()(d(x), torch.tensor([1, 2], device=gpu))
    loss.backward()
    v = d.grad_view(m.fc.weight)
    assert m.fc.weight.grad.data_ptr() == v.data_ptr()


@pytest.mark.parametrize("P", [37, 40, 130])
def test_conv2_backward_fused_with_bn2_pool(gpu, P):
    """fused_conv2_backward_y2 (dy2 rebuilt in LDS from y2 + g2m) vs the unfused path
    (dy2_build -> dy2 in HBM -> conv2 dgrad + wgrad)."""
    torch.manual_seed(P)
    B, NC = 2, 10
    Q = P // 2
    ops = _ops()
    y2 = torch.randn(B, P, P, 32, device=gpu)
    b2 = torch.randn(32, device=gpu) * 0.1
    g2 = torch.rand(32, device=gpu) + 0.5
    be2 = torch.randn(32, device=gpu) * 0.1
    wfc = torch.randn(NC, 32 * Q * Q, device=gpu) * 0.01
    bfc = torch.randn(NC, device=gpu)
    yc = (y2 - b2).double()
    partial2 = torch.stack([yc.sum((0, 1, 2)), (yc * yc).sum((0, 1, 2))], dim=1).contiguous()
    _, stats2, aff2 = ops.fused_head_forward(y2, partial2, b2, g2, be2, None, None, None, 0.1, 1e-5, wfc, bfc)
    dl = torch.randn(B, NC, device=gpu)
    _, _, _, _, dy2 = ops.fused_head_backward(dl, y2, stats2, aff2, g2, wfc, None, 1.0)
    _, _, _, _, g2m, kbuf = ops.fused_head_backward_g2m(dl, y2, stats2, aff2, g2, wfc, None, 1.0)
    p = torch.relu(torch.randn(B, P, P, 16, device=gpu))
    w2 = torch.randn(32, 16, 5, 5, device=gpu) * 0.05
    _, wd = ops.conv2_pack(w2)
    p1 = pack_hilo(p)
    dp1_r, dw2_r, db2_r = ops.fused_conv2_backward(dy2, p1, wd, True, 1.0)
    dp1, dw2, db2 = ops.fused_conv2_backward_y2(y2, g2m, aff2, kbuf, p1, wd, 1.0)
    _check(dp1, dp1_r, 1e-6, "dp1")
    _check(dw2, dw2_r, 1e-5, "dw2")
    # conv bias before BN: sum(dy2) is analytically zero, both sides are rounding noise
    assert (db2 - db2_r).abs().max().item() <= 1e-4 * dw2_r.abs().max().item()
