"""One fused-plan training step on an image past every 32-bit / 2 GiB boundary: B=1, H=24000
(x alone is 2.3 GB, the fc weight 11.5 G parameters = 46 GB), checked against a chunked fp64
reference computed on the same GPU -- the loss, BN running statistics, the fc weight gradient
past flat index 2^31 and the conv2 weight / bias gradients (the OOM story of the reference, README.md:9-15, scaled to
288 GB per MI355X).  The reference runs the reference model's ops (Conv2d -> BatchNorm2d(train) ->
ReLU -> MaxPool2d, twice, then Linear and CrossEntropy, mnist_onegpu.py:14-24) in fp64, row chunk
by row chunk, with the convolutions as unfold + GEMM."""
import gc

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

H, ROWS = 24000, 48  # image edge; reference chunk height (output rows of layer 1)


@torch.no_grad()
def _conv_rows(x, w, b, r0, r1):
    """conv2d(x, w, b, padding=2) output rows [r0, r1) in fp64 by unfold + GEMM; x [C, H, W]."""
    C, Hh, Ww = x.shape
    lo, hi = max(0, r0 - 2), min(Hh, r1 + 2)
    xc = x[:, lo:hi].double()
    xc = F.pad(xc, (2, 2, 2 - (r0 - lo), 2 - (hi - r1)))  # rows/cols outside the image are zeros
    cols = F.unfold(xc.unsqueeze(0), 5)[0]  # [C*25, (r1-r0)*W]
    y = w.double().reshape(w.shape[0], -1) @ cols + b.double().view(-1, 1)
    return y.view(w.shape[0], r1 - r0, Ww)


@torch.no_grad()
def _bn_stats(x, w, b, nrows):
    s = torch.zeros(w.shape[0], dtype=torch.float64, device=x.device)
    q = torch.zeros_like(s)
    for r0 in range(0, nrows, ROWS):
        y = _conv_rows(x, w, b, r0, min(nrows, r0 + ROWS))
        s += y.sum((1, 2))
        q += (y * y).sum((1, 2))
    n = nrows * x.shape[2]
    mean = s / n
    return mean, q / n - mean * mean, n


@torch.no_grad()
def _layer(x, w, b, g, be, nrows):
    """conv -> BN(batch stats) -> ReLU -> 2x2 max-pool, fp64, chunked; returns (pooled, mean, var, n)."""
    mean, var, n = _bn_stats(x, w, b, nrows)
    a = g.double() / torch.sqrt(var + 1e-5)
    sh = be.double() - mean * a
    out = []
    for r0 in range(0, nrows, ROWS):
        y = _conv_rows(x, w, b, r0, min(nrows, r0 + ROWS))
        z = torch.relu(y * a.view(-1, 1, 1) + sh.view(-1, 1, 1))
        out.append(F.max_pool2d(z.unsqueeze(0), 2, 2)[0])
    return torch.cat(out, 1), mean, var, n


@torch.no_grad()
def _cols(x, r0, r1):
    """im2col of conv output rows [r0, r1) of x [C, H, W] (5x5, zero padding 2): [C*25, rows*W]."""
    C, Hh, Ww = x.shape
    lo, hi = max(0, r0 - 2), min(Hh, r1 + 2)
    xc = F.pad(x[:, lo:hi].double(), (2, 2, 2 - (r0 - lo), 2 - (hi - r1)))
    return F.unfold(xc.unsqueeze(0), 5)[0]


def test_one_step_beyond_2gib(gpu):
    from torch_distributed_sandbox_amd.models import ConvNet
    from torch_distributed_sandbox_amd.ops import CrossEntropyLoss

    # what earlier tests of the same process still hold (module-scoped fixtures, caches) is not this step's
    gc.collect()
    base = torch.cuda.memory_allocated(gpu)
    torch.manual_seed(0)
    m = ConvNet(image_shape=(H, H), device=gpu, mode="fused")
    g = torch.Generator(device=gpu).manual_seed(3)
    x = torch.rand(1, 1, H, H, device=gpu, generator=g)
    assert x.numel() * 4 > 2**31
    y = torch.tensor([4], device=gpu)
    loss = CrossEntropyLoss()(m(x), y)
    loss.backward()
    ours = float(loss.item())
    assert all(torch.isfinite(p.grad).all().item() for p in m.parameters())
    # gradient slices to check against fp64 below: conv2's weight / bias (the fp16x2 backward over
    # 144 M positions) and the fc weight's last two pooled rows of channel 31 of class 9 (flat
    # index ~10.4 G, far past 2^31)
    Qg = H // 4
    fc_tail = m.fc.weight.grad.view(10, 32, Qg, Qg)[9, 31, -2:].clone()
    dw2_ours, db2_ours = m.layer2[0].weight.grad.clone(), m.layer2[0].bias.grad.clone()
    for p in m.parameters():
        p.grad = None
    del loss
    # nothing of the step outlives its backward: the fc weight and x remain
    held = torch.cuda.memory_allocated(gpu) - base
    assert held < m.fc.weight.numel() * 4 + x.numel() * 4 + 2**30, (held, base)
    torch.cuda.empty_cache()
    bn1, bn2 = m.layer1[1], m.layer2[1]
    c1, c2 = m.layer1[0], m.layer2[0]
    # BN1 statistics over 576 M positions (running stats after one step, momentum 0.1)
    p1, mean1, var1, n1 = _layer(x[0], c1.weight, c1.bias, bn1.weight, bn1.bias, H)
    torch.testing.assert_close(bn1.running_mean.double(), 0.1 * mean1, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(bn1.running_var.double(), 0.9 + 0.1 * var1 * n1 / (n1 - 1), rtol=1e-5, atol=1e-7)
    del x
    torch.cuda.empty_cache()
    P = H // 2
    p2, mean2, var2, n2 = _layer(p1, c2.weight, c2.bias, bn2.weight, bn2.bias, P)
    # TF32 class (conv2_common.h): p1 and the conv2 weights each rounded once to 11 significant
    # bits, so the batch mean of channel c is off by at most
    # 2 * 2^-11 * sum_{ci,tap} |w2[c,ci,tap]| * mean(p1[ci]) (p1 >= 0), plus fp32 accumulation
    pm = p1.mean((1, 2))
    bound = 0.1 * (2.0 * 2.0 ** -11 * (c2.weight.double().abs().sum((2, 3)) @ pm)) * 1.05 + 1e-6
    err = (bn2.running_mean.double() - 0.1 * mean2).abs()
    assert bool((err <= bound).all()), (err.max().item(), (err / bound).max().item())
    Q = P // 2
    W = m.fc.weight.detach().view(10, 32, Q, Q)
    logits = m.fc.bias.detach().double().clone()
    for r0 in range(0, Q, 256):
        r1 = min(Q, r0 + 256)
        logits += torch.einsum("jchw,chw->j", W[:, :, r0:r1].double(), p2[:, r0:r1])
    ref = float(F.cross_entropy(logits.unsqueeze(0), y))
    # (TF32-class conv2: the 64^2 model tests bound the loss by TF32 convolutions' own error)
    assert abs(ours - ref) <= 1e-3 * max(1.0, abs(ref)), (ours, ref)
    # fc weight gradient past 2^31: dW[j] = dl[j] * X (batch 1, mean loss)
    dl = torch.softmax(logits, 0)
    dl[int(y)] -= 1.0
    # X carries conv2's forward rounding (p1 stored as fp16, <= 2^-11 per product) through BN2's
    # normalisation; a 32-bit index wrap would give O(1) errors
    ft_ref = dl[9] * p2[31, -2:]
    ft_err = (fc_tail.double() - ft_ref).abs().max().item()
    assert ft_err <= 5e-3 * ft_ref.abs().max().item(), (ft_err, ft_ref.abs().max().item())
    # conv2 weight / bias gradient: dL/dp2 = sum_j dl[j] W[j], then the fp64 chain
    dp2 = torch.zeros_like(p2)
    for r0 in range(0, Q, 256):
        r1 = min(Q, r0 + 256)
        dp2[:, r0:r1] = torch.einsum("j,jchw->chw", dl, W[:, :, r0:r1].double())
    del p2
    # fp64 chain BN2(train) -> ReLU -> MaxPool backward, then conv2's weight gradient as
    # dy @ im2col(p1)^T, chunk by chunk: pass 1 forms the BN2 backward sums, pass 2 the gradient
    # (one im2col per chunk and pass, shared by the conv recompute and the gradient GEMM)
    w2 = c2.weight.detach().double().view(32, 400)
    b2 = c2.bias.detach().double().view(32, 1)
    a2 = bn2.weight.detach().double() / torch.sqrt(var2 + 1e-5)
    sh2 = bn2.bias.detach().double() - mean2 * a2
    inv = 1.0 / torch.sqrt(var2 + 1e-5)

    def chunk(r0, r1):
        cols = _cols(p1, r0, r1)
        yc = (w2 @ cols + b2).view(32, r1 - r0, P)
        z = yc * a2.view(-1, 1, 1) + sh2.view(-1, 1, 1)
        r = torch.relu(z)
        _, idx = F.max_pool2d(r.unsqueeze(0), 2, 2, return_indices=True)
        dr = F.max_unpool2d(dp2[:, r0 // 2:r1 // 2].unsqueeze(0), idx, 2, 2, output_size=r.shape[-2:])[0]
        dz = dr * (z > 0)
        xh = (yc - mean2.view(-1, 1, 1)) * inv.view(-1, 1, 1)
        return cols, dz, xh

    sdz = torch.zeros(32, dtype=torch.float64, device=gpu)
    sdzx = torch.zeros_like(sdz)
    for r0 in range(0, P, ROWS):
        _, dz, xh = chunk(r0, min(P, r0 + ROWS))
        sdz += dz.sum((1, 2))
        sdzx += (dz * xh).sum((1, 2))
    dw2 = torch.zeros(32, 400, dtype=torch.float64, device=gpu)
    db2 = torch.zeros(32, dtype=torch.float64, device=gpu)
    sady = torch.zeros(32, dtype=torch.float64, device=gpu)
    for r0 in range(0, P, ROWS):
        cols, dz, xh = chunk(r0, min(P, r0 + ROWS))
        dy = a2.view(-1, 1, 1) * (dz - (sdz / n2).view(-1, 1, 1) - xh * (sdzx / n2).view(-1, 1, 1))
        dw2 += dy.reshape(32, -1) @ cols.t()
        db2 += dy.sum((1, 2))
        sady += dy.abs().sum((1, 2))
    rel = ((dw2_ours.double().view(32, 400) - dw2).norm() / dw2.norm()).item()
    # fp16x2-class rounding amplified by BN2's backward over 144 M positions (the 64^2 model test
    # measures 1.1e-2 for this gradient against 3.2e-2 for TF32 convolutions); an index wrap is O(1)
    print(f"fc tail max err {ft_err:.3e}, layer2.0.weight grad rel L2 err {rel:.3e}")
    assert rel <= 5e-2, f"layer2.0.weight grad rel L2 err {rel:.2e}"
    # conv bias before BN: analytically zero (and cancelled by BN2 in the forward), both sides rounding
    # noise -- dy2 is rounded once to 11 significant bits per element (the TF32 class), so the sum is
    # off by at most 2^-11 sum |dy2| per channel (as tests/test_fused_gpu.py's conv2 backward test);
    # an index wrap gives O(sum |dy2|).  (Measured r6_s21: a max error of 2.7e-3 with g2m stored in
    # fp16, 4.2e-4 with g2m in fp32 -- the pooled gradient's extra rounding at the windows' argmax
    # shows in this sum of 144 M cancelling terms; the weight gradient above moved 2.30 -> 2.41e-2)
    db2_err = (db2_ours.double() - db2).abs()
    bound = sady * 2.0 ** -11 * 1.01 + 1e-9
    print(f"conv2 bias grad max err {db2_err.max().item():.3e}, its bound min {bound.min().item():.3e}; "
          f"ours max {db2_ours.abs().max().item():.3e}, ref max {db2.abs().max().item():.3e}")
    assert bool((db2_err <= bound).all()), (db2_err.max().item(), bound.min().item())
