"""One fused-plan training step on an image past every 32-bit / 2 GiB boundary: B=1, H=24000
(x alone is 2.3 GB, the fc weight 11.5 G parameters = 46 GB), checked against a chunked fp64
reference computed on the same GPU (the OOM story of the reference, README.md:9-15, scaled to
288 GB per MI355X).  The reference runs the reference model's ops (Conv2d -> BatchNorm2d(train) ->
ReLU -> MaxPool2d, twice, then Linear and CrossEntropy, mnist_onegpu.py:14-24) in fp64, row chunk
by row chunk, with the convolutions as unfold + GEMM."""
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


def test_one_step_beyond_2gib(gpu):
    from torch_distributed_sandbox_amd.models import ConvNet
    from torch_distributed_sandbox_amd.ops import CrossEntropyLoss

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
    for p in m.parameters():
        p.grad = None
    del loss
    # nothing of the step outlives its backward: the fc weight and x remain
    held = torch.cuda.memory_allocated(gpu)
    assert held < m.fc.weight.numel() * 4 + x.numel() * 4 + 2**30, held
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
    del p1
    torch.testing.assert_close(bn2.running_mean.double(), 0.1 * mean2, rtol=1e-4, atol=1e-6)
    Q = P // 2
    W = m.fc.weight.detach().view(10, 32, Q, Q)
    logits = m.fc.bias.detach().double().clone()
    for r0 in range(0, Q, 256):
        r1 = min(Q, r0 + 256)
        logits += torch.einsum("jchw,chw->j", W[:, :, r0:r1].double(), p2[:, r0:r1])
    del p2
    ref = float(F.cross_entropy(logits.unsqueeze(0), y))
    assert abs(ours - ref) <= 1e-4 * max(1.0, abs(ref)), (ours, ref)
