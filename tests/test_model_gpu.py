"""End-to-end ConvNet on the GPU vs the PyTorch reference model (same weights)."""
import copy

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


class RefConvNet(nn.Module):
    """The reference model, verbatim topology (mnist_onegpu.py:11-31), eager PyTorch."""

    def __init__(self, in_features, num_classes=10):
        super().__init__()
        self.layer1 = nn.Sequential(nn.Conv2d(1, 16, 5, 1, 2), nn.BatchNorm2d(16), nn.ReLU(), nn.MaxPool2d(2, 2))
        self.layer2 = nn.Sequential(nn.Conv2d(16, 32, 5, 1, 2), nn.BatchNorm2d(32), nn.ReLU(), nn.MaxPool2d(2, 2))
        self.fc = nn.Linear(in_features, num_classes)

    def forward(self, x):
        out = self.layer2(self.layer1(x))
        return self.fc(out.reshape(out.size(0), -1))


def _compare(mode, gpu, H=64, B=3, steps=2):
    from torch_distributed_sandbox_amd.models import ConvNet, fc_in_features
    from torch_distributed_sandbox_amd.ops import SGD, CrossEntropyLoss

    torch.manual_seed(0)
    ours = ConvNet(image_shape=(H, H), mode=mode)
    ref = RefConvNet(fc_in_features((H, H))).double()
    ref.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in ours.state_dict().items()})
    ours = ours.to(gpu)
    opt = SGD(ours.parameters(), 0.05)
    ropt = torch.optim.SGD(ref.parameters(), 0.05)
    crit = CrossEntropyLoss()
    for s in range(steps):
        x = torch.rand(B, 1, H, H, device=gpu)
        y = torch.randint(0, 10, (B,), device=gpu)
        loss = crit(ours(x), y)
        opt.zero_grad()
        loss.backward()
        rloss = nn.functional.cross_entropy(ref(x.double().cpu()), y.cpu())
        ropt.zero_grad()
        rloss.backward()
        assert abs(loss.item() - rloss.item()) < 1e-4 * max(1, abs(rloss.item())), (loss.item(), rloss.item())
        rp = dict(ref.named_parameters())
        for n, p in ours.named_parameters():
            g, rg = p.grad.double().cpu(), rp[n].grad
            if n.endswith("0.bias"):
                # conv bias before BN: analytically zero gradient, both sides are rounding
                # noise; bound it by the magnitude of the matching conv weight gradient
                wg = rp[n.replace("bias", "weight")].grad.abs().max().item()
                assert (g - rg).abs().max().item() <= 1e-3 * wg + 1e-5, f"step {s} {n}"
                continue
            # relative L2 error: robust to the rare max-pool argmax flips that any
            # non-fp64 arithmetic produces on near-tied windows
            rel = ((g - rg).norm() / rg.norm().clamp_min(1e-30)).item()
            assert rel <= 2e-3, f"step {s} {n}: rel L2 err {rel:.3e}"
        opt.step()
        ropt.step()
    rb = dict(ref.named_buffers())
    for n, b in ours.named_buffers():
        if b.is_floating_point():
            assert (b.double().cpu() - rb[n]).abs().max().item() < 1e-4, n
        else:
            assert int(b.item()) == int(rb[n].item()), n


def test_convnet_layers_matches_reference(gpu):
    _compare("layers", gpu)


def test_convnet_auto_matches_reference(gpu):
    _compare("auto", gpu, H=128, B=2)


def test_ddp_world1_flat_buckets(gpu):
    from torch_distributed_sandbox_amd.models import ConvNet
    from torch_distributed_sandbox_amd.ops import SGD, CrossEntropyLoss
    from torch_distributed_sandbox_amd.parallel import DistributedDataParallel

    torch.manual_seed(0)
    m = ConvNet(image_shape=(32, 32), device=gpu)
    ref = copy.deepcopy(m)
    ddp = DistributedDataParallel(m)
    opt = ddp.attach_optimizer(SGD(m.parameters(), 0.1))
    x = torch.rand(2, 1, 32, 32, device=gpu)
    y = torch.tensor([1, 2], device=gpu)
    loss = CrossEntropyLoss()(ddp(x), y)
    opt.zero_grad()
    loss.backward()
    fg = ddp.flat_grad
    for p in m.parameters():
        assert p.grad.untyped_storage().data_ptr() == fg.untyped_storage().data_ptr()
    rl = CrossEntropyLoss()(ref(x), y)
    rl.backward()
    for (n, p), q in zip(m.named_parameters(), ref.parameters()):
        assert torch.allclose(p.grad, q.grad, rtol=1e-4, atol=1e-6), n
    opt.step()
    with torch.no_grad():
        for p, q in zip(m.parameters(), ref.parameters()):
            assert torch.allclose(p, q - 0.1 * q.grad, rtol=1e-5, atol=1e-7)
