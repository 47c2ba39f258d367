"""End-to-end ConvNet on the GPU vs the PyTorch reference model (same weights)."""
import copy

import pytest
import torch
import torch.nn as nn

from _tf32ref import rel as _rel
from _tf32ref import tf32_convs

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


def near_tie_windows(a, rel=1e-5):
    """2x2 max-pool windows of the (post-ReLU, fp64) pooling input whose two largest values
    differ by less than rel x the layer's largest activation: windows an fp32 forward
    (relative rounding ~1e-6 of the activation scale) may resolve the other way."""
    B, C, H, W = a.shape
    w = a[:, :, : H // 2 * 2, : W // 2 * 2].reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5)
    top = w.reshape(B, C, H // 2, W // 2, 4).topk(2, dim=-1).values
    gap = top[..., 0] - top[..., 1]
    return int(((top[..., 0] > 0) & (gap <= rel * a.abs().max())).sum())


def _compare(mode, gpu, H=64, B=3, steps=2):
    from torch_distributed_sandbox_amd.models import ConvNet, fc_in_features
    from torch_distributed_sandbox_amd.ops import SGD, CrossEntropyLoss

    torch.manual_seed(0)
    ours = ConvNet(image_shape=(H, H), mode=mode)
    ref = RefConvNet(fc_in_features((H, H))).double()
    ref.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in ours.state_dict().items()})
    # the reference's precision class (TF32 convolutions), re-synced with ref every step: the
    # fused plan's fp16x2 conv2 is bounded by max(fixed tolerance, 1.5 x what TF32 makes)
    reft = tf32_convs(copy.deepcopy(ref))
    ours = ours.to(gpu)
    opt = SGD(ours.parameters(), 0.05)
    ropt = torch.optim.SGD(ref.parameters(), 0.05)
    crit = CrossEntropyLoss()
    pool_in = []
    for pool in (ref.layer1[3], ref.layer2[3]):
        pool.register_forward_hook(lambda mod, inp, out: pool_in.append(inp[0].detach()))
    for s in range(steps):
        # Re-sync the reference to our parameters every step: each step's gradients are then
        # checked on identical weights.  Free-running fp32 and fp64 trajectories drift apart
        # after one SGD step (at lr 0.05 a 1e-6 weight difference flips near-tied max-pool
        # windows), which made a multi-step comparison measure chaos, not kernel error.  The
        # update itself is pinned below against p - lr * p.grad.
        with torch.no_grad():
            for (n, p), q, qt in zip(ours.named_parameters(), ref.parameters(), reft.parameters()):
                q.copy_(p.detach().double().cpu())
                qt.copy_(q)
            for b, bt in zip(ref.buffers(), reft.buffers()):
                bt.copy_(b)
        x = torch.rand(B, 1, H, H, device=gpu)
        y = torch.randint(0, 10, (B,), device=gpu)
        loss = crit(ours(x), y)
        opt.zero_grad()
        loss.backward()
        pool_in.clear()
        rloss = nn.functional.cross_entropy(ref(x.double().cpu()), y.cpu())
        ties = sum(near_tie_windows(a) for a in pool_in)
        ropt.zero_grad()
        rloss.backward()
        reft.zero_grad()
        tloss = nn.functional.cross_entropy(reft(x.double().cpu()), y.cpu())
        tloss.backward()
        tl_err = abs(tloss.item() - rloss.item())
        assert abs(loss.item() - rloss.item()) < max(1e-4 * max(1, abs(rloss.item())), 1.5 * tl_err), \
            (loss.item(), rloss.item(), tloss.item())
        rp, rt = dict(ref.named_parameters()), dict(reft.named_parameters())
        for n, p in ours.named_parameters():
            g, rg = p.grad.double().cpu(), rp[n].grad
            if n.endswith("0.bias"):
                # conv bias before BN: analytically zero gradient, both sides are rounding
                # noise; bound it by the magnitude of the matching conv weight gradient
                wg = rp[n.replace("bias", "weight")].grad.abs().max().item()
                assert (g - rg).abs().max().item() <= 1e-3 * wg + 1e-5, f"step {s} {n}"
                continue
            # relative L2 error.  A non-fp64 forward can flip a near-tied max-pool window
            # against the fp64 reference; one flip reroutes one pooled gradient and moves a conv
            # weight gradient by ~1/sqrt(#windows) (5.6e-3 for one layer-2 flip at H=128, B=2,
            # tools/model_grad_check.py).  The wider bound applies only when the fp64 forward
            # itself shows a window tied to within fp32 rounding (near_tie_windows), and only to
            # the parameters a rerouted window reaches through a different input patch (conv
            # weights, BN1); BN2 and fc see the same tied value either way and stay at 2e-3.
            rel = ((g - rg).norm() / rg.norm().clamp_min(1e-30)).item()
            flip_reach = n.startswith("layer1.") or n.startswith("layer2.0.")
            tol = max(2e-2 if ties and flip_reach else 2e-3, 1.5 * _rel(rt[n].grad, rg))
            assert rel <= tol, f"step {s} {n}: rel L2 err {rel:.3e} > {tol:.3e} (near-tied windows: {ties})"
        before = {n: (p.detach().clone(), p.grad.detach().clone()) for n, p in ours.named_parameters()}
        opt.step()
        ropt.step()
        for n, p in ours.named_parameters():
            w0, g0 = before[n]
            assert torch.allclose(p.detach(), w0 - 0.05 * g0, rtol=1e-6, atol=1e-7), f"step {s} {n}: SGD update"
    rb, tb = dict(ref.named_buffers()), dict(reft.named_buffers())
    for n, b in ours.named_buffers():
        if b.is_floating_point():
            # reft's buffers: re-synced from ref, then updated by the last step's TF32 batch stats
            et = (tb[n] - rb[n]).abs().max().item()
            assert (b.double().cpu() - rb[n]).abs().max().item() < max(1e-4, 1.5 * et), n
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
