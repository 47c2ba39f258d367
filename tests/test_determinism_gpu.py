"""Run-to-run determinism of the flagship training step ("determinism check
(two runs, bitwise compare with deterministic split-K reductions)").

Two identical runs of the bench step (fused plan, DDP world 1 with the overlapped fc
update, SGD) from the same seed and data must produce bit-identical losses, parameters
and BN buffers: every cross-workgroup reduction in the kernels is a fixed-order partial
reduction, not a float atomic.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(gpu, H, B, steps):
    from torch_distributed_sandbox_amd.data import synthetic_batch
    from torch_distributed_sandbox_amd.models import ConvNet
    from torch_distributed_sandbox_amd.ops import SGD, CrossEntropyLoss
    from torch_distributed_sandbox_amd.ops import functional as TF
    from torch_distributed_sandbox_amd.parallel import DistributedDataParallel

    torch.manual_seed(0)
    model = ConvNet(image_shape=(H, H), device=gpu)
    opt = SGD(model.parameters(), 1e-4)
    ddp = DistributedDataParallel(model, device_ids=[gpu.index], overlap_optimizer=True)
    ddp.attach_optimizer(opt)
    crit = CrossEntropyLoss()
    src, lab = synthetic_batch(B * steps, (H, H), gpu, seed=7)
    src = src.view(steps, B, 28, 28)
    lab = lab.view(steps, B)
    losses = []
    for i in range(steps):
        out = ddp(TF.upsample_bilinear_u8(src[i], H, H))
        loss = crit(out, lab[i])
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.detach().clone())
    ddp.wait_pending_updates()
    torch.cuda.synchronize()
    state = {k: v.detach().clone() for k, v in model.state_dict().items()}
    del model, opt, ddp
    return torch.stack(losses), state


@pytest.mark.parametrize("H,B", [(264, 3), (3000, 5)])
def test_training_step_bitwise_deterministic(gpu, H, B):
    l1, s1 = _run(gpu, H, B, steps=3)
    l2, s2 = _run(gpu, H, B, steps=3)
    assert torch.isfinite(l1).all()
    assert torch.equal(l1, l2), (l1.tolist(), l2.tolist())
    for k in s1:
        assert torch.equal(s1[k], s2[k]), f"{k} differs between identical runs"
    torch.cuda.empty_cache()
