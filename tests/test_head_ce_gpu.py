"""The cross-entropy loss formed by the fused head forward's finalizing workgroup (labels attached to
the batch, models/convnet_fused.py attach_labels; csrc/kernels/ce_small.h shared with the CE
kernel): the loss and every gradient are bit-identical to the separate CE launch, and any use the
head did not prepare for (other labels, label smoothing, labels changed in place) takes the
separate launch."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _models(gpu, H=64):
    from torch_distributed_sandbox_amd.models import ConvNet

    torch.manual_seed(0)
    m1 = ConvNet(image_shape=(H, H), device=gpu, mode="fused")
    m2 = ConvNet(image_shape=(H, H), device=gpu, mode="fused")
    m2.load_state_dict(m1.state_dict())
    return m1, m2


@pytest.mark.parametrize("labels", [[1, 4, 7], [1, -100, 7]])
def test_loss_in_head_matches_separate_ce(gpu, labels):
    from torch_distributed_sandbox_amd.models import convnet_fused
    from torch_distributed_sandbox_amd.ops import CrossEntropyLoss

    m1, m2 = _models(gpu)
    x = torch.rand(3, 1, 64, 64, device=gpu)
    y = torch.tensor(labels, device=gpu)
    crit = CrossEntropyLoss()
    l1 = crit(m1(x), y)
    x2 = x.clone()
    convnet_fused.attach_labels(x2, y)
    before = convnet_fused.STATS["head_fused_ce"]
    out2 = m2(x2)
    assert convnet_fused.STATS["head_fused_ce"] == before + 1
    assert getattr(out2, "_tds_ce", None) is not None
    l2 = crit(out2, y)
    assert out2._tds_ce is None  # taken
    assert torch.equal(l1, l2)
    l1.backward()
    l2.backward()
    for p1, p2 in zip(m1.parameters(), m2.parameters()):
        assert torch.equal(p1.grad, p2.grad)


def test_loss_in_head_falls_back(gpu):
    from torch_distributed_sandbox_amd.models import convnet_fused
    from torch_distributed_sandbox_amd.ops import CrossEntropyLoss

    m1, m2 = _models(gpu)
    x = torch.rand(3, 1, 64, 64, device=gpu)
    y = torch.tensor([2, 3, 5], device=gpu)
    # label smoothing: the head's loss is not that loss
    x2 = x.clone()
    convnet_fused.attach_labels(x2, y)
    ref = torch.nn.functional.cross_entropy(m1(x), y, label_smoothing=0.1)
    got = CrossEntropyLoss(label_smoothing=0.1)(m2(x2), y)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)
    # other labels than the attached ones, and the attached ones changed in place
    y_other = torch.tensor([9, 0, 1], device=gpu)
    x3 = x.clone()
    convnet_fused.attach_labels(x3, y)
    got = CrossEntropyLoss()(m2(x3), y_other)
    torch.testing.assert_close(got, torch.nn.functional.cross_entropy(m1(x), y_other), rtol=1e-5, atol=1e-6)
    y4 = y.clone()
    x4 = x.clone()
    convnet_fused.attach_labels(x4, y4)
    out = m2(x4)
    y4[0] = 8
    got = CrossEntropyLoss()(out, y4)
    torch.testing.assert_close(got, torch.nn.functional.cross_entropy(m1(x), y4), rtol=1e-5, atol=1e-6)
