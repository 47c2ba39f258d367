"""uint8 level batches (the resized images before ToTensor) as model input, on the CPU plans:
ConvNet reads them as levels * fp32(1/255), exactly what the fp32 upsample produces."""
import torch

from torch_distributed_sandbox_amd.models import ConvNet
from torch_distributed_sandbox_amd.models.convnet import LEVEL_SCALE, to_image
from torch_distributed_sandbox_amd.ops import functional as TF


def test_to_image_matches_totensor_scale():
    lv = torch.arange(256, dtype=torch.uint8).view(1, 1, 16, 16)
    x = to_image(lv)
    assert x.dtype == torch.float32
    assert torch.equal(x, lv.float() * torch.tensor(LEVEL_SCALE, dtype=torch.float32))
    f = torch.rand(2, 1, 4, 4)
    assert to_image(f) is f


def test_upsample_levels_cpu():
    src = torch.randint(0, 256, (2, 28, 28), dtype=torch.uint8)
    lv = TF.upsample_bilinear_u8(src, 64, 64, levels=True)
    assert lv.dtype == torch.uint8 and lv.shape == (2, 1, 64, 64)
    assert torch.allclose(to_image(lv), TF.upsample_bilinear_u8(src, 64, 64), atol=1e-7)


def test_convnet_levels_input_equals_image_input():
    torch.manual_seed(0)
    m = ConvNet(image_shape=(32, 32))
    lv = torch.randint(0, 256, (2, 1, 32, 32), dtype=torch.uint8)
    out_l = m(lv)
    out_f = m(to_image(lv))
    assert torch.equal(out_l, out_f)


def test_layer1_backward_level_lds_layout():
    """The level layer-1 backward's LDS image (tools/micro/l1b_lds_check.py): every B-operand read
    returns its packed pair and no lane half hits two addresses in one bank; the default word layout
    (stride 137, ones block) likewise returns every tap word / the sum-dz 1.0 conflict-free."""
    import importlib.util
    import os

    path = os.path.join(os.path.dirname(__file__), "..", "tools", "micro", "l1b_lds_check.py")
    spec = importlib.util.spec_from_file_location("l1b_lds_check", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.main()
    assert mod.word_layout()


def test_upsample_levels_moments_cpu_is_plain_upsample():
    """On CPU the fused input op is the plain level upsample without partials."""
    src = torch.randint(0, 256, (2, 28, 28), dtype=torch.uint8)
    x, part = TF.upsample_levels_moments(src, 64, 64)
    assert part is None and torch.equal(x, TF.upsample_bilinear_u8(src, 64, 64, levels=True))
