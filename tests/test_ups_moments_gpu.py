"""The input op fused with the x moments (csrc/kernels/ups_moments.hip) and the border strips
formed inside the layer-1 reducer's launch (csrc/kernels/xmom_u8.h): the levels are the plain
upsample's byte for byte, the autocorrelation sums and everything layer 1 derives from them are the
separate kernels' exactly (integer sums in fp64), and the model consumes the partials."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ops():
    import torch_distributed_sandbox_amd as tds

    return tds._ext.ops()


@pytest.mark.parametrize("B,hw,H,W", [(3, 28, 300, 300), (2, 28, 131, 64), (1, 28, 1028, 1032), (5, 28, 3000, 3000),
                                      (2, 20, 97, 252)])
def test_upsample_levels_moments_matches_separate_kernels(gpu, B, hw, H, W):
    g = torch.Generator(device=gpu).manual_seed(H + W)
    src = torch.randint(0, 256, (B, hw, hw), dtype=torch.uint8, device=gpu, generator=g)
    x, part = _ops().upsample_levels_moments(src, H, W)
    ref = _ops().upsample_bilinear_u8(src, H, W, True)
    assert torch.equal(x, ref)
    assert part.numel() > 0 and part.numel() % 42 == 0
    asum = part.view(-1, 42).sum(0)
    if H == W:  # the separate kernels' sums (l1_input_stats takes square batches)
        asum_ref, _ = _ops().l1_input_stats(x)
        assert torch.equal(asum, asum_ref)
    # every lag against torch on the levels (small shapes: the sums stay exact in fp64)
    if H * W <= 1_100_000:
        xd = x.double()[:, 0]
        k = 0
        ref_sums = []
        for dy in range(5):
            for dx in range(-4, 5) if dy else range(5):
                a = xd[:, :H - dy, max(0, -dx):W - max(0, dx)]
                b = xd[:, dy:, max(0, dx):W - max(0, -dx)]
                ref_sums.append((a * b).sum())
                k += 1
        ref_sums.append(xd.sum())
        assert torch.equal(asum, torch.stack(ref_sums))


def test_upsample_levels_moments_unsupported_shape_falls_back(gpu):
    src = torch.randint(0, 256, (2, 28, 28), dtype=torch.uint8, device=gpu)
    x, part = _ops().upsample_levels_moments(src, 100, 102)  # W % 4 != 0
    assert part.numel() == 0 and torch.equal(x, _ops().upsample_bilinear_u8(src, 100, 102, True))


@pytest.mark.parametrize("B,H", [(2, 132), (3, 1028), (5, 3000)])
def test_layer1_forward_from_fused_partials(gpu, B, H):
    """fused_l1_forward on (levels, partials) -- the reducer's launch forming the border strips --
    is bit-identical to the forward that takes the separate kernels' (sums, strips), and to the
    one that forms everything itself."""
    g = torch.Generator(device=gpu).manual_seed(B * H)
    src = torch.randint(0, 256, (B, 28, 28), dtype=torch.uint8, device=gpu, generator=g)
    x, part = _ops().upsample_levels_moments(src, H, H)
    torch.manual_seed(2)
    w1 = torch.randn(16, 1, 5, 5, device=gpu) * 0.2
    b1 = torch.randn(16, device=gpu) * 0.1
    g1 = torch.rand(16, device=gpu) + 0.5
    be1 = torch.randn(16, device=gpu) * 0.1

    def run(asum=None, strips=None):
        rm, rv = torch.zeros(16, device=gpu), torch.ones(16, device=gpu)
        nbt = torch.zeros((), dtype=torch.long, device=gpu)
        out = _ops().fused_l1_forward(x, w1, b1, g1, be1, rm, rv, nbt, 0.1, 1e-5, asum, strips)
        return list(out) + [rm, rv]

    asum, strips = _ops().l1_input_stats(x)
    ref = run(asum, strips)
    for a, b in zip(run(part, None), ref):
        assert torch.equal(a, b)
    for a, b in zip(run(), ref):
        assert torch.equal(a, b)
    with pytest.raises(RuntimeError):  # partials come without strips
        _ops().fused_l1_forward(x, w1, b1, g1, be1, None, None, None, 0.1, 1e-5, part, strips)


def test_model_consumes_fused_partials(gpu):
    """ConvNet(fused) takes the partials attached by the input op: same loss and gradients as the
    batch without them, and the counter shows they were used."""
    from torch_distributed_sandbox_amd.models import ConvNet, convnet_fused
    from torch_distributed_sandbox_amd.ops import functional as TF

    torch.manual_seed(0)
    H = 128
    src = torch.randint(0, 256, (3, 28, 28), dtype=torch.uint8, device=gpu)
    y = torch.tensor([1, 4, 7], device=gpu)
    m1 = ConvNet(image_shape=(H, H), device=gpu, mode="fused")
    m2 = ConvNet(image_shape=(H, H), device=gpu, mode="fused")
    m2.load_state_dict(m1.state_dict())
    x1 = TF.upsample_bilinear_u8(src, H, H, levels=True)
    x2, part = TF.upsample_levels_moments(src, H, H)
    assert part is not None and torch.equal(x1, x2)
    convnet_fused.attach_input_stats(x2, (part, None))
    before = convnet_fused.STATS["precomputed_input_moments"]
    l1 = torch.nn.functional.cross_entropy(m1(x1), y)
    l2 = torch.nn.functional.cross_entropy(m2(x2), y)
    assert convnet_fused.STATS["precomputed_input_moments"] == before + 1
    assert torch.equal(l1, l2)
    l1.backward()
    l2.backward()
    for p1, p2 in zip(m1.parameters(), m2.parameters()):
        assert torch.equal(p1.grad, p2.grad)


def test_device_loader_attaches_partials(gpu):
    """The trainer's loader (levels, moments=True) yields the plain levels with the partials attached."""
    from torch_distributed_sandbox_amd.data.synthetic import DeviceUpsampleLoader, SyntheticMNIST
    from torch_distributed_sandbox_amd.models import convnet_fused

    ds = SyntheticMNIST(size=8)
    plain = DeviceUpsampleLoader(ds, 4, (64, 64), gpu, levels=True)
    fused = DeviceUpsampleLoader(ds, 4, (64, 64), gpu, levels=True, moments=True)
    for (xa, ya), (xb, yb) in zip(plain, fused):
        assert torch.equal(xa, xb) and torch.equal(ya, yb)
        part, strips = convnet_fused._take_input_stats(xb)
        assert strips is None and part is not None
        assert part.numel() % 42 == 0
        assert torch.equal(part.view(-1, 42).sum(0), _ops().l1_input_stats(xb)[0])
