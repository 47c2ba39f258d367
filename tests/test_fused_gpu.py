"""Numerics of the fused ConvNet plan (NHWC; conv1 bf16x3, conv2 TF32-class fp16 or fp16x2 by build;
pooled-blocked ya/g2m) vs fp64 PyTorch references of the same ops."""
import pytest
import torch
import torch.nn.functional as F

from _tf32ref import rel, tf32, unfold_conv

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


def _check_conv(a, ref, ref_tf32, name, k=1.5):
    """A conv2 result vs fp64 (csrc/kernels/conv2_common.h: one fp16 MFMA per product, both
    operands rounded to TF32's 11 significant bits): within k = 1.5x the error the same convolution
    with TF32-rounded operands makes (tests/_tf32ref.py), or 1e-5 when that is smaller."""
    e, s = _err(a, ref)
    et, _ = _err(ref_tf32, ref)
    assert e <= max(1e-5 * s, k * et) + 1e-12, f"{name}: max err {e:.3e} vs TF32 convs {et:.3e} (scale {s:.3e})"


def new_mag(gpu, B, P):
    """The step's magnitude-bound workspace (fused_ops.cpp: [0,32) max |y2 - b2| per channel, [32]
    max |g2m|, then the per-workgroup parts), filled with garbage."""
    return torch.full((_ops().mag_numel(B, P),), -1, dtype=torch.int32, device=gpu)


def ypart(mag):
    """The conv2 forward's per-workgroup max |y2 - b2| [32][nwg] (float bits) inside the workspace."""
    n = _ops().mag_ypart_count()
    return mag[64:64 + 32 * n].view(32, n)


def mag_floats(mag):
    return mag.view(torch.float32)


def y2h_decode_factor(mag):
    """y2 = y2h * d + b2 (kernels/conv2_common.h): d = inv / 2^k from the pack's scales."""
    m = mag_floats(mag)
    return (m[40] * m[41] / m[42]).item()


def _windows(t, Q):
    """[B, 2Q.., 2Q.., 32] -> [B, Q, Q, 32, 4] in the pooling scan order q = 2*dr + dc."""
    B = t.shape[0]
    return t[:, :2 * Q, :2 * Q].reshape(B, Q, 2, Q, 2, 32).permute(0, 1, 3, 5, 2, 4).reshape(B, Q, Q, 32, 4)


def _unwindows(w, out):
    B, Q = w.shape[0], w.shape[1]
    out[:, :2 * Q, :2 * Q] = w.reshape(B, Q, Q, 32, 2, 2).permute(0, 1, 4, 2, 5, 3).reshape(B, 2 * Q, 2 * Q, 32)
    return out


def first_extreme(w, neg):
    """index (0..3) of each window's first max (first min where neg) -- torch's max-pool choice."""
    key = torch.where(neg.view(1, 1, 1, 32, 1), -w, w)
    return (key == key.max(-1, keepdim=True).values).int().argmax(-1)


def _bits_to_half(b):
    """int32 fp16 bit patterns (0..65535) -> float16"""
    return (b - (b > 32767).int() * 65536).short().view(torch.half)


def y2h_encode(y2, b2, g2, mag):
    """The forward's y2h (kernels/conv2_common.h) of a synthetic fp32 y2 [B,P,P,32]: fp16(acc * 2^k)
    to nearest, acc = (y2 - b2) / inv, and an a2: each window's first extreme (max, or min where
    gamma2 < 0) of the stored values -- the pixel max_pool2d picks on the decoded y2 the references
    see.  Returns (y2h, a2, the decoded fp32 y2 the kernels see)."""
    m = mag_floats(mag)
    inv, ksc = (m[40] * m[41]).item(), m[42].item()
    acc = (y2 - b2) / inv
    h = (acc * ksc).half()
    Q = y2.shape[1] // 2
    a2 = a2_encode(first_extreme(_windows(h.float(), Q), g2 < 0))
    return h, a2, h.float() * (inv / ksc) + b2


def a2_encode(codes):
    """argmax codes [B,Q,Q,32] (0..3) -> a2 [B,Q,Q,2] int32 (kernels/conv2_common.h): word h, bit c =
    code bit 0 and bit 16 + c = code bit 1 of channel 16h + c"""
    c = codes.long().view(*codes.shape[:3], 2, 16)
    sh = torch.arange(16, device=codes.device)
    w = (((c & 1) << sh) | (((c >> 1) & 1) << (sh + 16))).sum(-1)
    return (w - (w >= 2 ** 31).long() * 2 ** 32).int()


def a2_decode(a2):
    """a2 [B,Q,Q,2] int32 -> codes [B,Q,Q,32]"""
    w = a2.long() & 0xFFFFFFFF
    sh = torch.arange(16, device=a2.device)
    c = ((w.unsqueeze(-1) >> sh) & 1) | (((w.unsqueeze(-1) >> (sh + 16)) & 1) << 1)
    return c.reshape(*a2.shape[:3], 32)


def dp1h_decode(dp1h, dec, P):
    """dp1h [B,P,ceil(P/4),16,4] fp16 (kernels/conv2_common.h) * dec -> dp1 [B,P,P,16] fp32"""
    B = dp1h.shape[0]
    return dp1h.float().permute(0, 1, 2, 4, 3).reshape(B, P, -1, 16)[:, :, :P] * dec


def dp1h_encode(dp1, dec):
    """fp32 dp1 [B,P,P,16] -> (dp1h at 1/dec, the decode as the int32 device view the op takes,
    the decoded fp32 dp1 the kernel sees)"""
    B, P = dp1.shape[:2]
    PG = (P + 3) // 4
    pad = torch.zeros(B, P, PG * 4, 16, device=dp1.device)
    pad[:, :, :P] = dp1 / dec
    h = pad.view(B, P, PG, 4, 16).permute(0, 1, 2, 4, 3).contiguous().half()
    d = torch.tensor([dec], dtype=torch.float32, device=dp1.device).view(torch.int32)
    return h, d, dp1h_decode(h, dec, P)


def pb_dims(Q):
    return (Q + 3) // 4, (Q + 7) // 8


def pb_to_planar(t, Q):
    """[B, 32, Q4*Q8*32] pooled-blocked (csrc/kernels/pooled_layout.h) -> [B, 32, Q, Q]."""
    B = t.shape[0]
    Q4, Q8 = pb_dims(Q)
    v = t.reshape(B, 32, Q4, Q8, 4, 8).permute(0, 1, 2, 4, 3, 5).reshape(B, 32, Q4 * 4, Q8 * 8)
    return v[:, :, :Q, :Q]


def planar_to_pb(x):
    B, C, Q, _ = x.shape
    Q4, Q8 = pb_dims(Q)
    pad = torch.zeros(B, C, Q4 * 4, Q8 * 8, dtype=x.dtype, device=x.device)
    pad[:, :, :Q, :Q] = x
    return pad.reshape(B, C, Q4, 4, Q8, 8).permute(0, 1, 2, 4, 3, 5).reshape(B, C, Q4 * Q8 * 32).contiguous()


def window_extreme(y2_nchw, neg):
    """per 2x2 window: max (neg False) or min (neg True) per channel; [B,32,Q,Q]"""
    mx = F.max_pool2d(y2_nchw, 2, 2)
    mn = -F.max_pool2d(-y2_nchw, 2, 2)
    return torch.where(neg.view(1, -1, 1, 1), mn, mx)


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
    p1, idx1, stats, gram, _ = _ops().fused_l1_forward(x, w1, b1, g1, be1, rm, rv, nbt, 0.1, 1e-5)
    xd = x.double().cpu()
    y = F.conv2d(xd, w1.double().cpu(), b1.double().cpu(), padding=2)
    rmr, rvr = torch.zeros(16, dtype=torch.float64), torch.ones(16, dtype=torch.float64)
    z = F.batch_norm(y, rmr, rvr, g1.double().cpu(), be1.double().cpu(), True, 0.1, 1e-5)
    ref, ridx = F.max_pool2d(F.relu(z), 2, 2, return_indices=True)
    assert p1.dtype == torch.float16 and p1.shape == (B, H // 2, H // 2, 16)
    got = p1.float().permute(0, 3, 1, 2)
    # p1 is conv2's single-rounded fp16 operand: <= 2^-11 relative representation error
    _check(got, ref, 5e-4, "p1")
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


def test_layer1_precomputed_input_stats(gpu):
    """fused_l1_forward with the x moments computed beforehand on another stream (the input
    pipeline hand-off) is bit-identical to computing them inline."""
    torch.manual_seed(1)
    B, H = 2, 132
    x = torch.rand(B, 1, H, H, device=gpu)
    w1 = torch.randn(16, 1, 5, 5, device=gpu) * 0.2
    b1 = torch.randn(16, device=gpu) * 0.1
    g1 = torch.rand(16, device=gpu) + 0.5
    be1 = torch.randn(16, device=gpu) * 0.1

    def run(asum=None, strips=None):
        rm, rv = torch.zeros(16, device=gpu), torch.ones(16, device=gpu)
        nbt = torch.zeros((), dtype=torch.long, device=gpu)
        out = _ops().fused_l1_forward(x, w1, b1, g1, be1, rm, rv, nbt, 0.1, 1e-5, asum, strips)
        return list(out) + [rm, rv]

    side = torch.cuda.Stream(gpu)
    side.wait_stream(torch.cuda.current_stream(gpu))
    with torch.cuda.stream(side):
        asum, strips = _ops().l1_input_stats(x)
    torch.cuda.current_stream(gpu).wait_stream(side)
    for a, b in zip(run(), run(asum, strips)):
        assert torch.equal(a, b)
    with pytest.raises(RuntimeError):
        _ops().fused_l1_forward(x, w1, b1, g1, be1, None, None, None, 0.1, 1e-5, asum[:41].contiguous(), strips)


def test_model_uses_attached_input_stats(gpu):
    """ConvNet(fused) consumes stats attached by the input pipeline; an in-place change of the
    batch invalidates them."""
    from torch_distributed_sandbox_amd.models import ConvNet, convnet_fused

    torch.manual_seed(0)
    H = 64
    x = torch.rand(2, 1, H, H, device=gpu)
    m1 = ConvNet(image_shape=(H, H), device=gpu, mode="fused")
    m2 = ConvNet(image_shape=(H, H), device=gpu, mode="fused")
    m2.load_state_dict(m1.state_dict())
    ref = m1(x)
    x2 = x.clone()
    convnet_fused.attach_input_stats(x2, convnet_fused.input_stats(x2))
    assert convnet_fused._take_input_stats(x2)[0] is not None
    assert torch.equal(m2(x2), ref)
    x2.mul_(2.0)
    assert convnet_fused._take_input_stats(x2) == (None, None)


@pytest.mark.parametrize("P", [40, 38, 37])
def test_conv2_forward(gpu, P):
    """y2, the BN2 partial sums, and ya = window max / min of y2 by the sign of gamma2
    (pooled-blocked), vs fp64; P = 38 gives an odd pooled size, P = 37 an unpooled last row."""
    torch.manual_seed(P)
    B = 2
    p = torch.relu(torch.randn(B, P, P, 16, device=gpu)).half()  # the fp16 operand as layer 1 stores it
    w2 = torch.randn(32, 16, 5, 5, device=gpu) * 0.05
    b2 = torch.randn(32, device=gpu)
    g2 = torch.randn(32, device=gpu)  # mixed signs: max and min windows
    mag = new_mag(gpu, B, P)
    wp, wd = _ops().conv2_pack(w2, mag)
    y2h, partial, ya, a2 = _ops().fused_conv2_forward(p, wp, b2, g2, mag)
    assert y2h.dtype == torch.float16 and y2h.shape == (B, P, P, 32)
    v = y2h.float() * y2h_decode_factor(mag)  # y2 - b2 as stored (fp16 grid: 2^-11 relative)
    y2 = v + b2
    ref = F.conv2d(p.permute(0, 3, 1, 2).double().cpu(), w2.double().cpu(), b2.double().cpu(), padding=2)
    reft = F.conv2d(p.permute(0, 3, 1, 2).double().cpu(), tf32(w2.cpu()), b2.double().cpu(), padding=2)
    # TF32 class: the weights rounded once, as TF32 rounds them, plus the y2h storage rounding
    # (<= half an fp16 step of |y2 - b2|)
    vmax = v.abs().max().item()
    e, sc = _err(y2.permute(0, 3, 1, 2), reft)
    assert e <= 2.0 ** -10 * vmax + 1e-5 * sc, (e, vmax)
    # the stored values come from the same products as the statistics: check those against the
    # references as before (TF32-rounded operands or exact)
    # max |y2 - b2| per channel: the workgroups' maxima (plain stores) reduce to the largest fp32
    # value, within the storage rounding of the decoded values
    ymax = ypart(mag).amax(1).view(torch.float32)
    assert ((ymax - v.abs().amax((0, 1, 2))).abs() <= 2.0 ** -10 * vmax).all()
    # BN2 partials: sum over workgroups of (sum, sumsq) of y2 - b2
    s = partial.view(32, -1, 2).sum(1).cpu()
    yc = ref - b2.double().cpu().view(1, 32, 1, 1)
    yct = reft - b2.double().cpu().view(1, 32, 1, 1)
    _check_conv(s[:, 0], yc.sum((0, 2, 3)), yct.sum((0, 2, 3)), "sum")
    _check_conv(s[:, 1], (yc * yc).sum((0, 2, 3)), (yct * yct).sum((0, 2, 3)), "sumsq")
    # ya: y2h at each window's extreme (fp16, decoded as y2h); rounding is monotone, so that is
    # exactly the extreme of the window's stored values. a2: each window's argmax pixel (first in
    # scan order)
    Q = P // 2
    assert ya.dtype == torch.float16
    want = window_extreme(y2h.float().permute(0, 3, 1, 2)[:, :, :2 * Q, :2 * Q], (g2 < 0))
    got = pb_to_planar(ya, Q).float()
    assert torch.equal(got, want), (got - want).abs().max()
    _check_argmax_kept(a2, reft, g2, Q)


def _check_argmax_kept(a2, ref_nchw, g2, Q, gap=1e-5):
    """The forward's stored argmax codes (a2) name the reference's first extreme of every window
    wherever the reference's top two values of the window differ by more than fp32 accumulation
    noise."""
    assert a2.dtype == torch.int32 and a2.shape == (ref_nchw.shape[0], Q, Q, 2)
    r = _windows(ref_nchw.permute(0, 2, 3, 1).to(a2.device), Q)
    neg = g2 < 0
    key = torch.where(neg.view(1, 1, 1, 32, 1), -r, r)
    top2 = key.topk(2, -1).values
    clear = (top2[..., 0] - top2[..., 1]) > gap * r.abs().max()
    got = a2_decode(a2)
    want = first_extreme(r, neg)
    assert clear.float().mean().item() > 0.5
    bad = (got != want) & clear
    assert not bad.any(), f"{int(bad.sum())} of {int(clear.sum())} windows lost their argmax"


@pytest.mark.parametrize("P", [40, 37])
def test_conv2_forward_argmax_codes_on_near_ties(gpu, P):
    """Inputs on a 2^-10 grid make neighbouring outputs differ by about one fp16 step of y2h:
    rounding to nearest merges many windows' top two values in y2h; the argmax codes (a2) come
    from the fp32 accumulators (kernels/conv2_common.h), so they still name the reference's."""
    torch.manual_seed(100 + P)
    B = 2
    p = (1.0 + torch.randint(0, 4, (B, P, P, 16), device=gpu).float() * 2.0 ** -10).half()
    w2 = torch.randn(32, 16, 5, 5, device=gpu) * 0.05
    b2 = torch.randn(32, device=gpu)
    g2 = torch.randn(32, device=gpu)
    mag = new_mag(gpu, B, P)
    wp, _ = _ops().conv2_pack(w2, mag)
    y2h, _, _, a2 = _ops().fused_conv2_forward(p, wp, b2, g2, mag)
    pin = p.permute(0, 3, 1, 2).double().cpu()
    ref = F.conv2d(pin, tf32(w2.cpu()), None, padding=2)
    Q = P // 2
    # the case is real: to nearest, many windows' top two values share one fp16
    r = _windows(ref.permute(0, 2, 3, 1), Q)
    key = torch.where((g2.cpu() < 0).view(1, 1, 1, 32, 1), -r, r)
    top2 = key.topk(2, -1).values * y2h_decode_factor(mag) ** -1
    merged = (top2[..., 0].float().half() == top2[..., 1].float().half()) & (top2[..., 0] > top2[..., 1])
    assert merged.float().mean().item() > 0.01
    _check_argmax_kept(a2, ref, g2, Q)


def set_ya_scale(mag, d=1.0):
    """ya's decode factor d = mag[40] * mag[41] / mag[42] (kernels/launchers.h TdsYaDec) in a
    workspace no conv2 pack wrote"""
    mag_floats(mag)[40:43] = torch.tensor([d, 1.0, 1.0])
    return mag


def ya_of(h, g2, Q):
    """ya (fp16, pooled-blocked) of stored values h [B,P,P,32] (y2 = h d + b2): each window's extreme"""
    return planar_to_pb(window_extreme(h.float().permute(0, 3, 1, 2)[:, :, :2 * Q, :2 * Q], g2 < 0)).half()


def _head_case(gpu, P, B, seed):
    """A synthetic conv2 output y2 on ya's fp16 grid (decode d = 1: y2 = h + b2, h fp16), so the
    fp64 references see the values the head kernels decode."""
    torch.manual_seed(seed)
    NC = 10
    Q = P // 2
    b2 = torch.randn(32, device=gpu) * 0.1
    h = torch.randn(B, P, P, 32, device=gpu).half()
    y2 = h.float() + b2
    g2 = torch.randn(32, device=gpu)  # negative gammas exercise the min windows
    be2 = torch.randn(32, device=gpu) * 0.1
    wfc = torch.randn(NC, 32 * Q * Q, device=gpu) * 0.01
    bfc = torch.randn(NC, device=gpu)
    yc = (y2 - b2).double()
    partial2 = torch.stack([yc.sum((0, 1, 2)), (yc * yc).sum((0, 1, 2))], dim=1).contiguous()  # [32][1][2]
    ya = ya_of(h, g2, Q)
    return y2, b2, g2, be2, wfc, bfc, partial2, ya


@pytest.mark.parametrize("P,B", [(64, 3), (200, 5), (38, 2), (130, 11)])
def test_head_forward_backward(gpu, P, B):
    """BN2(batch stats) + ReLU + pool + fc forward/backward over ya vs fp64 autograd: logits,
    dW, dgamma2, dbeta2, g2m (the ReLU-masked pooled gradient, pooled-blocked) and the fused SGD
    step.  P = 38: odd pooled size (rows 1, 3, ... start off the 16-B grid); B = 11: two image
    passes."""
    y2, b2, g2, be2, wfc, bfc, partial2, ya = _head_case(gpu, P, B, P + B)
    Q, NC = P // 2, wfc.shape[0]
    ops = _ops()
    xo = torch.empty(B, 32 * Q * Q, device=gpu)
    logits, stats2, aff2 = ops.fused_head_forward(ya, partial2, b2, g2, be2, None, None, None, 0.1, 1e-5, wfc, bfc, P,
                                                  xo)
    yr = y2.permute(0, 3, 1, 2).double().cpu().requires_grad_(True)
    gr = g2.double().cpu().requires_grad_(True)
    ber = be2.double().cpu().requires_grad_(True)
    wr = wfc.double().cpu().requires_grad_(True)
    z = F.batch_norm(yr, None, None, gr, ber, True, 0.1, 1e-5)
    pz = F.max_pool2d(F.relu(z), 2, 2)
    pz.retain_grad()
    ref = F.linear(pz.reshape(B, -1), wr, bfc.double().cpu())
    _check(logits, ref, 1e-5, "logits")
    _check(xo.view(B, 32, Q, Q), pz, 1e-5, "x_out (fc input rows)")
    dl = torch.randn(B, NC, device=gpu)
    ref.backward(dl.double().cpu())
    mag = set_ya_scale(new_mag(gpu, B, P))
    ypart(mag).zero_()
    ypart(mag)[5, 3] = torch.tensor(2.5).view(torch.int32)  # a forward part: reduced per channel
    dW, dbfc, dg2, dbe2, g2m, kbuf = ops.fused_head_backward(dl, ya, stats2, aff2, b2, g2, wfc, P, None, 1.0, True,
                                                             mag=mag)
    # g2m: fp16 at a power-of-two scale per channel (kbuf[96 + c] = 2^-e_c), bounded by the forward's
    # max |W| per channel and class: below 2^14 by construction, 11 significant bits
    assert g2m.shape == (B, 32, Q, Q) and g2m.dtype == torch.float16 and kbuf.shape == (128,)
    ginv = kbuf[96:]
    assert torch.equal(torch.frexp(ginv).mantissa, torch.full_like(ginv, 0.5))  # powers of two
    assert g2m.float().abs().max().item() < 2.0 ** 14
    g2f = g2m.float() * ginv.view(1, 32, 1, 1)
    gm32 = mag_floats(mag)[32].item()  # max |g2m| before rounding: the conv2 backward's bound
    assert abs(gm32 - g2f.abs().max().item()) <= 2.0 ** -11 * gm32
    want = torch.zeros(32, device=gpu)
    want[5] = 2.5
    assert torch.equal(mag_floats(mag)[:32], want)  # max |y2 - b2| per channel from the forward parts
    _check(dW, wr.grad, 1e-5, "dW")
    _check(dbfc, dl.double().sum(0), 1e-6, "dbfc")
    _check(dg2, gr.grad, 1e-5, "dgamma2")
    _check(dbe2, ber.grad, 1e-5, "dbeta2")
    mask = (pz > 0).double()
    _check(g2f, pz.grad * mask, 2.0 ** -11 + 1e-5, "g2m (fp16, 2^-11 relative)")
    # no-dW form (activation exchange) leaves the same g2m / BN2 gradients
    _, _, dg2b, dbe2b, g2mb, kbufb = ops.fused_head_backward(dl, ya, stats2, aff2, b2, g2, wfc, P, None, 1.0, False)
    assert torch.equal(g2mb, g2m) and torch.equal(kbufb, kbuf) and torch.equal(dg2b, dg2)
    if B <= 8:
        # SGD step fused into the backward: W <- W - lr dW (in place), dW still written
        w0 = wfc.clone()
        dW2 = torch.empty_like(wfc)
        ops.fused_head_backward(dl, ya, stats2, aff2, b2, g2, wfc, P, dW2, 1.0, True, 0.5)
        assert torch.equal(dW2, dW)
        assert torch.allclose(wfc, w0 - 0.5 * dW, rtol=0, atol=1e-6)


@pytest.mark.parametrize("P,B,W", [(64, 3, 2), (38, 5, 1), (130, 2, 3)])
def test_head_update_pooled(gpu, P, B, W):
    """The pooled activation exchange's fc step (ops.head_update_pooled, parallel/factored.py "pooled")
    from W ranks' ya and head records (each rank its own BN2 affine): the X it recomputes is bit for
    bit the head forward's own X rows (x_out), and W -= lr*scale*dl^T X, dW = / += scale*dl^T X match
    fp64 on those rows.  P = 38: odd pooled size (rows off the 16-B grid)."""
    ops = _ops()
    Q, NC = P // 2, 10
    torch.manual_seed(P + 10 * B + W)
    wfc = torch.randn(NC, 32 * Q * Q, device=gpu) * 0.01
    bfc = torch.randn(NC, device=gpu)
    b2 = torch.randn(32, device=gpu) * 0.1
    mag = set_ya_scale(new_mag(gpu, B, P), 0.5)  # ya decode d = 0.5
    yas, recs, xs = [], [], []
    for _ in range(W):
        h = torch.randn(B, P, P, 32, device=gpu).half()
        ya = ya_of(h, torch.randn(32, device=gpu), Q)
        aff2 = torch.cat([torch.randn(32, device=gpu), torch.randn(32, device=gpu) * 0.1])
        xo = torch.empty(B, 32 * Q * Q, device=gpu)
        ops.fused_head_forward_aff(ya, aff2, b2, mag, wfc, bfc, P, xo)
        yas.append(ya)
        recs.append(ops.head_pooled_record(aff2, b2, mag))
        xs.append(xo)
    ya_all, rec_all, x_all = torch.stack(yas), torch.stack(recs), torch.cat(xs)
    M = W * B
    # one-hot dl, scale 1: row j of the result is rank / image j's X itself (exact products and sums)
    eye = torch.zeros(M, NC, device=gpu)
    eye[torch.arange(M), torch.arange(M)] = 1.0
    out = torch.full_like(wfc, 7.0)
    ops.head_update_pooled(eye, ya_all, rec_all, wfc, out, P, 1.0, 0.0, 1)
    assert torch.equal(out[:M], x_all), (out[:M] - x_all).abs().max()
    assert (out[M:] == 0).all()
    dl = torch.randn(M, NC, device=gpu)
    scale, lr = 1.0 / W, 0.25
    ref = (dl.double().t() @ x_all.double()) * scale
    ops.head_update_pooled(dl, ya_all, rec_all, wfc, out, P, scale, 0.0, 1)
    _check(out, ref, 1e-6, "dW (=)")
    ops.head_update_pooled(dl, ya_all, rec_all, wfc, out, P, scale, 0.0, 2)
    _check(out, 2 * ref, 1e-6, "dW (+=)")
    w0 = wfc.double()
    ops.head_update_pooled(dl, ya_all, rec_all, wfc, None, P, scale, lr, 0)
    _check(wfc, w0 - lr * ref, 1e-6, "W update")


@pytest.mark.parametrize("P,dscale", [(37, 1.0), (40, 1.0), (130, 1.0), (40, 1e-7), (40, 3e4)])
def test_conv2_backward_fused_with_bn2_pool(gpu, P, dscale):
    """fused_conv2_backward_y2 (dy2 rebuilt in LDS from y2 + g2m + the BN2 constants) vs the fp64
    chain BN2 -> ReLU -> pool -> fc backward -> conv2 data and weight gradients.  dscale moves
    the gradient by orders of magnitude: dy2 travels in fp16 with a per-step power-of-two
    scale from the magnitude bounds, so the relative accuracy must not depend on it (unscaled,
    1e-7-sized gradients would be fp16 subnormals)."""
    B = 2
    y2, b2, g2, be2, wfc, bfc, _, _ = _head_case(gpu, P, B, 7 * P)
    ops = _ops()
    dl = torch.randn(B, wfc.shape[0], device=gpu) * dscale
    p = torch.relu(torch.randn(B, P, P, 16, device=gpu)).half()
    w2 = torch.randn(32, 16, 5, 5, device=gpu) * 0.05
    mag = new_mag(gpu, B, P)
    _, wd = ops.conv2_pack(w2, mag)
    # the forward's y2h of the synthetic y2; everything below (head, references) sees its decode
    y2h, a2, y2 = y2h_encode(y2, b2, g2, mag)
    Q = P // 2
    yc = (y2 - b2).double()
    partial2 = torch.stack([yc.sum((0, 1, 2)), (yc * yc).sum((0, 1, 2))], dim=1).contiguous()
    ya = ya_of(y2h, g2, Q)
    _, stats2, aff2 = ops.fused_head_forward(ya, partial2, b2, g2, be2, None, None, None, 0.1, 1e-5, wfc, bfc, P,
                                             mag=mag)
    yp = ypart(mag)  # (the conv2 forward's per-workgroup bounds; y2 is synthetic here)
    yp.zero_()
    yp[:, 0] = (y2 - b2).abs().amax((0, 1, 2)).view(torch.int32)  # max |y2 - b2| per channel
    _, _, _, _, g2m, kbuf = ops.fused_head_backward(dl, ya, stats2, aff2, b2, g2, wfc, P, None, 1.0, True, mag=mag)
    dp1h, dw2, db2 = ops.fused_conv2_backward_y2(y2h, a2, g2m, aff2, kbuf, b2, mag, p, wd, 1.0)
    dp1 = dp1h_decode(dp1h, mag_floats(mag)[44].item(), P)
    # fp64 reference: dy2 from the head chain, then the conv2 backward with that dy2
    yr = y2.permute(0, 3, 1, 2).double().cpu().requires_grad_(True)
    z = F.batch_norm(yr, None, None, g2.double().cpu(), be2.double().cpu(), True, 0.1, 1e-5)
    pz = F.max_pool2d(F.relu(z), 2, 2)
    F.linear(pz.reshape(B, -1), wfc.double().cpu(), bfc.double().cpu()).backward(dl.double().cpu())
    dy2 = yr.grad
    pr = p.permute(0, 3, 1, 2).double().cpu().requires_grad_(True)
    wr = w2.double().cpu().requires_grad_(True)
    br = torch.zeros(32, dtype=torch.float64, requires_grad=True)
    F.conv2d(pr, wr, br, padding=2).backward(dy2)
    # the same convolution backward with TF32 operands (dy2 and w2 rounded; p1 is fp16 already)
    prt = p.permute(0, 3, 1, 2).double().cpu().requires_grad_(True)
    wrt = tf32(w2.cpu()).requires_grad_(True)
    F.conv2d(prt, wrt, None, padding=2).backward(tf32(dy2))
    # dgrad: dy2 is the single-rounded fp16 operand (2^-11 per element) built from the pooled
    # gradient g2m as stored in fp16 (one more 2^-11 rounding where it enters: up to 2x the TF32
    # operand error), w2 rounded, and the result is stored once as dp1h (fp16: <= 2^-11 more)
    e, sc = _err(dp1.permute(0, 3, 1, 2), pr.grad)
    et, _ = _err(prt.grad, pr.grad)
    bound = max(1e-5 * sc, 2.5 * et) + 2.0 ** -11 * sc
    assert e <= bound, f"dp1: max err {e:.3e} vs bound {bound:.3e} (scale {sc:.3e})"
    # wgrad: dy2 rounded (after g2m's fp16 storage), p1 the stored fp16 operand itself
    _check_conv(dw2, wr.grad, wrt.grad, "dw2", k=2.5)
    # conv bias before BN: sum(dy2) is analytically zero, both sides are rounding noise; with dy2
    # rounded once to 11 significant bits (TF32 class) the noise is bounded by 2^-11 sum|dy2|
    err = (db2.double().cpu() - br.grad).abs()
    # (k2, k3 come from the sums over the stored fp16 g2m: sum dy2 stays 0 before dy2's own rounding)
    bound = dy2.abs().sum((0, 2, 3)) * 2.0 ** -11 * 1.01 + 1e-4 * wr.grad.abs().max().item()
    assert bool((err <= bound).all()), (err.max().item(), bound.min().item())


def _fused_vs_ref(gpu, B, H, steps=2, lr=0.05, levels=False, gamma1=None, w2_scale=None, p1_above=None, g2_zero=()):
    import torch.nn as nn

    from torch_distributed_sandbox_amd.models import ConvNet, fc_in_features
    from torch_distributed_sandbox_amd.models.convnet import to_image
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
    with torch.no_grad():
        ours.layer2[1].weight[::3].neg_()  # some negative BN2 gammas: min-pooled windows
        if gamma1 is not None:  # BN1 output (= p1, conv2's fp16 operand) scaled up
            ours.layer1[1].weight.fill_(gamma1)
        if w2_scale is not None:  # conv2 weights scaled down (the exactly carried fp16 operand)
            ours.layer2[0].weight.mul_(w2_scale)
        for c in g2_zero:  # BN2 gamma 0 with beta > 0: every window ties, torch pools its first position
            ours.layer2[1].weight[c] = 0.0
            ours.layer2[1].bias[c] = 0.25 + 0.1 * c
    ref = Ref(fc_in_features((H, H))).double()
    ref.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in ours.state_dict().items()})
    # the reference's precision class: its convolutions with TF32 operands (tests/_tf32ref.py)
    # (its own trajectory, like ours: both are compared with the fp64 one step by step)
    reft = Ref(fc_in_features((H, H))).double()
    reft.load_state_dict(ref.state_dict())
    for layer in (reft.layer1, reft.layer2):
        layer[0].forward = unfold_conv(layer[0], tf32_operands=True)
    topt = torch.optim.SGD(reft.parameters(), lr)
    ours = ours.to(gpu)
    opt = SGD(ours.parameters(), lr)
    ropt = torch.optim.SGD(ref.parameters(), lr)
    crit = CrossEntropyLoss()
    for s in range(steps):
        if levels:  # uint8 levels of resized 28x28 sources (the input pipeline's), the references get
            # the ToTensor image
            from torch_distributed_sandbox_amd.ops import functional as TF

            src = torch.randint(0, 256, (B, 28, 28), device=gpu, dtype=torch.uint8)
            xin = TF.upsample_bilinear_u8(src, H, H, levels=True)
            x = to_image(xin)
        else:
            x = xin = torch.rand(B, 1, H, H, device=gpu)
        y = torch.randint(0, 10, (B,), device=gpu)
        if p1_above is not None and s == 0:  # the case is real: fp32 p1 leaves fp16's range
            with torch.no_grad():
                import copy  # (a copy: the probe forward must not touch ref's BN running stats)

                assert copy.deepcopy(ref.layer1)(x.double().cpu()).max().item() > p1_above
        loss = crit(ours(xin), y)
        opt.zero_grad()
        loss.backward()
        topt.zero_grad()
        tl = F.cross_entropy(reft(x.double().cpu()), y.cpu())
        tl.backward()
        rl = F.cross_entropy(ref(x.double().cpu()), y.cpu())
        ropt.zero_grad()
        rl.backward()
        assert abs(loss.item() - rl.item()) <= max(2e-4 * max(1.0, abs(rl.item())), 1.5 * abs(tl.item() - rl.item())), (
            loss.item(), rl.item(), tl.item())
        rp = dict(ref.named_parameters())
        rt = dict(reft.named_parameters())
        for n, p in ours.named_parameters():
            g, rg = p.grad.double().cpu(), rp[n].grad
            if n.endswith("0.bias"):  # analytically zero (bias before BN): rounding noise both sides
                wsc = rp[n.replace("bias", "weight")].grad.abs().max().item()
                assert (g - rg).abs().max().item() <= 1e-3 * wsc + 1e-6, f"step {s} {n}"
                continue
            # relative L2 (robust to rare argmax flips on near-tied pool windows), bounded by 1e-3
            # or by what the TF32 convolutions themselves make: conv1's weight gradient comes out
            # of BN over every position, and that cancellation amplifies the per-product rounding
            # of the conv2 data gradient (<= 2^-11 here, up to 2^-10 with TF32)
            e, et = rel(g, rg), rel(rt[n].grad, rg)
            print(f"step {s} {n:18s} ours {e:.3e}  tf32 {et:.3e}")
            assert e <= max(1e-3, 1.5 * et), f"step {s} {n}: rel L2 err {e:.3e} (TF32 convs: {et:.3e})"
            if n == "layer2.1.weight" and s == 0:
                for c in g2_zero:  # dgamma2 = sum g * xhat at the pooled (first) position
                    assert abs(g[c] - rg[c]).item() <= 1e-3 * rg.abs().max().item(), (c, g[c].item(), rg[c].item())
        opt.step()
        ropt.step()
        topt.step()
    rb, tb = dict(ref.named_buffers()), dict(reft.named_buffers())
    for n, b in ours.named_buffers():
        if b.is_floating_point():
            e, sc = _err(b, rb[n])
            et, _ = _err(tb[n], rb[n])
            print(f"buffer {n:24s} ours {e:.3e}  tf32 {et:.3e}  (scale {sc:.3e})")
            assert e <= max(1e-4 * max(sc, 1.0), 1.5 * et), n
        else:
            assert int(b.item()) == int(rb[n].item()), n


def test_fused_model_matches_reference(gpu):
    _fused_vs_ref(gpu, B=3, H=64)


def test_fused_model_p1_beyond_fp16_range(gpu):
    """BN1's gamma at 3e4: the fp32 p1 passes fp16's 65504.  The layer-1 epilogue stores p1 at
    the power-of-two scale its Samuelson bound (|xhat| <= sqrt(n-1)) asks for and the conv2
    kernels take it out: forward, gradients and buffers still match the fp64 reference within
    the TF32 class, never inf / NaN."""
    # one step: at this gamma the lr-0.05 step moves conv2's weights by O(1e3) and the next step
    # is a different problem for each trajectory
    _fused_vs_ref(gpu, B=3, H=64, steps=1, gamma1=3e4, p1_above=65504.0)


def test_fused_model_zero_bn2_gamma(gpu):
    """BN2 gamma exactly 0 on two channels (beta > 0): every pooling window of those channels ties
    at beta and torch's max-pool routes to the window's first position; the conv2 forward stores
    argmax code 0 and that position's value (conv2_fwd2.hip f2_stage), so dgamma2 / dbeta2 and the
    conv2 gradients match the fp64 reference."""
    _fused_vs_ref(gpu, B=3, H=64, steps=1, g2_zero=(5, 6))


def test_fused_conv2_bias_inplace_change_raises(gpu):
    """The conv2 output is stored without its bias (y2h) and the backward rebuilds it with b2: b2 is
    saved for backward, so an in-place change between forward and backward raises."""
    from torch_distributed_sandbox_amd.models import ConvNet

    m = ConvNet(image_shape=(64, 64), device=gpu, mode="fused")
    out = m(torch.rand(2, 1, 64, 64, device=gpu))
    with torch.no_grad():
        m.layer2[0].bias.add_(1.0)
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        out.sum().backward()


def test_fused_model_tiny_conv2_weights(gpu):
    """conv2 weights ~5e-6 (below fp16's normal range 2^-14): packed at a power-of-two scale
    (conv2_pack.hip) so hi + lo stay exact; the step matches the fp64 reference within the TF32
    class."""
    _fused_vs_ref(gpu, B=3, H=64, w2_scale=1e-4)


@pytest.mark.parametrize("H", [64, 76])
def test_fused_model_levels_input_matches_reference(gpu, H):
    """uint8 level batches (ToTensor's 1/255 folded into conv1, the x moments from exact integer
    dot products) against the fp64 / TF32 references fed the fp32 image."""
    _fused_vs_ref(gpu, B=3 if H == 64 else 2, H=H, steps=2 if H == 64 else 1, levels=True)


@pytest.mark.parametrize("H", [68, 264])
def test_layer1_levels_forward_backward(gpu, H):
    """fused_l1_forward / fused_l1_backward on uint8 levels == the same ops on the fp32 image
    (x = level * fp32(1/255)): the Gram exactly as fp64 (integer moments), p1 / argmax and the
    layer-1 gradients to the bf16x3 class of the fp32-image path."""
    from torch_distributed_sandbox_amd.models.convnet import to_image

    torch.manual_seed(3)
    B = 3
    lv = torch.randint(0, 256, (B, 1, H, H), device=gpu, dtype=torch.uint8)
    lv[0, 0, :7, :9] = 255  # saturated corner blocks: the Gram's corner terms
    lv[1, 0, -6:, -6:] = 0
    x = to_image(lv)
    w1 = torch.randn(16, 1, 5, 5, device=gpu) * 0.2
    b1 = torch.randn(16, device=gpu) * 0.1
    g1 = torch.rand(16, device=gpu) + 0.5
    be1 = torch.randn(16, device=gpu) * 0.1

    def fwd(inp):
        rm, rv = torch.zeros(16, device=gpu), torch.ones(16, device=gpu)
        nbt = torch.zeros((), dtype=torch.long, device=gpu)
        return _ops().fused_l1_forward(inp, w1, b1, g1, be1, rm, rv, nbt, 0.1, 1e-5), rm, rv

    (p1l, idxl, statsl, graml, _), rml, rvl = fwd(lv)
    (p1f, idxf, statsf, gramf, _), rmf, rvf = fwd(x)
    # exact integer moments of the levels, scaled in fp64 by the fp32 constant
    sc = float(torch.tensor(1.0 / 255.0, dtype=torch.float32))
    pat = F.unfold(lv.double().cpu(), 5, padding=2)
    G = torch.einsum("bkp,bjp->kj", pat, pat) * (sc * sc)
    S = pat.sum((0, 2)) * sc
    _check(graml[:625].view(25, 25), G, 1e-13, "G (levels)")
    _check(graml[625:], S, 1e-13, "S (levels)")
    # ... and of the fp32 image within its own per-pixel rounding (2^-24)
    pat = F.unfold(x.double().cpu(), 5, padding=2)
    _check(graml[:625].view(25, 25), torch.einsum("bkp,bjp->kj", pat, pat), 1e-7, "G (image)")
    _check(statsl, statsf, 1e-5, "stats1")
    _check(rml, rmf, 1e-5, "running_mean")
    _check(rvl, rvf, 1e-5, "running_var")
    _check(p1l.float(), p1f.float(), 2e-3, "p1")
    assert (idxl == idxf).float().mean().item() > 0.999
    P = H // 2
    dp1h, dec, dp1 = dp1h_encode(torch.randn(B, P, P, 16, device=gpu), 2.0 ** -9)
    outl = _ops().fused_l1_backward(dp1h, dec, lv, p1l, idxl, w1, b1, g1, statsl, graml, 1.0)
    outf = _ops().fused_l1_backward(dp1h, dec, x, p1f, idxf, w1, b1, g1, statsf, gramf, 1.0)
    # fp64 reference: the same layer in autograd, dp1 routed by max-pool's own argmax
    prm = [t.detach().double().cpu().requires_grad_() for t in (w1, b1, g1, be1)]
    y = F.conv2d(x.double().cpu(), prm[0], prm[1], padding=2)
    z = F.batch_norm(y, None, None, prm[2], prm[3], True, 0.1, 1e-5)
    F.max_pool2d(F.relu(z), 2, 2).backward(dp1.double().cpu().permute(0, 3, 1, 2))
    for a, b, r, n in zip(outl, outf, prm, ("dw1", "db1", "dgamma1", "dbeta1")):
        if n == "db1":  # analytically ~0 (bias before BN): rounding noise on both sides
            assert (a - b).abs().max().item() <= 1e-3 * outf[0].abs().max().item() + 1e-6, n
            continue
        el, ef = rel(a.double().cpu(), r.grad.view(a.shape)), rel(b.double().cpu(), r.grad.view(b.shape))
        print(f"{n}: levels {el:.3e}  fp32 image {ef:.3e}")
        assert el <= max(1e-3, 1.5 * ef), n


def test_upsample_levels(gpu):
    """levels=True returns the rounded levels the fp32 output is made of (x = level * fp32(1/255))."""
    from torch_distributed_sandbox_amd.models.convnet import to_image
    from torch_distributed_sandbox_amd.ops import functional as TF

    src = torch.randint(0, 256, (3, 28, 28), device=gpu, dtype=torch.uint8)
    for H in (300, 302):  # 302: rows not 4-byte aligned -> the scalar tail path
        lv = TF.upsample_bilinear_u8(src, H, H, levels=True)
        assert lv.dtype == torch.uint8 and lv.shape == (3, 1, H, H)
        assert torch.equal(to_image(lv), TF.upsample_bilinear_u8(src, H, H))


def test_fused_model_matches_reference_odd_pool(gpu):
    # P = 38 (not a multiple of the 16-column conv2 tile), Q = 19 (odd: scalar fc-weight path)
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


def test_bad_launch_raises(gpu):
    """A launch the hardware refuses (dynamic LDS above 160 KiB, a 2048-thread block) surfaces
    as a Python exception from the op, and the next good launch is unaffected."""
    ops = _ops()
    like = torch.empty(1, device=gpu)
    ops.launch_probe(like, 4096, 256)
    with pytest.raises(RuntimeError, match="launch"):
        ops.launch_probe(like, 200 * 1024, 256)
    with pytest.raises(RuntimeError, match="launch"):
        ops.launch_probe(like, 0, 2048)
    ops.launch_probe(like, 1024, 64)
    torch.cuda.synchronize()
