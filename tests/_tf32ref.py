"""TF32-emulated convolutions for the numerics tests: the precision class the reference is
quoted at.  The reference's convolutions run on cuDNN with PyTorch's default
``torch.backends.cudnn.allow_tf32 = True`` on Ampere: every operand of the forward, data
gradient and weight gradient is rounded to TF32 (10 explicit mantissa bits), products are exact
and sums fp32.  gfx950 has no TF32, so the tests emulate it in fp64 (operands rounded, arithmetic
exact) and bound our kernels' errors by the error that precision class itself makes."""
import torch
import torch.nn.functional as F


def tf32(t):
    """Round to TF32 (round to nearest even on 10 explicit mantissa bits), kept in fp64."""
    b = t.float().view(torch.int32)
    b = (b + 0xFFF + ((b >> 13) & 1)) & ~0x1FFF
    return b.view(torch.float32).double()


def unfold_conv(conv, tf32_operands=False):
    """fp64 5x5 'same' convolution as unfold + GEMM (MIOpen has no fp64 convolutions), as a
    replacement ``forward`` of ``conv``; with ``tf32_operands`` every operand of the three
    convolution GEMMs is rounded to TF32 first."""

    if not tf32_operands:
        def fwd(x):
            Bx, _, Hx, Wx = x.shape
            cols = F.unfold(x, 5, padding=2)  # [B, C*25, H*W]
            y = conv.weight.reshape(conv.out_channels, -1) @ cols + conv.bias.view(1, -1, 1)
            return y.view(Bx, conv.out_channels, Hx, Wx)

        return fwd

    class _TF32Conv(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, w, b):
            xr, wr = tf32(x), tf32(w)
            ctx.save_for_backward(xr, wr)
            Bx, _, Hx, Wx = x.shape
            y = wr.reshape(wr.shape[0], -1) @ F.unfold(xr, 5, padding=2) + b.view(1, -1, 1)
            return y.view(Bx, wr.shape[0], Hx, Wx)

        @staticmethod
        def backward(ctx, dy):
            xr, wr = ctx.saved_tensors
            dyr = tf32(dy)
            Bx, C, Hx, Wx = xr.shape
            dcols = wr.reshape(wr.shape[0], -1).t() @ dyr.reshape(Bx, wr.shape[0], -1)
            dx = F.fold(dcols, (Hx, Wx), 5, padding=2)
            dw = torch.einsum("bok,bck->oc", dyr.reshape(Bx, wr.shape[0], -1), F.unfold(xr, 5, padding=2))
            return dx, dw.view_as(wr), dy.sum((0, 2, 3))

    return lambda x: _TF32Conv.apply(x, conv.weight, conv.bias)


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def tf32_convs(model):
    """Patch a reference ConvNet (layer1 / layer2 Sequentials, conv first) in place so its
    convolutions run with TF32 operands; returns the model."""
    for layer in (model.layer1, model.layer2):
        layer[0].forward = unfold_conv(layer[0], tf32_operands=True)
    return model
