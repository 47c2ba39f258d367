"""Autograd-aware functional ops backed by the gfx950 kernels.

Each op has a native HIP path for GPU tensors (``torch.ops.tdsa.*``) and a
reference PyTorch path for CPU tensors (tests, gloo rehearsals).  The GPU
path never falls back: a missing extension raises (see ``_ext.ops``).

Reference ops replaced (mnist_onegpu.py:14-24,48-49):
Conv2d(k=5,s=1,p=2), BatchNorm2d (train/eval), ReLU, MaxPool2d(2,2),
Linear, CrossEntropyLoss, SGD.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import _ext
from . import grad_sink


# --------------------------------------------------------------------------- ReLU
class _ReLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y = _ext.ops().relu_fwd(x.contiguous())
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, gy):
        (y,) = ctx.saved_tensors
        return _ext.ops().relu_bwd(gy.contiguous(), y)


def relu(x: torch.Tensor) -> torch.Tensor:
    if not x.is_cuda:
        return F.relu(x)
    return _ReLU.apply(x)


# --------------------------------------------------------------------------- MaxPool 2x2 / 2
class _MaxPool2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y, idx = _ext.ops().maxpool2_fwd(x.contiguous())
        ctx.save_for_backward(idx)
        ctx.hw = (x.shape[2], x.shape[3])
        ctx.mark_non_differentiable(idx)
        return y

    @staticmethod
    def backward(ctx, gy):
        (idx,) = ctx.saved_tensors
        return _ext.ops().maxpool2_bwd(gy.contiguous(), idx, ctx.hw[0], ctx.hw[1])


def max_pool2x2(x: torch.Tensor) -> torch.Tensor:
    if not x.is_cuda:
        return F.max_pool2d(x, kernel_size=2, stride=2)
    return _MaxPool2.apply(x)


# --------------------------------------------------------------------------- Conv2d (stride 1, 'same')
class _Conv2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, pad):
        x = x.contiguous()
        w = w.contiguous()
        out = _ext.ops().conv2d_fwd(x, w, b, pad)
        ctx.save_for_backward(x, w)
        ctx.pad = pad
        ctx.has_bias = b is not None
        return out

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gy = gy.contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = _ext.ops().conv2d_dgrad(gy, w, ctx.pad)
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            dw, db = _ext.ops().conv2d_wgrad(x, gy, w.shape[2], ctx.pad, ctx.has_bias)
            if not ctx.needs_input_grad[1]:
                dw = None
            if not (ctx.has_bias and ctx.needs_input_grad[2]):
                db = None
        return dx, dw, db, None


def conv2d(x, weight, bias=None, padding: int = 0):
    if not x.is_cuda:
        return F.conv2d(x, weight, bias, stride=1, padding=padding)
    return _Conv2d.apply(x, weight, bias, int(padding))


# --------------------------------------------------------------------------- BatchNorm2d
class _BatchNormTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, running_mean, running_var, num_batches, momentum, eps, fuse_relu):
        x = x.contiguous()
        y, mean, invstd = _ext.ops().bn_fwd_train(
            x, gamma, beta, running_mean, running_var, num_batches, momentum, eps, fuse_relu
        )
        ctx.fuse_relu = fuse_relu
        ctx.save_for_backward(x, gamma, mean, invstd, y if fuse_relu else None)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, gamma, mean, invstd, y = ctx.saved_tensors
        gy = gy.contiguous()
        if ctx.fuse_relu:
            gy = _ext.ops().relu_bwd(gy, y)
        dx, dgamma, dbeta = _ext.ops().bn_bwd(gy, x, gamma, mean, invstd, ctx.needs_input_grad[0])
        return (
            dx if ctx.needs_input_grad[0] else None,
            dgamma if gamma is not None and ctx.needs_input_grad[1] else None,
            dbeta if ctx.needs_input_grad[2] else None,
            None, None, None, None, None, None,
        )


def batch_norm(x, running_mean, running_var, weight=None, bias=None, training=True, momentum=0.1, eps=1e-5,
               num_batches_tracked=None, fuse_relu=False):
    """``F.batch_norm`` semantics (+ optional fused ReLU).  ``momentum=None`` ->
    cumulative moving average, as ``nn.BatchNorm2d``."""
    if not x.is_cuda:
        if training and num_batches_tracked is not None:
            num_batches_tracked.add_(1)
        eff_m = momentum
        if momentum is None and training and num_batches_tracked is not None:
            eff_m = 1.0 / float(num_batches_tracked.item())
        y = F.batch_norm(x, running_mean, running_var, weight, bias, training, eff_m if eff_m is not None else 0.0, eps)
        return F.relu(y) if fuse_relu else y
    if training:
        eff_m = momentum
        if momentum is None:
            # cumulative average needs the post-increment count on the host
            cnt = int(num_batches_tracked.item()) + 1 if num_batches_tracked is not None else 1
            eff_m = 1.0 / cnt
        return _BatchNormTrain.apply(x, weight, bias, running_mean, running_var, num_batches_tracked,
                                     float(eff_m), float(eps), bool(fuse_relu))
    y = _ext.ops().bn_fwd_eval(x.contiguous(), weight, bias, running_mean, running_var, float(eps), bool(fuse_relu))
    return y


# --------------------------------------------------------------------------- Linear (skinny split-K)
class _LinearSkinny(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        x = x.contiguous()
        w = w.contiguous()
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        ctx.w_param = w
        return _ext.ops().linear_fwd(x, w, b)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gy = gy.contiguous()
        need_dx = ctx.needs_input_grad[0]
        need_dw = ctx.needs_input_grad[1]
        need_db = ctx.has_bias and ctx.needs_input_grad[2]
        # Gradients go straight into the DDP bucket when a sink is registered
        # (no copy-in, no AccumulateGrad clone): see ops/grad_sink.py.
        dw_out = grad_sink.acquire(ctx.w_param if need_dw else None, w.shape, w)
        db_out = torch.empty(w.shape[0], device=w.device, dtype=w.dtype) if need_db else None
        dx = _ext.ops().linear_bwd_into(gy, x, w, dw_out, db_out, 1.0, False, need_dx)
        return (dx if need_dx else None, dw_out, db_out)


class _ExchangedLinear(torch.autograd.Function):
    """Linear whose weight/bias gradients come from DDP's activation exchange
    (parallel/factored.py): backward returns only dX and hands dY to the exchange."""

    @staticmethod
    def forward(ctx, x2, w, b, ex):
        ctx.save_for_backward(x2, w)
        ctx.ex = ex
        if x2.is_cuda and x2.shape[0] <= 8 and w.shape[0] <= 16:
            return _ext.ops().linear_fwd(x2, w.contiguous(), b)
        return F.linear(x2, w, b)

    @staticmethod
    def backward(ctx, gy):
        x2, w = ctx.saved_tensors
        gy = gy.contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            if gy.is_cuda and x2.shape[0] <= 8 and w.shape[0] <= 16:
                dx = _ext.ops().linear_bwd_into(gy, x2, w.contiguous(), None, None, 1.0, False, True)
            else:
                dx = gy.mm(w)
        # only now: on the GPU defer() issues the rest of the exchange on a side stream right
        # away, and under the overlapped optimizer that includes the in-place SGD step of w
        # (update-only linear_dw) -- the dX kernel above must be queued first, or the side
        # stream could update w while dX still reads it (the stream wait in defer() orders the
        # side stream after everything already on this one)
        ctx.ex.defer(gy, x2)
        return dx, None, None, None


def linear(x, weight, bias=None):
    from ..parallel import factored
    from . import param_fence

    if x.is_cuda:  # a deferred (side-stream) optimizer update of this layer must land first
        param_fence.wait(weight)
        param_fence.wait(bias)
    ex = factored.get(weight)
    if ex is not None and torch.is_grad_enabled() and weight.requires_grad:
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        if ex.begin(x2):
            y = _ExchangedLinear.apply(x2, weight, bias, ex)
            return y.reshape(*x.shape[:-1], weight.shape[0])
    if not x.is_cuda:
        return F.linear(x, weight, bias)
    if x.dim() == 2 and x.shape[0] <= 8 and weight.shape[0] <= 16:
        return _LinearSkinny.apply(x, weight, bias)
    # plain library GEMM (hipBLASLt/rocBLAS) for non-skinny shapes
    return F.linear(x, weight, bias)


# --------------------------------------------------------------------------- CrossEntropy
class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index, label_smoothing):
        loss, dlogits = _ext.ops().cross_entropy(logits.contiguous(), labels.contiguous(), ignore_index,
                                                 label_smoothing)
        ctx.save_for_backward(dlogits)  # (labels are integer: autograd already treats them as constants)
        return loss

    @staticmethod
    def backward(ctx, gloss):
        (dlogits,) = ctx.saved_tensors
        if _is_unit_seed(gloss):  # backward(loss) seeded with the cached 1: dlogits as they are
            return dlogits, None, None, None
        g = _ext.ops().scale_by_scalar(dlogits, gloss.reshape(1).contiguous().float())
        return g, None, None, None


_UNIT_SEEDS = {}


def _unit_seed(loss):
    """A cached 0-d 1.0 on loss's device (never written: its version is checked at use)."""
    key = (loss.device, loss.dtype)
    one = _UNIT_SEEDS.get(key)
    if one is None or one._version != 0:
        one = _UNIT_SEEDS[key] = torch.ones((), device=loss.device, dtype=loss.dtype)
    return one


def _is_unit_seed(g) -> bool:
    one = _UNIT_SEEDS.get((g.device, g.dtype))
    return one is not None and g.data_ptr() == one.data_ptr() and g.dim() == 0 and one._version == 0


def backward(loss):
    """``loss.backward()`` for a scalar loss, seeded with a cached device 1.0: autograd's seed
    fill and the loss backward's scale-by-seed kernel are skipped (two ~5 us launches per step)."""
    if loss.dim() != 0 or not loss.is_cuda:
        loss.backward()
        return
    loss.backward(_unit_seed(loss))


class _CrossEntropyFromHead(torch.autograd.Function):
    """The loss and dlogits the fused ConvNet head formed with the logits (models/convnet_fused.py
    attach_labels, csrc/kernels/ce_small.h): the same arithmetic as _CrossEntropy, no launch."""

    @staticmethod
    def forward(ctx, logits, pre):
        loss, dlogits = pre
        ctx.save_for_backward(dlogits)
        return loss

    @staticmethod
    def backward(ctx, gloss):
        (dlogits,) = ctx.saved_tensors
        if _is_unit_seed(gloss):
            return dlogits, None
        return _ext.ops().scale_by_scalar(dlogits, gloss.reshape(1).contiguous().float()), None


def cross_entropy(logits, labels, ignore_index: int = -100, label_smoothing: float = 0.0):
    """Mean-reduced CE (``nn.CrossEntropyLoss()`` defaults) with a fused fwd+bwd kernel."""
    if not logits.is_cuda or logits.dim() != 2:
        return F.cross_entropy(logits, labels, ignore_index=ignore_index, label_smoothing=label_smoothing)
    pre = getattr(logits, "_tds_ce", None)
    if pre is not None:
        logits._tds_ce = None
        version, lab, loss, dlogits = pre
        same = (torch.is_tensor(labels) and labels.dtype == torch.int64 and labels.is_cuda
                and lab == (labels.data_ptr(), tuple(labels.shape), labels.stride(), labels._version))
        if version == logits._version and same and int(ignore_index) == -100 and float(label_smoothing) == 0.0:
            return _CrossEntropyFromHead.apply(logits, (loss, dlogits))
    return _CrossEntropy.apply(logits, labels.long(), int(ignore_index), float(label_smoothing))


# --------------------------------------------------------------------------- data: bilinear u8 upsample
def upsample_bilinear_u8(src: torch.Tensor, H: int, W: int, levels: bool = False) -> torch.Tensor:
    """[B,h,w] uint8 -> [B,1,H,W] float32 in [0,1] (PIL-style bilinear + ToTensor).

    ``levels=True`` returns the rounded uint8 levels instead (the resized PIL image before
    ToTensor): ``ConvNet`` takes such a batch as ``levels / 255`` and its fused plan folds the
    1/255 into conv1, so the 4x larger fp32 image is never written or read."""
    if not src.is_cuda:
        x = src.float().unsqueeze(1)
        y = F.interpolate(x, size=(H, W), mode="bilinear", align_corners=False)
        y = y.round_().clamp_(0, 255)
        return y.to(torch.uint8) if levels else y.div_(255.0)
    return _ext.ops().upsample_bilinear_u8(src.contiguous(), int(H), int(W), bool(levels))


def upsample_levels_moments(src: torch.Tensor, H: int, W: int):
    """``upsample_bilinear_u8(src, H, W, levels=True)`` that also forms the batch's x
    autocorrelation partials -- the weight-independent half of BN1's batch statistics in the fused
    ConvNet plan -- in the same pass over the levels (csrc/kernels/ups_moments.hip).  Returns
    ``(levels, partials)``; hand both to the model with ``convnet_fused.attach_input_stats(levels,
    (partials, None))``.  ``partials`` is None on CPU and for shapes the fused kernel does not take."""
    if not src.is_cuda:
        return upsample_bilinear_u8(src, H, W, levels=True), None
    x, part = _ext.ops().upsample_levels_moments(src.contiguous(), int(H), int(W))
    return x, (part if part.numel() > 0 else None)
