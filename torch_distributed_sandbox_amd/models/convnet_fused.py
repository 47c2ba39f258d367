"""Fused gfx950 execution plan for the ConvNet (training mode).

The reference runs 13 ATen kernels forward and ~20 backward per step on
fp32 NCHW tensors.  This plan runs the network as three
autograd Functions over NHWC/bf16x3 activations (kernels in
``csrc/kernels/convnet_fused.hip`` and ``conv2_bf16x3.hip``):

``_Layer1``  x -> p1            conv1 + BN1(batch stats) + ReLU + pool, conv1 never stored
``_Conv2``   p1 -> y2           conv2 (bf16x3 MFMA) with BN2 batch-stat partials fused
``_Head``    y2 -> logits       BN2 + ReLU + pool + fc in one pass; fc grads into the DDP bucket

Autograd runs the backward head -> conv2 -> layer1, so the fc gradient (the
720 MB DDP bucket) is complete — and its all-reduce launched — before the
conv backward starts (SURVEY.md §3.4 overlap property).

Numerics: conv1, BN, pooling, fc and the loss are exact fp32; conv2
(fwd/dgrad/wgrad) uses the bf16x3 split (hi*hi + hi*lo + lo*hi, fp32
accumulate): ~2^-16 relative error per product, tighter than the TF32
convolutions cuDNN runs for the reference by default.  ``mode='layers'`` is
the exact-fp32 generic path.
"""
from __future__ import annotations

import torch

from .. import _ext
from ..ops import grad_sink, param_fence
from ..parallel import factored


def supported(model, x) -> bool:
    if not (x.is_cuda and model.training and torch.is_grad_enabled()):
        return False
    if x.dim() != 4 or x.shape[1] != 1 or x.dtype != torch.float32:
        return False
    B, _, H, W = x.shape
    if H != W or H < 8 or B > 32 or H % 4 != 0:
        return False
    bn1, bn2 = model.layer1[1], model.layer2[1]
    for bn in (bn1, bn2):
        if not bn.track_running_stats or bn.momentum is None or not bn.affine:
            return False
    c1, c2 = model.layer1[0], model.layer2[0]
    if c1.bias is None or c2.bias is None or model.fc.out_features > 10 or model.fc.bias is None:
        return False
    if any(p.dtype != torch.float32 or not p.is_cuda for p in model.parameters()):
        return False
    return True


class _Layer1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, g1, be1, rm1, rv1, nbt1, momentum, eps):
        ops = _ext.ops()
        x = x.contiguous()
        p1, idx1, stats1, gram = ops.fused_l1_forward(x, w1, b1, g1, be1, rm1, rv1, nbt1, momentum, eps)
        ctx.save_for_backward(x, p1, idx1, w1, b1, g1, stats1, gram)
        ctx.mark_non_differentiable(idx1)
        return p1

    @staticmethod
    def backward(ctx, dp1):
        x, p1, idx1, w1, b1, g1, stats1, gram = ctx.saved_tensors
        dw1, db1, dg1, dbe1 = _ext.ops().fused_l1_backward(dp1.contiguous(), x, p1, idx1, w1, b1, g1, stats1, gram, 1.0)
        return None, dw1, db1, dg1, dbe1, None, None, None, None, None


class _Conv2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, p1, w2, b2):
        ops = _ext.ops()
        wp, wd = ops.conv2_pack(w2.contiguous())
        y2, partial2 = ops.fused_conv2_forward(p1, wp, b2)
        ctx.save_for_backward(p1, wd)
        ctx.mark_non_differentiable(partial2)
        return y2, partial2

    @staticmethod
    def backward(ctx, dy2, _unused):
        p1, wd = ctx.saved_tensors
        dp1, dw2, db2 = _ext.ops().fused_conv2_backward(dy2.contiguous(), p1, wd, ctx.needs_input_grad[0], 1.0)
        return (dp1 if ctx.needs_input_grad[0] else None), dw2, db2


class _Head(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y2, partial2, b2, g2, be2, rm2, rv2, nbt2, momentum, eps, wfc, bfc, ex):
        ops = _ext.ops()
        x_out = None
        if ex is not None:
            B, P = y2.shape[0], y2.shape[1]
            x_out = torch.empty((B, wfc.shape[1]), device=y2.device, dtype=torch.float32)
        logits, stats2, aff2 = ops.fused_head_forward(y2, partial2, b2, g2, be2, rm2, rv2, nbt2, momentum, eps, wfc,
                                                      bfc, x_out)
        if ex is not None and not ex.begin(x_out):
            raise RuntimeError("activation exchange refused to start after ready() agreed")
        ctx.save_for_backward(y2, stats2, aff2, g2, wfc)
        ctx.wfc_param = wfc
        ctx.ex = ex
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        y2, stats2, aff2, g2, wfc = ctx.saved_tensors
        dlogits = dlogits.contiguous().float()
        ex = ctx.ex
        if ex is not None:
            # fc gradients come from the activation exchange (parallel/factored.py)
            _, _, dg2, dbe2, dy2 = _ext.ops().fused_head_backward(dlogits, y2, stats2, aff2, g2, wfc, None, 1.0,
                                                                  False)
            ex.defer(dlogits)
            return dy2, None, None, dg2, dbe2, None, None, None, None, None, None, None, None
        dw_out = grad_sink.acquire(ctx.wfc_param if ctx.needs_input_grad[10] else None, wfc.shape, wfc)
        dW, dbfc, dg2, dbe2, dy2 = _ext.ops().fused_head_backward(dlogits, y2, stats2, aff2, g2, wfc, dw_out, 1.0)
        return dy2, None, None, dg2, dbe2, None, None, None, None, None, dW, dbfc, None


def forward(model, x):
    conv1, bn1 = model.layer1[0], model.layer1[1]
    conv2, bn2 = model.layer2[0], model.layer2[1]
    fc = model.fc
    p1 = _Layer1.apply(x, conv1.weight, conv1.bias, bn1.weight, bn1.bias, bn1.running_mean, bn1.running_var,
                       bn1.num_batches_tracked, float(bn1.momentum), float(bn1.eps))
    y2, partial2 = _Conv2.apply(p1, conv2.weight, conv2.bias)
    # the fc update may still be running on DDP's side stream (overlap_optimizer): wait here,
    # after the convolutions were queued, not before
    param_fence.wait(fc.weight)
    param_fence.wait(fc.bias)
    ex = factored.get(fc.weight)
    if ex is not None and not ex.ready(x.shape[0]):
        ex = None
    return _Head.apply(y2, partial2, conv2.bias, bn2.weight, bn2.bias, bn2.running_mean, bn2.running_var,
                       bn2.num_batches_tracked, float(bn2.momentum), float(bn2.eps), fc.weight, fc.bias, ex)
