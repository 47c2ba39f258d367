"""Fused gfx950 execution plan for the ConvNet (training mode).

The reference runs 13 ATen kernels forward and ~20 backward per step on
fp32 NCHW tensors.  This plan runs the network as three
autograd Functions over NHWC fp16 / uint8-level activations (kernels in
``csrc/kernels/convnet_fused.hip``, ``conv2_fwd2.hip``, ``conv2_bwd.hip``, ``head_pb.hip``):

``_Layer1``  x -> p1            conv1 + BN1(batch stats) + ReLU + pool, conv1 never stored; p1 in fp16
``_Conv2``   p1 -> y2, ya       conv2 (TF32-class fp16 MFMA) with BN2 batch-stat partials and the 2x2
                                max-pool (ya = y2 at each window's argmax, resolved by the sign
                                of BN2's gamma, in fp16 as y2h stores it) fused; its backward
                                rebuilds dy2 from y2 in LDS
                                (BN2/pool backward fused)
``_Head``    ya -> logits       BN2 affine + ReLU + fc streamed over ya and the fc weight; fc
                                grads into the DDP bucket (or the SGD step fused in)

ya and the pooled gradient g2m use the pooled-blocked layout of
``csrc/kernels/pooled_layout.h``.  Autograd runs the backward head -> conv2 ->
layer1, so the fc gradient (the 720 MB DDP bucket) is complete — and its
collective launched — before the conv backward starts (SURVEY.md §3.4 overlap
property).

Numerics: BN, pooling, fc, the loss and SGD are exact fp32.  conv1 (fwd + wgrad) uses the
bf16x3 split (hi*hi + hi*lo + lo*hi, fp32 accumulate, ~2^-16 per product; on uint8 level input
bf16x2, the level exact; the level-input weight gradient one fp16 MFMA, dp1h and the level both
exact in fp16).  conv2 (fwd, dgrad, wgrad) runs in the TF32 class (round-4 default): ONE fp16 MFMA
per product with both operands rounded once to 11 significant bits -- TF32's significand, the
arithmetic of the cuDNN convolutions the reference runs under PyTorch's default ``allow_tf32`` --
at exact power-of-two range scales (p1 by BN1's Samuelson bound, the weights by their max, the
conv2 output gradient by the step's magnitude bounds ``mag``); docs/KERNELS.md "conv2 in the TF32
class".
``mode='layers'`` is the exact-fp32 generic path.

Gradient hand-off beside autograd: the fp16 p1 is an autograd output, but its gradient dp1 is
fp32; the conv2 backward hands dp1 to the layer-1 backward through a link object and gives
autograd a zero-stride fp16 placeholder (no kernel, no memory), as it does for y2.
"""
from __future__ import annotations

import os

import torch

from .. import _ext
from ..ops import fused_update, grad_sink, param_fence
from ..parallel import factored


def supported(model, x) -> bool:
    if not (x.is_cuda and model.training and torch.is_grad_enabled()):
        return False
    # uint8: ToTensor's levels, x = levels / 255 folded into conv1 (models/convnet.py to_image)
    if x.dim() != 4 or x.shape[1] != 1 or x.dtype not in (torch.float32, torch.uint8):
        return False
    B, _, H, W = x.shape
    # H % 4: conv2 runs on the pooled P = H/2 grid and pools again; H >= 16: the head's 4-column
    # weight groups fit in a pooled row (Q >= 4); H <= 65520: the conv2 tile
    # order table packs tile rows/columns in 12 bits (P/8 <= 4095); B <= 32: layer-1 partials
    if H != W or H < 16 or B > 32 or H % 4 != 0 or H > 65520:
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


# ---- input pipeline hand-off ---------------------------------------------------------
# BN1's batch statistics are the batch's x moments (autocorrelation sums + border strips,
# ops.l1_input_stats) contracted with conv1's weights.  The moments depend on the batch only, so
# an input pipeline may compute them with the batch, on its own stream, and attach them to it;
# _Layer1 then skips that part.  The pipeline is responsible for ordering (the consuming stream
# waits on the producing stream before the forward, and the tensors are record_stream'ed).


def input_stats(x):
    """(asum[42], strips[B*8*82]) fp64 x moments of a [B,1,H,W] fp32 batch, on the current stream
    (of the levels for a uint8 batch: l1_gram scales them)."""
    return _ext.ops().l1_input_stats(x.contiguous())


def attach_input_stats(x, stats):
    """Hand precomputed ``input_stats(x)`` -- or ``(partials, None)`` from
    ``ops.functional.upsample_levels_moments`` -- to the forward that consumes ``x`` (valid until x
    is modified in place)."""
    x._tds_l1_stats = (x._version, stats)
    return x


def _take_input_stats(x):
    st = getattr(x, "_tds_l1_stats", None)
    if st is None or st[0] != x._version:
        return None, None
    return st[1]


# The batch's labels, attached by the training loop before the forward: the head forward's
# finalizing workgroup then forms the cross-entropy loss and dlogits right after the logits
# (ops.fused_head_forward_aff_ce), and ops.functional.cross_entropy takes them from the logits
# instead of launching its own kernel.  Only torch's CrossEntropyLoss defaults (mean, ignore_index
# -100, no label smoothing) are formed in the head; any other use of the logits is unaffected.
def attach_labels(x, labels):
    """Hand the batch's labels to the forward that consumes ``x`` (valid until x is modified in place)."""
    x._tds_labels = (x._version, labels)
    return x


def _take_labels(x):
    lb = getattr(x, "_tds_labels", None)
    if lb is None or lb[0] != x._version:
        return None
    labels = lb[1]
    if not (torch.is_tensor(labels) and labels.dtype == torch.int64 and labels.dim() == 1 and labels.is_cuda
            and labels.device == x.device and labels.shape[0] == x.shape[0] and labels.is_contiguous()):
        return None
    return labels


# One-shot callbacks run (on the host, in the backward's thread) right before the conv2
# backward -- the step's longest, MFMA-bound kernel -- is enqueued: work they put on another
# stream after waiting on the current one runs beside it (bench.py / trainer input prefetch).
_before_conv2_backward = []
_before_head_forward = []


def before_conv2_backward(fn):
    _before_conv2_backward.append(fn)


def before_head_forward(fn):
    """``fn()`` runs once, when the next fused head forward is about to be queued (the input
    pipeline's prefetch point: work queued on another stream there runs beside the memory-bound
    head kernels, whose register and LDS use leave room for it -- the persistent conv kernels
    before and after them leave none)."""
    _before_head_forward.append(fn)


def _run_before_conv2_backward():
    while _before_conv2_backward:
        _before_conv2_backward.pop(0)()


def _run_before_head_forward():
    while _before_head_forward:
        _before_head_forward.pop(0)()


def _sinks(ctx, params, first):
    """Gradient destinations for ``params`` (bucket views when DDP registered sinks,
    ops/grad_sink.py; None for parameters that need no gradient).  ``first`` is the
    forward-input index of params[0], or a tuple of indices."""
    idx = first if isinstance(first, tuple) else tuple(range(first, first + len(params)))
    return [grad_sink.acquire(p, p.shape, p) if p is not None and ctx.needs_input_grad[i] else None
            for p, i in zip(params, idx)]


_ZERO = {}
# counters the tests read: forward passes that applied the exchange's weight update in the head kernel,
# and layer-1 forwards that took x moments precomputed by the input pipeline
STATS = {"precomputed_input_moments": 0, "head_fused_ce": 0, "head_range_launches": 0}


def _zero_scalar(device, dtype):
    """Cached 0-d zero per (device, dtype): the y2 gradient placeholder costs no fill kernel."""
    key = (device, dtype)
    z = _ZERO.get(key)
    if z is None:
        z = _ZERO[key] = torch.zeros((), device=device, dtype=dtype)
    return z


class _Layer1Link:
    """Carries the conv2 backward's dp1h (fp16, scaled: csrc/kernels/conv2_common.h) and its decode
    factor to the layer-1 backward, and the power-of-two scale p1 is stored at to the conv2 kernels."""

    __slots__ = ("dp1", "dp1_dec", "p1_scale", "mag", "pack")

    def __init__(self):
        self.mag = None  # the step's magnitude workspace when layer 1 packs conv2's weights
        self.pack = (None, None, None)  # (w2, wp, wd) for that packing


class _Layer1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, g1, be1, rm1, rv1, nbt1, momentum, eps, link1):
        ops = _ext.ops()
        asum, strips = _take_input_stats(x)
        if asum is not None:
            STATS["precomputed_input_moments"] += 1
        x = x.contiguous()
        p1, idx1, stats1, gram, p1_scale = ops.fused_l1_forward(x, w1, b1, g1, be1, rm1, rv1, nbt1, momentum, eps,
                                                                asum, strips, link1.mag, *link1.pack)
        link1.pack = (None, None, None)
        link1.p1_scale = p1_scale  # p1's fp16 range guard (a power of two, 1 normally): conv2 takes it out
        ctx.save_for_backward(x, p1, idx1, w1, b1, g1, stats1, gram)
        ctx.params = (w1, b1, g1, be1)
        ctx.link1 = link1
        ctx.mark_non_differentiable(idx1)
        return p1

    @staticmethod
    def backward(ctx, _dp1_placeholder):
        x, p1, idx1, w1, b1, g1, stats1, gram = ctx.saved_tensors
        dp1, dp1_dec = ctx.link1.dp1, ctx.link1.dp1_dec
        ctx.link1.dp1 = ctx.link1.dp1_dec = None
        outs = _sinks(ctx, ctx.params, 1)
        dw1, db1, dg1, dbe1 = _ext.ops().fused_l1_backward(dp1, dp1_dec, x, p1, idx1, w1, b1, g1, stats1, gram, 1.0,
                                                           *outs)
        return None, dw1, db1, dg1, dbe1, None, None, None, None, None, None


class _Layer2Link:
    """Carries the head backward's pooled gradient (g2m) and BN2 backward constants to the
    conv2 backward, which rebuilds dy2 tile by tile in LDS (never in HBM).  The two stay
    separate autograd nodes so the fc gradient's AccumulateGrad — and with it the DDP bucket
    all-reduce — fires before the conv2 backward runs."""

    __slots__ = ("g2m", "kbuf", "aff2", "mag", "bn_done", "fc_update", "labels", "ce", "pack", "pooled")

    def __init__(self):
        self.fc_update = None  # the activation exchange's grouped deferred update, run range by range
        self.pack = None  # (wp, wd): conv2's weights packed by the layer-1 forward (_pack_in_layer1)
        self.mag = None
        self.labels = None  # the batch's labels (attach_labels) -> ce = (labels, loss, dlogits) from the head
        self.ce = None
        self.pooled = False  # the activation exchange started from the pooled input (forward below)


# The small reductions behind BN2 (forward statistics, backward constants) and the logits run
# inside the producing kernels' launches (the last workgroup to arrive finalizes: common.h
# tds_arrive) instead of as separate launches; TDS_FUSED_FIN=0 restores the separate launches.
_FUSED_FIN = os.environ.get("TDS_FUSED_FIN", "1").strip() != "0"


class _Conv2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, p1, w2, b2, g2, be2, rm2, rv2, nbt2, momentum, eps, link, link1):
        ops = _ext.ops()
        # magnitude bounds of this step (per-workgroup max |y2 - b2| here, max |g2m| in the head
        # backward): the conv2 backward's fp16 scale of dy2
        if link.pack is not None:  # packed by the layer-1 reducer's launch (its Gram stored 1 / p1_scale)
            wp, wd = link.pack
            link.pack = None
        else:
            link.mag = torch.empty(ops.mag_numel(p1.shape[0], p1.shape[1]), device=p1.device, dtype=torch.int32)
            wp, wd = ops.conv2_pack(w2.contiguous(), link.mag, getattr(link1, "p1_scale", None))
        # a2: each pooling window's argmax, saved for the backward (max_pool2d_with_indices' indices)
        link.bn_done = _FUSED_FIN
        if _FUSED_FIN:
            # BN2 finalized in the conv2 forward's launch: (stats2, aff2) instead of the partials
            y2, ya, a2, bn_a, bn_b = ops.fused_conv2_forward_bn(p1, wp, b2, g2, be2, rm2, rv2, nbt2, momentum, eps,
                                                                link.mag)
        else:
            y2, bn_a, ya, a2 = ops.fused_conv2_forward(p1, wp, b2, g2, link.mag)
            bn_b = bn_a.new_empty(0)
        # b2 saved (autograd's version check): y2h is stored without the conv bias and the backward
        # rebuilds y2 with it, so an in-place change to b2 before the backward must raise
        ctx.save_for_backward(p1, wd, y2, a2, b2)
        ctx.params = (w2, b2)
        ctx.link = link
        ctx.link1 = link1
        ctx.mark_non_differentiable(ya, bn_a, bn_b)
        # no zero-filled gradients for ya / the BN2 tensors (a 360 MB fill per step at the bench shape)
        ctx.set_materialize_grads(False)
        return y2, ya, bn_a, bn_b

    @staticmethod
    def backward(ctx, _dy2_placeholder, _unused_ya, _unused_a, _unused_b):
        p1, wd, y2, a2, b2 = ctx.saved_tensors
        link = ctx.link
        _run_before_conv2_backward()
        # BN2 / ReLU / pool backward fused into the conv2 data + weight gradients
        dp1, dw2, db2 = _ext.ops().fused_conv2_backward_y2(y2, a2, link.g2m, link.aff2, link.kbuf, b2, link.mag,
                                                           p1, wd, 1.0, *_sinks(ctx, ctx.params, 1))
        mag = link.mag
        link.g2m = link.kbuf = link.aff2 = link.mag = None
        dp1_ph = None
        if ctx.needs_input_grad[0]:
            # dp1h (fp16, scaled) and its decode factor, which the conv2 backward wrote into mag
            ctx.link1.dp1, ctx.link1.dp1_dec = dp1, mag[44:45]
            dp1_ph = _zero_scalar(p1.device, p1.dtype).expand(p1.shape)
        return dp1_ph, dw2, db2, None, None, None, None, None, None, None, None, None


def _head_forward_grouped(ops, ya, aff2, b2, wfc, bfc, P, ex, upd, link):
    """The head forward with the grouped zero-suppressed activation exchange (parallel/factored.py):
    one launch per column group (whole channel planes), each group's fc input rows handed to the
    exchange right after its launch is queued -- its encode and gathers start there, while the next
    ranges run -- and the previous step's exchanged update (``upd``) queued group by group right
    before the launch that reads those columns.  The launch completing the 32nd channel finishes
    the logits (and, with the batch's labels, the cross-entropy) in itself."""
    B, K = ya.shape[0], wfc.shape[1]
    QQ = K // 32
    groups = ex.begin_groups(B, K, ya.device, planes=32)
    ws = ops.head_forward_range_ws(ya, wfc, P)
    for gi, (k0, k1) in enumerate(groups):
        if upd is not None:
            upd.run_until(k1)
        xg = torch.empty((B, k1 - k0), device=ya.device, dtype=torch.float32)
        ops.fused_head_forward_range(ya, aff2, b2, link.mag, wfc, bfc, P, k0 // QQ, k1 // QQ, *ws, link.labels, xg)
        ex.group_ready(gi, xg)
    if upd is not None:
        upd()  # (groups past the last range, had the geometry changed)
    STATS["head_range_launches"] += len(groups)
    if link.labels is not None:
        link.ce = (link.labels, ws[4], ws[3])
        STATS["head_fused_ce"] += 1
    return ws[2]


class _Head(torch.autograd.Function):
    """BN2 finalize + affine + ReLU + fc over ya.  y2 is an input only so that autograd routes
    the conv2 backward through this node: its gradient travels in the link (g2m, BN2 backward
    constants), autograd gets a zero-stride placeholder."""

    @staticmethod
    def forward(ctx, y2, ya, bn_a, bn_b, b2, g2, be2, rm2, rv2, nbt2, momentum, eps, wfc, bfc, ex, link):
        ops = _ext.ops()
        _run_before_head_forward()
        P = y2.shape[1]
        B, K = ya.shape[0], wfc.shape[1]
        upd, link.fc_update = link.fc_update, None
        pooled = link.pooled  # (its gathers were started right after the conv2 forward: forward below)
        if pooled:
            pass
        elif link.bn_done and ex is not None and _FUSED_FIN and B <= 8 and ex.grouped(B, K):
            logits = _head_forward_grouped(ops, ya, bn_b, b2, wfc, bfc, P, ex, upd, link)
            ctx.save_for_backward(ya, bn_a, bn_b, b2, g2, wfc)
            ctx.P = P
            ctx.y2_meta = (y2.shape, y2.dtype, y2.device)
            ctx.wfc_param = wfc
            ctx.small = (bfc, g2, be2)
            ctx.ex = ex
            ctx.link = link
            return logits
        if upd is not None:
            upd()  # the whole deferred update, before the weight is read
        x_out = None
        # the activation / sharded exchanges send the fc input rows X, which the head writes
        if ex is not None and not pooled and ex.planned(B) in ("activations", "sharded"):
            x_out = torch.empty((B, K), device=ya.device, dtype=torch.float32)
        if link.bn_done:  # (bn_a, bn_b) = BN2's (stats, affine), finalized by the conv2 forward
            stats2, aff2 = bn_a, bn_b
            if link.labels is not None:
                # the loss and dlogits formed by the head forward's finalizing workgroup
                logits, loss, dlogits = ops.fused_head_forward_aff_ce(ya, aff2, b2, link.mag, wfc, bfc, P, link.labels,
                                                                      x_out)
                link.ce = (link.labels, loss, dlogits)
                STATS["head_fused_ce"] += 1
            else:
                logits = ops.fused_head_forward_aff(ya, aff2, b2, link.mag, wfc, bfc, P, x_out)
        else:  # bn_a = the conv2 forward's BN2 partials
            logits, stats2, aff2 = ops.fused_head_forward(ya, bn_a, b2, g2, be2, rm2, rv2, nbt2, momentum, eps, wfc,
                                                          bfc, P, x_out, mag=link.mag)
        if ex is not None and not pooled:
            started = ex.begin(x_out, rows=B)
            if not started:
                raise RuntimeError("fc gradient exchange refused to start after ready() agreed")
        ctx.save_for_backward(ya, stats2, aff2, b2, g2, wfc)
        ctx.P = P
        ctx.y2_meta = (y2.shape, y2.dtype, y2.device)
        ctx.wfc_param = wfc
        ctx.small = (bfc, g2, be2)
        ctx.ex = ex
        ctx.link = link
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        ya, stats2, aff2, b2, g2, wfc = ctx.saved_tensors
        dlogits = dlogits.contiguous().float()
        ex = ctx.ex
        ops = _ext.ops()
        P = ctx.P
        if ex is not None and ex.active == "chunked":
            # K-chunked fc gradient (parallel/factored.py): one launch per channel group, each
            # group's dW columns all-reduced as soon as it lands; grads published by the exchange
            (dw, acc_w), (db, acc_b) = ex.chunk_targets()
            B, Q = ya.shape[0], P // 2
            # fp16 at per-channel scales (kernels/head_pb.hip), with 64 B of slack past the end: the conv2
            # backward's row loads (ops.fused_conv2_backward_y2)
            g2m_buf = torch.empty(B * 32 * Q * Q + 32, device=ya.device, dtype=torch.float16)[:B * 32 * Q * Q].view(
                B, 32, Q, Q)
            part = torch.empty(ops.head_bwd_workspace(B, P), device=ya.device, dtype=torch.float64)
            _, dg_o, dbe_o = _sinks(ctx, ctx.small, (13, 5, 6))
            # accumulating under no_sync(): this step's chunk goes to a scratch dW, then is added
            dst = torch.empty_like(dw) if acc_w else dw
            chunks = ex.column_chunks(wfc.shape[1], planes=32)
            for i, (k0, k1) in enumerate(chunks):
                last = i == len(chunks) - 1
                res = ops.fused_head_backward(dlogits, ya, stats2, aff2, b2, g2, wfc, P, dst, 1.0, True, 0.0,
                                              None, dg_o if last else None, dbe_o if last else None, True,
                                              k0 // (Q * Q), k1 // (Q * Q), last, g2m_buf, part, ctx.link.mag)
                if acc_w:
                    dw[:, k0:k1].add_(dst[:, k0:k1])
                ex.chunk_ready(dw, k0, k1)
            _, dbfc_c, dg2, dbe2, g2m, kbuf = res
            if db is not None:
                db.add_(dbfc_c) if acc_b else db.copy_(dbfc_c)
            ex.chunked_done(dw, db)
            dW = dbfc = None
        elif ex is not None:
            # fc gradients come from the activation exchange (parallel/factored.py)
            _, _, dg2, dbe2, g2m, kbuf = ops.fused_head_backward(dlogits, ya, stats2, aff2, b2, g2, wfc, P, None, 1.0,
                                                                 False, mag=ctx.link.mag, ypart_done=ctx.link.bn_done)
            ex.defer(dlogits)
            dW = dbfc = None
        else:
            # world size 1 under DDP(overlap_optimizer): the SGD step of the fc weight runs in
            # this same kernel (ops/fused_update.py)
            lr = None
            if ctx.needs_input_grad[12] and ya.shape[0] <= 8:  # one pass of head_bwd_pb_kernel
                lr = fused_update.take(ctx.wfc_param)
            keep = not lr or fused_update.keep_grad(ctx.wfc_param)
            # the gradient's destination (DDP's bucket slot) only when a gradient is written: an
            # update-only step never requests the slot, so DDP never allocates it (ddp.py _lazy_from)
            dw_out = grad_sink.acquire(ctx.wfc_param if ctx.needs_input_grad[12] and keep else None, wfc.shape, wfc)
            dbfc_o, dg_o, dbe_o = _sinks(ctx, ctx.small, (13, 5, 6))
            dW, dbfc, dg2, dbe2, g2m, kbuf = ops.fused_head_backward(dlogits, ya, stats2, aff2, b2, g2, wfc, P,
                                                                     dw_out if keep else None, 1.0, True,
                                                                     float(lr or 0.0), dbfc_o, dg_o, dbe_o, keep,
                                                                     mag=ctx.link.mag, ypart_done=ctx.link.bn_done)
            if lr:
                # update-only step: no gradient for the weight (dW is None), as in torch's
                # optimizer-in-backward; the owner marks the parameter ready
                fused_update.applied(ctx.wfc_param, grad_written=keep)
        link = ctx.link
        link.g2m, link.kbuf, link.aff2 = g2m, kbuf, aff2
        shape, dtype, device = ctx.y2_meta
        dy2 = _zero_scalar(device, dtype).expand(shape)
        return (dy2, None, None, None, None, dg2, dbe2, None, None, None, None, None, dW, dbfc, None, None)


# conv2's weight packing (conv2_pack: fp16 fragments of the forward / data gradient and their range
# scales; 64 workgroups, ~9 us as its own launch) depends on the weights only, except for the
# inverse of p1's range scale, which the layer-1 Gram then stores itself: it runs as extra
# workgroups of the layer-1 reducer's launch (fused_l1_forward's w2 / wp_out / wd_out), one launch
# fewer between layer 1 and conv2.  (Queued on a side stream instead it cost a cross-stream wait
# before the conv2 forward and host time before layer 1: not faster, r5_s32.)
_PACK_IN_L1 = os.environ.get("TDS_PACK_IN_L1", "1").strip() != "0"


def _pack_in_layer1(w2, x, link, link1):
    if not (_PACK_IN_L1 and x.is_cuda and x.dim() == 4):
        return
    ops = _ext.ops()
    dev = x.device
    param_fence.wait(w2)  # a deferred update of the weights (overlap_optimizer) lands first
    mag = torch.empty(ops.mag_numel(x.shape[0], x.shape[2] // 2), device=dev, dtype=torch.int32)
    wp = torch.empty(13 * 2 * 4 * 16 * 8, device=dev, dtype=torch.int16)
    wd = torch.empty(25 * 4 * 16 * 8, device=dev, dtype=torch.int16)
    link.mag = link1.mag = mag
    link1.pack = (w2.detach(), wp, wd)
    link.pack = (wp, wd)


def forward(model, x):
    conv1, bn1 = model.layer1[0], model.layer1[1]
    conv2, bn2 = model.layer2[0], model.layer2[1]
    fc = model.fc
    link1 = _Layer1Link()
    link = _Layer2Link()
    _pack_in_layer1(conv2.weight, x, link, link1)
    p1 = _Layer1.apply(x, conv1.weight, conv1.bias, bn1.weight, bn1.bias, bn1.running_mean, bn1.running_var,
                       bn1.num_batches_tracked, float(bn1.momentum), float(bn1.eps), link1)
    y2, ya, bn_a, bn_b = _Conv2.apply(p1, conv2.weight, conv2.bias, bn2.weight, bn2.bias, bn2.running_mean,
                                      bn2.running_var, bn2.num_batches_tracked, float(bn2.momentum), float(bn2.eps),
                                      link, link1)
    # the activation exchange from the pooled input (parallel/factored.py "pooled"): ya and this
    # rank's head constants leave right here, after the conv2 forward and before the previous step's
    # deferred fc update and the head forward, which then write no fc input rows
    ex = factored.get(fc.weight)
    B = x.shape[0]
    if ex is not None and link.bn_done and B <= 8 and ex.ready(B) and ex.pooled(B):
        ops = _ext.ops()
        ex.begin_pooled(ya, ops.head_pooled_record(bn_b, conv2.bias, link.mag), y2.shape[1])
        link.pooled = True
    # the fc update may still be running on DDP's side stream (overlap_optimizer), or deferred to
    # here (the activation exchange's update sweep, factored.py _Update): wait / queue it now, after
    # the convolutions were queued, not before.  A grouped update goes to the head forward, which
    # queues it range by range
    link.fc_update = param_fence.take(fc.weight, "groups")
    param_fence.wait(fc.weight)
    param_fence.wait(fc.bias)
    if ex is not None and not link.pooled and not ex.ready(x.shape[0]):
        ex = None
    link.labels = _take_labels(x)
    logits = _Head.apply(y2, ya, bn_a, bn_b, conv2.bias, bn2.weight, bn2.bias, bn2.running_mean, bn2.running_var,
                         bn2.num_batches_tracked, float(bn2.momentum), float(bn2.eps), fc.weight, fc.bias, ex, link)
    if link.ce is not None:
        lab = link.ce[0]
        # (ops.functional.cross_entropy takes it for these very labels: same memory, unchanged since)
        logits._tds_ce = (logits._version, (lab.data_ptr(), tuple(lab.shape), lab.stride(), lab._version)) + link.ce[1:]
        link.ce = None
    link.labels = None
    return logits
