"""Numerics of every native HIP kernel vs a plain PyTorch fp32/fp64 reference (GPU only)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ops():
    import torch_distributed_sandbox_amd as tds

    return tds._ext.ops()


def _close(a, b, rtol=1e-4, atol=1e-5):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    scale = b.abs().max().item() + 1e-12
    err = (a - b).abs().max().item()
    assert err <= atol + rtol * scale, f"max abs err {err:.3e} vs scale {scale:.3e}"


def test_relu(gpu):
    x = torch.randn(3, 5, 33, 17, device=gpu)
    y = _ops().relu_fwd(x)
    _close(y, F.relu(x), 0, 0)
    g = torch.randn_like(x)
    _close(_ops().relu_bwd(g, y), g * (x > 0), 0, 0)


@pytest.mark.parametrize("shape", [(2, 3, 8, 8), (1, 4, 37, 70), (3, 2, 5, 9)])
def test_maxpool(gpu, shape):
    x = torch.randn(*shape, device=gpu)
    y, idx = _ops().maxpool2_fwd(x)
    ref, ref_idx = F.max_pool2d(x, 2, 2, return_indices=True)
    _close(y, ref, 0, 0)
    gy = torch.randn_like(y)
    gx = _ops().maxpool2_bwd(gy, idx, shape[2], shape[3])
    xr = x.clone().requires_grad_(True)
    F.max_pool2d(xr, 2, 2).backward(gy)
    _close(gx, xr.grad, 0, 0)


@pytest.mark.parametrize("cin,cout,h,w", [(1, 16, 40, 70), (16, 32, 23, 131), (3, 5, 9, 9), (16, 32, 64, 64)])
def test_conv_fwd_bwd(gpu, cin, cout, h, w):
    torch.manual_seed(0)
    x = torch.randn(2, cin, h, w, device=gpu)
    wt = torch.randn(cout, cin, 5, 5, device=gpu) * 0.1
    b = torch.randn(cout, device=gpu)
    y = _ops().conv2d_fwd(x, wt, b, 2)
    ref = F.conv2d(x.double().cpu(), wt.double().cpu(), b.double().cpu(), padding=2)
    _close(y, ref, 1e-5, 1e-5)
    gy = torch.randn_like(y)
    xr = x.double().cpu().requires_grad_(True)
    wr = wt.double().cpu().requires_grad_(True)
    br = b.double().cpu().requires_grad_(True)
    F.conv2d(xr, wr, br, padding=2).backward(gy.double().cpu())
    dx = _ops().conv2d_dgrad(gy, wt, 2)
    _close(dx, xr.grad, 1e-5, 1e-5)
    dw, db = _ops().conv2d_wgrad(x, gy, 5, 2, True)
    _close(dw, wr.grad, 1e-5, 1e-4)
    _close(db, br.grad, 1e-5, 1e-4)


def test_batchnorm_train(gpu):
    torch.manual_seed(0)
    x = torch.randn(4, 6, 19, 23, device=gpu) * 3 + 1.5
    g = torch.rand(6, device=gpu) + 0.5
    be = torch.randn(6, device=gpu)
    rm, rv = torch.zeros(6, device=gpu), torch.ones(6, device=gpu)
    nb = torch.zeros((), dtype=torch.long, device=gpu)
    y, mean, invstd = _ops().bn_fwd_train(x, g, be, rm, rv, nb, 0.1, 1e-5, False)
    rm2, rv2 = torch.zeros(6, dtype=torch.float64), torch.ones(6, dtype=torch.float64)
    xr = x.double().cpu().requires_grad_(True)
    gr = g.double().cpu().requires_grad_(True)
    br = be.double().cpu().requires_grad_(True)
    ref = F.batch_norm(xr, rm2, rv2, gr, br, True, 0.1, 1e-5)
    _close(y, ref, 1e-5, 1e-5)
    _close(rm, rm2, 1e-5, 1e-6)
    _close(rv, rv2, 1e-5, 1e-6)
    assert int(nb.item()) == 1
    gy = torch.randn_like(x)
    ref.backward(gy.double().cpu())
    dx, dg, db = _ops().bn_bwd(gy, x, g, mean, invstd, True)
    _close(dx, xr.grad, 1e-4, 1e-5)
    _close(dg, gr.grad, 1e-5, 1e-4)
    _close(db, br.grad, 1e-5, 1e-4)
    # eval
    ye = _ops().bn_fwd_eval(x, g, be, rm, rv, 1e-5, True)
    _close(ye, F.relu(F.batch_norm(x, rm, rv, g, be, False, 0.1, 1e-5)), 1e-5, 1e-5)


@pytest.mark.parametrize("m,n,k", [(5, 10, 4096 * 3 + 4), (3, 7, 1001), (8, 16, 100000)])
def test_linear(gpu, m, n, k):
    torch.manual_seed(0)
    x = torch.randn(m, k, device=gpu)
    w = torch.randn(n, k, device=gpu) * 0.01
    b = torch.randn(n, device=gpu)
    y = _ops().linear_fwd(x, w, b)
    _close(y, F.linear(x.double(), w.double(), b.double()), 1e-5, 1e-5)
    gy = torch.randn(m, n, device=gpu)
    dw = torch.empty_like(w)
    db = torch.empty_like(b)
    dx = _ops().linear_bwd_into(gy, x, w, dw, db, 1.0, False, True)
    _close(dx, gy.double() @ w.double(), 1e-5, 1e-5)
    _close(dw, gy.double().t() @ x.double(), 1e-5, 1e-5)
    _close(db, gy.double().sum(0), 1e-5, 1e-6)
    # scaled accumulate into existing buffer
    dw2 = dw.clone()
    _ops().linear_bwd_into(gy, x, w, dw2, None, 0.5, True, False)
    _close(dw2, dw.double() * 1.5, 1e-5, 1e-5)


def test_cross_entropy(gpu):
    torch.manual_seed(0)
    z = torch.randn(5, 10, device=gpu) * 3
    lab = torch.tensor([1, 0, 9, -100, 4], device=gpu)
    loss, dz = _ops().cross_entropy(z, lab, -100, 0.0)
    zr = z.double().cpu().requires_grad_(True)
    ref = F.cross_entropy(zr, lab.cpu())
    ref.backward()
    _close(loss, ref, 1e-6, 1e-6)
    _close(dz, zr.grad, 1e-6, 1e-6)
    loss2, dz2 = _ops().cross_entropy(z, lab, -100, 0.1)
    zr2 = z.double().cpu().requires_grad_(True)
    ref2 = F.cross_entropy(zr2, lab.cpu(), label_smoothing=0.1)
    ref2.backward()
    _close(loss2, ref2, 1e-6, 1e-6)
    _close(dz2, zr2.grad, 1e-6, 1e-6)


def test_cross_entropy_out_of_range_label_gives_nan(gpu):
    """torch raises 'Target out of bounds'; the kernel cannot raise, so a label outside [0, N)
    (not ignore_index) makes the loss and that row's dlogits NaN -- never a read past the row.
    The other rows' dlogits are unchanged."""
    torch.manual_seed(0)
    z = torch.randn(4, 10, device=gpu)
    for bad in (10, -1, 1 << 40):
        lab = torch.tensor([1, bad, 3, -100], device=gpu)
        loss, dz = _ops().cross_entropy(z, lab, -100, 0.0)
        torch.cuda.synchronize()
        assert torch.isnan(loss).all()
        assert torch.isnan(dz[1]).all()
        assert torch.isfinite(dz[[0, 2, 3]]).all()


def test_cross_entropy_backward_seeds(gpu):
    """TF.backward(loss) (cached unit seed, no scale kernel) == loss.backward() == 2x for a 2 seed."""
    from torch_distributed_sandbox_amd.ops import functional as TF

    torch.manual_seed(0)
    z0 = torch.randn(5, 10, device=gpu) * 3
    lab = torch.tensor([1, 0, 9, 2, 4], device=gpu)
    grads = []
    for how in ("unit", "plain", "two"):
        z = z0.clone().requires_grad_(True)
        loss = TF.cross_entropy(z, lab)
        if how == "unit":
            TF.backward(loss)
        elif how == "plain":
            loss.backward()
        else:
            loss.backward(torch.full((), 2.0, device=gpu))
        grads.append(z.grad)
    assert torch.equal(grads[0], grads[1])
    assert torch.equal(grads[2], 2 * grads[1])
    zr = z0.double().cpu().requires_grad_(True)
    F.cross_entropy(zr, lab.cpu()).backward()
    _close(grads[0], zr.grad, 1e-6, 1e-6)


def test_sgd(gpu):
    ps = [torch.randn(n, device=gpu) for n in (7, 1000, 33)]
    gs = [torch.randn_like(p) for p in ps]
    ref = [p - 0.1 * g for p, g in zip(ps, gs)]
    _ops().sgd_step_(ps, gs, [], 0.1, 0.0, 0.0, 0.0, False, False)
    for a, b in zip(ps, ref):
        _close(a, b, 1e-6, 1e-7)
    ms = [torch.zeros_like(p) for p in ps]
    p2 = [p.clone() for p in ps]
    _ops().sgd_step_(ps, gs, ms, 0.1, 0.01, 0.9, 0.0, False, True)
    tp = [p.cpu().clone().requires_grad_(False) for p in p2]
    opt = torch.optim.SGD(tp, lr=0.1, momentum=0.9, weight_decay=0.01)
    for t, g in zip(tp, gs):
        t.grad = g.cpu()
    opt.step()
    for a, b in zip(ps, tp):
        _close(a, b, 1e-6, 1e-6)


@pytest.mark.parametrize("hw,HW", [(28, (300, 301)), (28, (301, 300)), (70, (300, 300)), (70, (37, 301))])
def test_upsample(gpu, hw, HW):
    # 28^2: the whole-source kernel (8 rows per workgroup); 70^2 > 4096 px: one row per workgroup
    src = torch.randint(0, 256, (3, hw, hw), dtype=torch.uint8, device=gpu)
    y = _ops().upsample_bilinear_u8(src, *HW)
    lv = _ops().upsample_bilinear_u8(src, *HW, True)
    assert torch.equal(lv.float() * torch.tensor(1.0 / 255.0, dtype=torch.float32), y)
    ref = F.interpolate(src.float().unsqueeze(1).cpu().double(), size=HW, mode="bilinear",
                        align_corners=False).round().clamp(0, 255) / 255.0
    # bilinear weights in fp32 vs fp64 may round a half differently: <= 1 LSB
    assert (y.double().cpu() - ref).abs().max().item() <= 1.0 / 255 + 1e-6
    assert ((y.double().cpu() - ref).abs() > 1e-6).float().mean().item() < 5e-3


@pytest.mark.parametrize("n", [1, 2047, 2048, 100_003, 3 * 2048 * 5, 20_000_003])
def test_zs_encode_decode_matches_reference(gpu, n):
    """Zero-suppressed fc-row codec (csrc/kernels/zs_exchange.hip) vs the torch reference of
    parallel/zs.py: identical meta and values, a bitwise round trip, -0.0 and NaN kept, values
    past the capacity dropped (count still exact)."""
    from torch_distributed_sandbox_amd.parallel import zs

    torch.manual_seed(n % 97)
    x = torch.relu(torch.randn(n, device=gpu))
    x[::9] = -0.0
    if n > 10:
        x[3] = float("nan")
    meta = torch.empty(zs.meta_numel(n), dtype=torch.int32, device=gpu)
    vals = torch.empty(n, device=gpu)
    nnz = zs.encode(x, meta, vals)
    rmeta, rvals, rnnz = zs.encode_ref(x.cpu())
    assert int(nnz) == rnnz
    assert torch.equal(meta.cpu(), rmeta)
    assert torch.equal(vals[:rnnz].cpu().view(torch.int32), rvals.view(torch.int32))
    out = torch.full((n,), 3.0, device=gpu)
    zs.decode(meta, vals[:max(1, rnnz)], out)
    assert torch.equal(out.view(torch.int32), x.view(torch.int32))
    if rnnz > 8:  # capacity below the count: the count stays exact, the extra values are dropped
        small = torch.full((rnnz // 2,), -1.0, device=gpu)
        assert int(zs.encode(x, meta, small)) == rnnz
        assert torch.equal(small.cpu().view(torch.int32), rvals[:rnnz // 2].view(torch.int32))


@pytest.mark.parametrize("K", [10_004, 4096])
def test_linear_dw_zs_matches_dense(gpu, K):
    """The exchange's dW formation straight from the all-gathered zero-suppressed rows
    (linear_dw_zs: decoded in registers) is bitwise the dense linear_dw on the decoded rows --
    gradient mode (with the bias) and the update-only step -- and matches fp64.  K = 10 004: a
    partial last 1024-column block, rows crossing pages."""
    from torch_distributed_sandbox_amd.parallel import zs

    torch.manual_seed(K)
    W, rows, N = 3, 2, 10
    xs = torch.relu(torch.randn(W, rows, K, device=gpu))
    xs[:, :, ::7] = -0.0
    n = rows * K
    M = zs.meta_numel(n)
    enc = [zs.encode_ref(xs[r].cpu()) for r in range(W)]
    cap = max(e[2] for e in enc)
    meta_all = torch.zeros(W, M + 2, dtype=torch.int32, device=gpu)
    vals_all = torch.zeros(W, cap, device=gpu)
    for r, (mt, vl, nz) in enumerate(enc):
        meta_all[r, :M] = mt.to(gpu)
        vals_all[r, :nz] = vl.to(gpu)
    dy = torch.randn(W * rows, N, device=gpu)
    x_rows = xs.reshape(W * rows, K).contiguous()
    ops = _ops()
    dw, db = torch.empty(N, K, device=gpu), torch.empty(N, device=gpu)
    ops.linear_dw_zs(dy, meta_all, vals_all, rows, dw, db, 0.5, False)
    dw_ref, db_ref = torch.empty_like(dw), torch.empty_like(db)
    ops.linear_dw(dy, x_rows, dw_ref, db_ref, 0.5, False)
    assert torch.equal(dw, dw_ref) and torch.equal(db, db_ref)
    ref = 0.5 * dy.double().t() @ x_rows.double()
    _check_rel(dw, ref, 1e-6)
    # update-only step (the exchange's optimizer-in-backward): W -= lr * scale * dyᵀX
    w0 = torch.randn(N, K, device=gpu)
    w1, w2 = w0.clone(), w0.clone()
    ops.linear_dw_zs(dy, meta_all, vals_all, rows, w1, None, 0.5, False, 0.1)
    ops.linear_dw(dy, x_rows, w2, None, 0.5, False, 0.1)
    assert torch.equal(w1, w2)
    _check_rel(w1, w0.double() - 0.1 * ref, 1e-6)


def _check_rel(a, ref, tol):
    a, ref = a.double().cpu(), ref.double().cpu()
    e = (a - ref).abs().max().item()
    assert e <= tol * max(ref.abs().max().item(), 1e-30), e


def test_zs_segmented_codec_matches_reference(gpu):
    """Segmented codec of the sharded exchange (zs_seg_* kernels) vs the torch reference:
    (destination shard, row) segments of uneven length, an empty one, capacity slots."""
    from torch_distributed_sandbox_amd.parallel import zs

    torch.manual_seed(4)
    B, K = 3, 9000
    x = torch.relu(torch.randn(B, K, device=gpu))
    bounds = [(0, 2560), (2560, 2560), (2560, 6400), (6400, 9000)]  # one empty shard
    segs = [(b * K + a, e - a) for (a, e) in bounds for b in range(B)]
    cap = 2100
    lay_g, lay_c = zs.SegLayout(segs, gpu), zs.SegLayout(segs, "cpu")
    meta = torch.empty(lay_g.meta_numel, dtype=torch.int32, device=gpu)
    vals = torch.empty(lay_g.nseg * cap, device=gpu)
    cnt = zs.seg_encode(x, lay_g, meta, vals, cap)
    rmeta = torch.empty(lay_c.meta_numel, dtype=torch.int32)
    rvals = torch.zeros(lay_c.nseg * cap)
    rcnt = zs.seg_encode(x.cpu(), lay_c, rmeta, rvals, cap)
    assert torch.equal(cnt.cpu(), rcnt) and torch.equal(meta.cpu(), rmeta)
    out = torch.full((B, K), 9.0, device=gpu)
    zs.seg_decode(meta, lay_g, vals, cap, out)
    assert torch.equal(out, x)
