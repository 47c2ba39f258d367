"""Native RCCL communicator + C++ reducer on a real GPU (world size 1 on the
one-GPU box; the multi-rank logic is covered on CPU by the host ring backend,
which drives the same C++ reducer)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg(gpu):
    from torch_distributed_sandbox_amd.parallel import distributed as dist
    from torch_distributed_sandbox_amd.parallel import launch

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = launch.find_free_port()
    dist.init_process_group("rccl-native", rank=0, world_size=1)
    yield dist
    dist.destroy_process_group()


def test_rccl_native_collectives(pg, gpu):
    import torch.distributed as tdist

    assert tdist.get_backend() == "tds_rccl"
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        # producer work queued on a side stream right before the collective: the
        # comm stream must wait for it (event fence), and the consumer for the comm
        x = torch.arange(1 << 20, device=gpu, dtype=torch.float32)
        x.mul_(2)
        w = pg.all_reduce(x, pg.ReduceOp.AVG, async_op=True)
        w.wait()
        y = x + 1
    torch.cuda.synchronize()
    assert torch.equal(y, torch.arange(1 << 20, device=gpu, dtype=torch.float32) * 2 + 1)
    for dt in (torch.float32, torch.bfloat16, torch.float16, torch.int32, torch.int64, torch.float64):
        t = torch.ones(1000, dtype=dt, device=gpu)
        pg.all_reduce(t)
        assert (t == 1).all(), dt
    t = torch.tensor([3.0], device=gpu)
    pg.all_reduce(t, pg.ReduceOp.MAX)
    assert t.item() == 3.0
    b = torch.arange(10.0, device=gpu)
    pg.broadcast(b, 0)
    assert torch.equal(b, torch.arange(10.0, device=gpu))
    out = torch.empty(7, device=gpu)
    pg.all_gather_into_tensor(out, torch.arange(7.0, device=gpu))
    assert torch.equal(out, torch.arange(7.0, device=gpu))
    rs = torch.empty(5, device=gpu)
    pg.reduce_scatter_tensor(rs, torch.arange(5.0, device=gpu))
    assert torch.equal(rs, torch.arange(5.0, device=gpu))
    a = torch.arange(6.0, device=gpu)
    o = torch.empty_like(a)
    tdist.all_to_all_single(o, a)
    assert torch.equal(o, a)
    lst = [torch.empty(3, device=gpu)]
    pg.all_gather(lst, torch.ones(3, device=gpu))
    assert (lst[0] == 1).all()
    pg.barrier()


def test_rccl_native_coalesced_broadcast(pg, gpu):
    from torch_distributed_sandbox_amd.parallel.rccl_backend import native_comm_of
    import torch.distributed as tdist

    comm, kind = native_comm_of(tdist.group.WORLD)
    assert kind == "rccl"
    ts = [torch.full((5,), 2.0, device=gpu), torch.tensor([7], dtype=torch.int64, device=gpu)]
    comm.broadcast_coalesced(ts, 0).wait()
    torch.cuda.synchronize()
    assert ts[0][0].item() == 2.0 and ts[1].item() == 7
    assert comm.pending() >= 0


def test_native_reducer_ddp_on_rccl(pg, gpu):
    """DDP on the native RCCL PG uses the C++ reducer; grads land in the flat buffer
    and equal the plain single-process gradients (world 1)."""
    import copy

    from torch_distributed_sandbox_amd.models import ConvNet
    from torch_distributed_sandbox_amd.ops import SGD, CrossEntropyLoss
    from torch_distributed_sandbox_amd.parallel import DistributedDataParallel

    torch.manual_seed(0)
    m = ConvNet(image_shape=(64, 64), device=gpu)
    ref = copy.deepcopy(m)
    ddp = DistributedDataParallel(m)
    assert ddp.reducer_kind == "native"
    opt = ddp.attach_optimizer(SGD(m.parameters(), 0.1))
    x = torch.rand(3, 1, 64, 64, device=gpu)
    y = torch.tensor([1, 2, 3], device=gpu)
    for _ in range(2):
        loss = CrossEntropyLoss()(ddp(x), y)
        opt.zero_grad()
        loss.backward()
        for p in m.parameters():
            assert p.grad.untyped_storage().data_ptr() == ddp.flat_grad.untyped_storage().data_ptr()
        ref.zero_grad()
        CrossEntropyLoss()(ref(x), y).backward()
        for (n, p), q in zip(m.named_parameters(), ref.parameters()):
            rel = ((p.grad - q.grad).norm() / q.grad.norm().clamp_min(1e-30)).item()
            assert rel < 1e-4 or n.endswith("0.bias"), (n, rel)
        opt.step()
        with torch.no_grad():
            for p, q in zip(m.parameters(), ref.parameters()):
                q.copy_(p)
    assert ddp._native.ready_order()[0] == 0  # the fc bucket is reduced first


def test_linear_dw_kernel(gpu):
    import torch_distributed_sandbox_amd as tds

    torch.manual_seed(0)
    for M, N, K in ((10, 10, 100_003), (15, 10, 4096), (40, 16, 777), (1, 3, 33)):
        dy = torch.randn(M, N, device=gpu)
        x = torch.randn(M, K, device=gpu)
        dw = torch.empty(N, K, device=gpu)
        db = torch.empty(N, device=gpu)
        tds._ext.ops().linear_dw(dy, x, dw, db, 0.5, False)
        ref = (dy.double().t() @ x.double()) * 0.5
        assert ((dw.double() - ref).abs().max() / ref.abs().max()).item() < 1e-6, (M, N, K)
        assert torch.allclose(db.double(), dy.double().sum(0) * 0.5, rtol=1e-6, atol=1e-6)
        tds._ext.ops().linear_dw(dy, x, dw, db, 0.5, True)  # accumulate
        assert ((dw.double() - 2 * ref).abs().max() / ref.abs().max()).item() < 1e-6
    # column shard written in place into a wider matrix (row stride > K), > 64 rows in passes
    dy = torch.randn(100, 10, device=gpu)
    x = torch.randn(100, 3000, device=gpu)
    full = torch.full((10, 9000), 7.0, device=gpu)
    tds._ext.ops().linear_dw(dy, x, full[:, 3000:6000], None, 0.25, False)
    ref = (dy.double().t() @ x.double()) * 0.25
    assert ((full[:, 3000:6000].double() - ref).abs().max() / ref.abs().max()).item() < 1e-6
    assert (full[:, :3000] == 7).all() and (full[:, 6000:] == 7).all()


@pytest.mark.parametrize("mode,source", [("activations", "pooled"), ("activations", "rows"), ("sharded", "pooled"),
                                         ("chunked", "pooled")])
def test_activation_exchange_fused_convnet(pg, gpu, mode, source):
    """Forced activation exchange at world size 1 runs the whole GPU path (the pooled input and the
    head constants gathered, or the head forward writing the fc input rows; head backward without
    dW; dW into the bucket) and must reproduce the plain fused gradients."""
    import copy

    from torch_distributed_sandbox_amd.models import ConvNet
    from torch_distributed_sandbox_amd.ops import SGD, CrossEntropyLoss
    from torch_distributed_sandbox_amd.parallel import DistributedDataParallel

    torch.manual_seed(0)
    H = 256  # fc: 10 x 131072 (exchange candidate)
    m = ConvNet(image_shape=(H, H), device=gpu, mode="fused")
    ref = copy.deepcopy(m)
    ddp = DistributedDataParallel(m, grad_exchange=mode, exchange_source=source)
    assert len(ddp.exchanges) == 1
    opt = ddp.attach_optimizer(SGD(m.parameters(), 0.01))
    x = torch.rand(3, 1, H, H, device=gpu)
    y = torch.tensor([1, 2, 3], device=gpu)
    for step in range(2):
        loss = CrossEntropyLoss()(ddp(x), y)
        opt.zero_grad()
        loss.backward()
        ref.zero_grad()
        CrossEntropyLoss()(ref(x), y).backward()
        for (n, p), q in zip(m.named_parameters(), ref.parameters()):
            if n.endswith("0.bias"):
                continue
            rel = ((p.grad - q.grad).norm() / q.grad.norm().clamp_min(1e-30)).item()
            assert rel < 1e-5, (step, n, rel)
        assert m.fc.weight.grad.data_ptr() == ddp.grad_view(m.fc.weight).data_ptr()
        opt.step()
        with torch.no_grad():
            for p, q in zip(m.parameters(), ref.parameters()):
                q.copy_(p)
    assert ddp.exchanges[0].steps_exchanged == 2
    if mode == "activations":
        assert ddp.fc_grad_path() == ("activation-exchange(pooled)" if source == "pooled" else
                                      "activation-exchange(zs)")


@pytest.mark.parametrize("exchange,fuse", [("allreduce", False), ("activations", False), ("sharded", False),
                                           ("chunked", False), ("activations:rows", False),
                                           ("allreduce", True), ("activations", True), ("sharded", True),
                                           ("activations:rows", True)])
def test_overlap_optimizer_matches_sequential(pg, gpu, exchange, fuse):
    """overlap_optimizer: the fc bucket's collective + SGD update run on a side stream
    and the next forward's head waits on a parameter fence; the trajectory must be
    identical to the sequential step.  fuse=True: at world size 1 the fc weight's SGD
    step runs inside the head backward kernel, or with an exchange forced inside the
    exchange's dW formation (update-only linear_dw; ops/fused_update.py)."""
    import copy

    from torch_distributed_sandbox_amd.models import ConvNet
    from torch_distributed_sandbox_amd.ops import SGD, CrossEntropyLoss, param_fence
    from torch_distributed_sandbox_amd.parallel import DistributedDataParallel

    exchange, _, source = exchange.partition(":")
    source = source or "pooled"  # activations: the pooled input (default) or the zero-suppressed rows
    zs_path = exchange == "sharded" or (exchange == "activations" and source == "rows")
    torch.manual_seed(0)
    H = 256
    m1 = ConvNet(image_shape=(H, H), device=gpu, mode="fused")
    m2 = copy.deepcopy(m1)
    d1 = DistributedDataParallel(m1, grad_exchange=exchange, overlap_optimizer=True, fuse_update_in_backward=fuse,
                                 exchange_source=source)
    d2 = DistributedDataParallel(m2, grad_exchange=exchange, exchange_source=source)
    assert d1.overlap_optimizer and len(d1._deferred) == 1
    o1 = d1.attach_optimizer(SGD(m1.parameters(), 1e-4))
    o2 = d2.attach_optimizer(SGD(m2.parameters(), 1e-4))
    crit = CrossEntropyLoss()
    g = torch.Generator(device=gpu).manual_seed(5)
    for step in range(4):
        x = torch.rand(3, 1, H, H, device=gpu, generator=g)
        y = torch.randint(0, 10, (3,), device=gpu, generator=g)
        if step == 2 and d1.exchanges:  # a capacity below this step's counts: the dense re-send path
            d1.exchanges[0].force_capacity_once(1)
        for d, o in ((d1, o1), (d2, o2)):
            loss = crit(d(x), y)
            o.zero_grad()
            loss.backward()
            o.step()
        # a side-stream update fences the weight for the next forward -- unless everything left
        # of the fc bucket (the bias, the weight stepped in its backward) was stepped inline by the
        # optimizer's own sweep (world size 1, nothing to wait for: ddp.py take_inline_deferred)
        assert param_fence.pending(m1.fc.weight) or d1.last_deferred_inline
        if fuse and exchange == "allreduce":
            assert d1.last_deferred_inline and not param_fence.pending(m1.fc.bias)
        if step == 0 and zs_path:
            assert d1.fc_grad_path().endswith("(zs)")  # tagged on the first step (its count check is deferred)
        elif step == 0 and exchange == "activations":
            assert d1.fc_grad_path().endswith("(pooled)")
        if fuse:
            assert not d1._fused_done  # consumed by the step: the bias was updated, the weight skipped
    d1.wait_pending_updates()
    torch.cuda.synchronize()
    if zs_path:
        assert d1.exchanges[0].zs_stats["overflows"] >= 1  # step 2 went through the dense re-send
    for (n, p), q in zip(m1.named_parameters(), m2.parameters()):
        if fuse:  # same arithmetic (p - lr*g) in another kernel: equal up to fma contraction
            assert torch.allclose(p, q, rtol=1e-6, atol=1e-9), n
        else:
            assert torch.equal(p, q), n


@pytest.mark.parametrize("keep", [False, True])
def test_fused_update_grad_semantics(pg, gpu, keep):
    """World-1 fc SGD step inside the head backward: by default the weight's gradient is never
    materialised (.grad None after backward, torch's optimizer-in-backward semantics, update-only
    kernel); keep_fused_grads=True also writes it.  Either way the update equals p - lr * g of
    an unfused twin."""
    import copy

    from torch_distributed_sandbox_amd.models import ConvNet
    from torch_distributed_sandbox_amd.ops import SGD, CrossEntropyLoss
    from torch_distributed_sandbox_amd.parallel import DistributedDataParallel

    torch.manual_seed(0)
    H = 256  # fc weight >= 1 Mi elements: a deferred (overlapped) bucket
    m1 = ConvNet(image_shape=(H, H), device=gpu, mode="fused")
    m2 = copy.deepcopy(m1)
    d1 = DistributedDataParallel(m1, overlap_optimizer=True, keep_fused_grads=keep)
    assert d1._deferred
    d2 = DistributedDataParallel(m2)
    o1 = d1.attach_optimizer(SGD(m1.parameters(), 1e-3))
    o2 = d2.attach_optimizer(SGD(m2.parameters(), 1e-3))
    crit = CrossEntropyLoss()
    x = torch.rand(2, 1, H, H, device=gpu)
    y = torch.tensor([3, 7], device=gpu)
    for d, o in ((d1, o1), (d2, o2)):
        o.zero_grad()
        crit(d(x), y).backward()
    if keep:
        torch.testing.assert_close(m1.fc.weight.grad, m2.fc.weight.grad, rtol=1e-5, atol=1e-9)
    else:
        assert m1.fc.weight.grad is None
    assert m1.fc.bias.grad is not None
    o1.step()
    o2.step()
    d1.wait_pending_updates()
    torch.cuda.synchronize()
    for (n, p), q in zip(m1.named_parameters(), m2.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-6, atol=1e-9, msg=n)


def test_rccl_native_count_and_sendrecv(pg, gpu):
    """ncclCommCount of the live communicator, and the grouped point-to-point
    primitive (self-exchange at world 1; strided row slices as sources)."""
    from torch_distributed_sandbox_amd.parallel.rccl_backend import native_comm_of
    import torch.distributed as tdist

    comm, _ = native_comm_of(tdist.group.WORLD)
    assert comm.comm_count() == 1
    x = torch.arange(40.0, device=gpu).view(4, 10)
    out = torch.zeros(4, 3, device=gpu)
    sends = [x[b, 2:5] for b in range(4)]
    recvs = [out[b] for b in range(4)]
    comm.sendrecv(sends, [0] * 4, recvs, [0] * 4).wait()
    torch.cuda.synchronize()
    assert torch.equal(out, x[:, 2:5])


def test_cu_reserve_and_masked_stream(gpu):
    """utils/streams.py: a CU-masked compute stream with 32 CUs left to communication kernels;
    the persistent kernels size their grids to the remaining CUs and the step matches the
    full-chip one (summation order of the per-workgroup partials differs)."""
    import copy

    from torch_distributed_sandbox_amd.models import ConvNet
    from torch_distributed_sandbox_amd.ops import CrossEntropyLoss
    from torch_distributed_sandbox_amd import _ext
    from torch_distributed_sandbox_amd.utils.streams import comm_stream, compute_cus, reserve_cus_for_comm

    torch.manual_seed(0)
    H = 128
    m1 = ConvNet(image_shape=(H, H), device=gpu, mode="fused")
    m2 = copy.deepcopy(m1)
    x = torch.rand(2, 1, H, H, device=gpu)
    y = torch.tensor([1, 8], device=gpu)
    full = compute_cus()
    CrossEntropyLoss()(m1(x), y).backward()
    try:
        with pytest.raises(ValueError):
            reserve_cus_for_comm(16, gpu)
        assert comm_stream(gpu) is None
        s = reserve_cus_for_comm(32, gpu)
        assert compute_cus() == full - 32
        cs = comm_stream(gpu)
        # the two sides of the split land on disjoint CUs: 4 per XCC on the comm side
        with torch.cuda.stream(cs):
            where_c = _ext.ops().cu_probe(x, 50, 512).cpu()
        with torch.cuda.stream(s):
            where_s = _ext.ops().cu_probe(x, 50, 2048).cpu()
        torch.cuda.synchronize()
        cu_c = {(a, (b >> 8) & 0xFF) for a, b in where_c.tolist()}
        cu_s = {(a, (b >> 8) & 0xFF) for a, b in where_s.tolist()}
        assert not cu_c & cu_s
        assert len(cu_c) == 32 and len(cu_s) == full - 32
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            CrossEntropyLoss()(m2(x), y).backward()
        torch.cuda.current_stream().wait_stream(s)
    finally:
        reserve_cus_for_comm(0)
    assert compute_cus() == full
    torch.cuda.synchronize()
    for (n, p), q in zip(m1.named_parameters(), m2.parameters()):
        if n.endswith("0.bias"):
            continue
        torch.testing.assert_close(q.grad, p.grad, rtol=1e-4, atol=1e-7, msg=n)


_RELEASE_SCRIPT = r"""
import torch
from torch_distributed_sandbox_amd.models import ConvNet
from torch_distributed_sandbox_amd.ops import CrossEntropyLoss
from torch_distributed_sandbox_amd.utils.streams import (comm_stream, compute_cus, release_streams,
                                                         reserve_cus_for_comm)
dev = torch.device("cuda", 0)
full = compute_cus()
torch.manual_seed(0)
m = ConvNet(image_shape=(64, 64), device=dev, mode="fused")
x = torch.rand(2, 1, 64, 64, device=dev)
y = torch.tensor([3, 5], device=dev)
torch.cuda.set_stream(reserve_cus_for_comm(32, dev))
assert comm_stream(dev) is not None and compute_cus() == full - 32
CrossEntropyLoss()(m(x), y).backward()
n = release_streams()
assert n == 2, n  # the compute stream and the comm side
assert compute_cus() == full and comm_stream(dev) is None
assert torch.cuda.current_stream() == torch.cuda.default_stream()
CrossEntropyLoss()(m(x), y).backward()  # the default stream works on
torch.cuda.synchronize()
print("release ok")
"""


def test_release_masked_streams(gpu):
    """utils/streams.release_streams: the CU-masked streams are destroyed at the end of a run
    (not left to process exit, where their teardown races rocprofv3's finalization); the
    reserve returns to 0 and the default stream carries on.  In a child process: the streams
    of this one stay untouched."""
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _RELEASE_SCRIPT], cwd=repo, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0 and "release ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


def test_loss_in_head_with_activation_exchange(pg, gpu):
    """The activation exchange's head forward (writing X rows) also forms the loss when the labels
    come with the batch: same losses and parameters over two steps as without them."""
    import copy

    from torch_distributed_sandbox_amd.models import ConvNet, convnet_fused
    from torch_distributed_sandbox_amd.ops import SGD, CrossEntropyLoss
    from torch_distributed_sandbox_amd.parallel import DistributedDataParallel

    torch.manual_seed(0)
    H = 128
    m1 = ConvNet(image_shape=(H, H), device=gpu, mode="fused")
    m2 = copy.deepcopy(m1)
    d1 = DistributedDataParallel(m1, grad_exchange="activations")
    d2 = DistributedDataParallel(m2, grad_exchange="activations")
    o1 = d1.attach_optimizer(SGD(m1.parameters(), 1e-3))
    o2 = d2.attach_optimizer(SGD(m2.parameters(), 1e-3))
    crit = CrossEntropyLoss()
    g = torch.Generator(device=gpu).manual_seed(7)
    before = convnet_fused.STATS["head_fused_ce"]
    for _ in range(2):
        x = torch.rand(3, 1, H, H, device=gpu, generator=g)
        y = torch.randint(0, 10, (3,), device=gpu, generator=g)
        x2 = x.clone()
        convnet_fused.attach_labels(x2, y)
        losses = []
        for d, o, xi in ((d1, o1, x), (d2, o2, x2)):
            loss = crit(d(xi), y)
            o.zero_grad()
            loss.backward()
            o.step()
            losses.append(loss)
        assert torch.equal(losses[0], losses[1])
    d1.wait_pending_updates()
    d2.wait_pending_updates()
    torch.cuda.synchronize()
    assert convnet_fused.STATS["head_fused_ce"] >= before + 2
    for p1, p2 in zip(m1.parameters(), m2.parameters()):
        assert torch.equal(p1, p2)
