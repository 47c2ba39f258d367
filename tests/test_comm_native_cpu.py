"""CPU tests of the native comm stack: the C++ TCP rendezvous store
(parallel/store.py) and the C++ ring host backend (parallel/host_backend.py)."""
import datetime
import math
import os
import threading
import time

import pytest
import torch

from torch_distributed_sandbox_amd.parallel import launch


def _store(port, world=1, server=True, timeout_s=5):
    from torch_distributed_sandbox_amd.parallel.store import NativeStore

    return NativeStore("127.0.0.1", port, world, server, datetime.timedelta(seconds=timeout_s))


def test_store_single_process_ops():
    s = _store(0)
    c = _store(s.port, server=False)
    s.set("a", b"hello")
    assert c.get("a") == b"hello"
    assert c.add("cnt", 3) == 3 and s.add("cnt", 4) == 7
    assert s.check(["a", "cnt"]) and not s.check(["nope"])
    assert c.num_keys() == 2
    # compare-and-set: mismatch returns current value, match swaps
    assert c.compare_set("a", b"zzz", b"x") == b"hello"
    assert c.compare_set("a", b"hello", b"world") == b"world"
    assert s.get("a") == b"world"
    assert c.delete_key("a") and not c.delete_key("a")
    # blocking get is released by a set from another client
    t = threading.Thread(target=lambda: (time.sleep(0.3), s.set("late", b"v")))
    t.start()
    assert c.get("late") == b"v"
    t.join()
    c.wait(["late"])
    with pytest.raises(RuntimeError):
        c.wait(["never"], datetime.timedelta(milliseconds=300))


def test_store_timed_out_wait_does_not_desync():
    """A WAIT that timed out stays registered on the server until its key appears; the late reply
    must not be read as the answer to the client's next request (the client reconnects)."""
    s = _store(0)
    c = _store(s.port, server=False)
    with pytest.raises(RuntimeError):
        c.wait(["late_key"], datetime.timedelta(milliseconds=200))
    s.set("late_key", b"")  # the server answers the stale WAIT now
    s.set("other", b"value")
    time.sleep(0.1)
    assert c.get("other") == b"value"
    assert c.add("n", 2) == 2 and c.get("late_key") == b""


def test_store_client_fails_fast_when_server_is_gone():
    """A client whose server exited (rank 0 at teardown or after a crash) must fail at once --
    not retry a connect for its whole timeout (here 60 s) -- on a plain request, on a WAIT that
    was blocked when the server went away, and on every later call."""
    s = _store(0, timeout_s=60)
    c = _store(s.port, server=False, timeout_s=60)
    s.set("k", b"v")
    assert c.get("k") == b"v"
    err = []

    def blocked_wait():
        try:
            c.wait(["never"], datetime.timedelta(seconds=60))
        except RuntimeError as e:
            err.append((time.monotonic(), str(e)))

    t = threading.Thread(target=blocked_wait)
    t.start()
    time.sleep(0.3)
    t_stop = time.monotonic()
    del s  # rank 0's store object: its server thread stops and closes every connection
    t.join(timeout=10)
    assert not t.is_alive() and err, "the blocked WAIT did not fail when the server went away"
    assert err[0][0] - t_stop < 5 and "lost" in err[0][1], err
    for op in (lambda: c.get("k"), lambda: c.set("a", b"b"), lambda: c.add("n", 1)):
        t0 = time.monotonic()
        with pytest.raises(RuntimeError, match="lost"):
            op()
        assert time.monotonic() - t0 < 5


def _w_store_8rank_traffic(rank, world, port, out_dir):
    """The rendezvous traffic of a real job through the default (native) store: the process
    group's init, the RCCL communicator's ncclUniqueId exchange (the real ncclGetUniqueId bytes,
    rccl_backend.exchange_unique_id), and the reference's per-step new_group -- 1000 calls
    (mnist_distributed.py:99-100) -- plus real subgroup creations and collectives on them."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.pop("TDS_STORE", None)
    from torch_distributed_sandbox_amd.parallel import distributed as dist
    from torch_distributed_sandbox_amd.parallel.rccl_backend import exchange_unique_id

    dist.init_process_group("gloo", rank=rank, world_size=world)
    assert dist.store_kind() == "native", dist.store_kind()
    store = dist._state["store"]
    uids = [bytes(exchange_unique_id(store, rank, key=f"uid/{i}").numpy().tobytes()) for i in range(8)]
    assert all(len(u) == 128 for u in uids) and len(set(uids)) == 8
    with open(os.path.join(out_dir, f"uid{rank}"), "wb") as f:
        f.write(b"".join(uids))
    g0 = None
    for step in range(1000):
        g = dist.new_group(list(range(world)))
        g0 = g if g0 is None else g0
        assert g is g0
    subs = [list(range(k)) for k in range(2, world + 1)] + [[r, (r + 1) % world] for r in range(world)]
    for ranks in subs:
        g = dist.new_group(ranks)
        if rank in ranks:
            t = torch.tensor([float(rank)])
            dist.all_reduce(t, group=g)
            assert t.item() == float(sum(ranks))
    dist.barrier()
    dist.destroy_process_group()


def test_native_store_carries_8_rank_rendezvous(tmp_path):
    launch.spawn(_w_store_8rank_traffic, args=(8, launch.find_free_port(), str(tmp_path)), nprocs=8, timeout=240)
    blobs = {open(tmp_path / f"uid{r}", "rb").read() for r in range(8)}
    assert len(blobs) == 1  # every rank got rank 0's ids


def test_rendezvous_falls_back_to_c10d_on_every_rank():
    """A native store rank 0 cannot create: every rank ends up on c10d's store and says why."""
    from torch_distributed_sandbox_amd.parallel import store as S

    class _Broken:
        def __init__(self, *a, **k):
            raise RuntimeError("no native store here")

    real = S.NativeStore
    S.NativeStore = _Broken
    try:
        st, kind = S.rendezvous(0, 1, port=launch.find_free_port(), timeout=datetime.timedelta(seconds=10))
    finally:
        S.NativeStore = real
    assert kind.startswith("c10d (fallback: rank 0: RuntimeError: no native store here")
    st.set("k", "v")
    assert st.get("k") == b"v"


def _w_store_rdzv(rank, world, port, backend):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from torch_distributed_sandbox_amd.parallel import distributed as dist

    dist.init_process_group(backend, rank=rank, world_size=world, store="native")
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t)
    assert t.item() == world * (world + 1) / 2
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("backend", ["gloo", "host"])
def test_native_store_rendezvous(backend):
    launch.spawn(_w_store_rdzv, args=(3, launch.find_free_port(), backend), nprocs=3, timeout=120)


def _w_host_sweep(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as tdist

    from torch_distributed_sandbox_amd.parallel import distributed as dist

    dist.init_process_group("host", rank=rank, world_size=world)
    assert tdist.get_backend() == "tds_host"
    # sizes that do not divide by world, and one > the 1 MiB broadcast chunk
    for n in [1, 2, 7, 1000, 600_001]:
        t = torch.arange(n, dtype=torch.float32) + rank
        dist.all_reduce(t)
        assert torch.equal(t, torch.arange(n, dtype=torch.float32) * world + sum(range(world))), n
    for dt in (torch.float64, torch.bfloat16, torch.float16, torch.int64, torch.int32, torch.uint8):
        t = torch.ones(33, dtype=dt)
        dist.all_reduce(t)
        assert (t == world).all(), dt
    t = torch.tensor([rank + 1], dtype=torch.int64)
    dist.all_reduce(t, dist.ReduceOp.PRODUCT)
    assert t.item() == math.factorial(world)
    t = torch.tensor([float(rank)])
    dist.all_reduce(t, dist.ReduceOp.MIN)
    assert t.item() == 0
    b = torch.arange(400_000, dtype=torch.float64) if rank == 1 else torch.zeros(400_000, dtype=torch.float64)
    dist.broadcast(b, 1)
    assert torch.equal(b, torch.arange(400_000, dtype=torch.float64))
    nc = torch.arange(12.0).view(3, 4).t() * (rank + 1)  # non-contiguous: staged
    dist.all_reduce(nc)
    assert torch.equal(nc, torch.arange(12.0).view(3, 4).t() * sum(range(1, world + 1)))
    o = torch.empty(world * 4)
    dist.all_gather_into_tensor(o, torch.full((4,), float(rank)))
    assert torch.equal(o, torch.arange(world).float().repeat_interleave(4))
    inp = torch.arange(world * 6, dtype=torch.float32) * (rank + 1)
    out = torch.empty(6)
    dist.reduce_scatter_tensor(out, inp)
    assert torch.equal(out, torch.arange(rank * 6, rank * 6 + 6).float() * sum(range(1, world + 1)))
    x = torch.arange(world * 2, dtype=torch.float32) + 100 * rank
    y = torch.empty_like(x)
    tdist.all_to_all_single(y, x)
    assert torch.equal(y, torch.cat([torch.arange(rank * 2, rank * 2 + 2).float() + 100 * s for s in range(world)]))
    w = dist.all_reduce(torch.ones(3), dist.ReduceOp.AVG, async_op=True)
    w.wait()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_host_backend_sweep(world):
    launch.spawn(_w_host_sweep, args=(world, launch.find_free_port()), nprocs=world, timeout=180)


def _w_host_timeout(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from torch_distributed_sandbox_amd.parallel import distributed as dist

    dist.init_process_group("host", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=2))
    if rank == 1:
        time.sleep(6)  # never joins the collective
        return
    t0 = time.time()
    with pytest.raises(RuntimeError, match="timed out|closed the ring"):
        dist.all_reduce(torch.ones(4))
    assert time.time() - t0 < 5.5


def test_host_backend_bounded_wait_on_hung_peer():
    launch.spawn(_w_host_timeout, args=(2, launch.find_free_port()), nprocs=2, timeout=60)
