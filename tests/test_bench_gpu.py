"""bench.py on the GPU box: the 1-GPU headline path at a small image size, and the
self-spawned multi-rank path rehearsed with gloo ranks sharing cuda:0 (the only
multi-rank GPU run a one-GPU box allows; RCCL refuses two ranks on one device)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, timeout=240):
    # a fresh rendezvous for the child: a MASTER_PORT left in this process's environment by another
    # test's process group (tests/test_comm_gpu.py) is still bound by that group's store
    env = {k: v for k, v in os.environ.items() if k not in ("MASTER_PORT", "MASTER_ADDR", "RANK", "WORLD_SIZE",
                                                             "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    p = subprocess.run([sys.executable, "bench.py"] + args, cwd=ROOT, capture_output=True, text=True,
                       timeout=timeout, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    recs = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(recs) == 1, p.stdout
    return recs[0]


@pytest.mark.parametrize("prefetch", [False, True])
def test_bench_one_gpu_small(gpu, prefetch):
    r = _bench(["--image-size", "512", "--steps", "3", "--warmup", "1",
                "--prefetch" if prefetch else "--no-prefetch"])
    assert r["n_gpus"] == 1 and r["config"]["fc_grad"] == "local" and r["value"] > 0
    assert r["config"]["prefetch"] is prefetch
    assert r["config"]["input_moments"] == "upsample" and r["config"]["loss_in_head"] is True


@pytest.mark.parametrize("exchange", ["auto", "allreduce"])
def test_bench_self_spawn_shared_device(gpu, exchange):
    r = _bench(["--gpus", "2", "--backend", "gloo", "--shared-device", "--image-size", "512", "--steps", "2",
                "--warmup", "1", "--grad-exchange", exchange])
    assert r["n_gpus"] == 2 and r["config"]["shared_device"] is True
    assert r["config"]["parallelism"] == "dp2" and r["config"]["global_batch"] == 10


@pytest.mark.parametrize("exchange", ["activations", "activations:rows", "sharded"])
def test_bench_preflight_rccl_native_cu_split(gpu, exchange):
    """The multi-GPU default stack's preflight, at world 1 on the real communicator: rccl-native
    with 32 CUs split off (the comm stream confined to them, maxCTAs 32) and the fc exchange
    forced, so every collective the exchange uses runs once with a bounded wait before the
    warmup and reports its time."""
    exchange, _, source = exchange.partition(":")
    r = _bench(["--image-size", "1000", "--steps", "2", "--warmup", "1", "--backend", "rccl-native",
                "--reserve-cus", "32", "--grad-exchange", exchange, "--exchange-source", source or "pooled"])
    c = r["config"]
    assert c["reserve_cus"] == 32 and c["rccl_max_ctas"] == 32 and c["tier"] == "1/1"
    pf = c["preflight"]
    assert pf["fc_path"] == exchange
    ops = [x["op"] for x in pf["collectives"]]
    if exchange == "activations" and source == "rows":
        assert ops[:3] == ["zs records all-gather (int32)", "zs values all-gather (first-step capacity)",
                           "dY all-gather"]
    elif exchange == "activations":  # the pooled source (parallel/factored.py): head records, then ya
        assert ops[:3] == ["head record all-gather", "pooled input (ya) all-gather (fp16)", "dY all-gather"]
        assert c["fc_grad"] == "activation-exchange(pooled)"
    else:
        assert "zs segment counts all-gather (int64)" in ops and "updated W shard exchange (per peer)" in ops
    assert ops[-1] == "barrier" and all(x["ms"] > 0 for x in pf["collectives"])
