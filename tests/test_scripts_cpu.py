"""The four reference entry points, run end to end on CPU (gloo) at small sizes."""
import json
import os
import re
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=300, env=None):
    e = dict(os.environ)
    e.update(env or {})
    e["CUDA_VISIBLE_DEVICES"] = ""  # CPU rehearsal even on a GPU box
    e["HIP_VISIBLE_DEVICES"] = ""
    p = subprocess.run([sys.executable] + args, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=e)
    return p


def test_allreduce_toy_gloo():
    p = _run(["allreduce_toy.py", "-s", "3", "--backend", "gloo", "--steps", "4"])
    assert p.returncode == 0, p.stderr
    lines = re.findall(r"rank: (\d), step: (\d+), value: (\d+), reduced sum: (\d+)\.", p.stdout)
    assert {r for r, *_ in lines} == {"0", "1"}  # only ranks 0 and 1 print (allreduce_toy.py:35-38)
    steps = {}
    for r, s, v, tot in lines:
        steps.setdefault(s, set()).add(tot)
    assert sorted(steps, key=int) == ["1", "2", "3", "4"]  # --steps honoured
    for s, tots in steps.items():
        assert len(tots) == 1  # every printing rank agrees on the reduced sum
    assert p.stdout.count("--> done setting up rank=") == 3


def test_test_init_script():
    p = _run(["test_init.py"])
    assert p.returncode == 0, p.stderr
    assert p.stdout.count("--> done setting up rank=") == 4
    assert "successful test_setup!" in p.stdout
    assert p.stdout.count("backend='gloo'") == 4


def test_test_init_pytest_collectable():
    sys.path.insert(0, ROOT)
    import test_init

    test_init.test_setup()


def test_mnist_onegpu_cpu_learns():
    p = _run(["mnist_onegpu.py", "--device", "cpu", "--image-size", "32", "--epochs", "1", "--max-steps", "60",
              "--log-interval", "20", "--lr", "0.05", "--dataset-size", "600", "--json", "--phase-times"])
    assert p.returncode == 0, p.stderr
    losses = [float(x) for x in re.findall(r"Epoch \[1/1\], Step \[\d+/60\], Loss: ([\d.]+)", p.stdout)]
    assert len(losses) == 3
    assert "Training complete in: " in p.stdout
    summ = json.loads(p.stdout.strip().splitlines()[-1])
    assert summ["steps"] == 60
    assert set(summ["phases"]) == {"forward", "backward", "optimizer"}  # StepTimer (host wall time on CPU)


def test_mnist_distributed_cpu(tmp_path):
    ck = str(tmp_path / "ck.pt")
    p = _run(["mnist_distributed.py", "-g", "2", "--device", "cpu", "--backend", "gloo", "--image-size", "32",
              "--epochs", "1", "--max-steps", "20", "--log-interval", "10", "--lr", "0.05", "--dataset-size", "400",
              "--checkpoint", ck, "--avg-loss"])
    assert p.returncode == 0, p.stderr
    assert len(re.findall(r"Rank \[0\], Epoch \[1/1\], Step \[\d+/20\], Loss: ", p.stdout)) == 2
    assert "Training complete in: " in p.stdout
    assert os.path.exists(ck)
    sd = torch.load(ck, weights_only=True)
    assert "fc.weight" in sd["model"] or "module.fc.weight" in sd["model"]
    # resume
    p2 = _run(["mnist_distributed.py", "-g", "2", "--device", "cpu", "--backend", "gloo", "--image-size", "32",
               "--epochs", "2", "--max-steps", "5", "--dataset-size", "400", "--resume", ck])
    assert p2.returncode == 0, p2.stderr


def test_mnist_distributed_fault_fails_fast():
    p = _run(["mnist_distributed.py", "-g", "2", "--device", "cpu", "--backend", "gloo", "--image-size", "32",
              "--epochs", "1", "--max-steps", "10", "--dataset-size", "200"],
             env={"TDS_FAULT_RANK": "1", "TDS_FAULT_STEP": "3", "TDS_FAULT_MODE": "raise"}, timeout=200)
    assert p.returncode != 0
    assert "injected fault on rank 1 at step 3" in p.stderr


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_bench_self_spawns_ranks_cpu():
    """`python bench.py --gpus 2` with no external launcher starts both ranks itself
    (reference: mp.spawn(train, nprocs=args.gpus), mnist_distributed.py:127) and rank 0
    prints exactly one JSON line for the whole job."""
    p = _run(["bench.py", "--gpus", "2", "--device", "cpu", "--image-size", "32", "--steps", "2", "--warmup", "1"])
    assert p.returncode == 0, p.stderr
    recs = _json_lines(p.stdout)
    assert len(recs) == 1
    r = recs[0]
    assert r["n_gpus"] == 2 and r["steps"] == 2 and r["warmup"] == 1
    assert r["config"]["global_batch"] == 10 and r["config"]["parallelism"] == "dp2"
    assert r["config"]["backend"] == "gloo" and r["value"] > 0
    assert r["config"]["store"] == "native"  # the C++ rendezvous store (parallel/store.py rendezvous)
    assert r["dtype"] == "fp32 (CPU rehearsal: torch ops)"
    (pr,) = r["config"]["allreduce_probe"]  # post-timing all-reduce bandwidth over the same communicator
    assert pr["MB"] > 0 and pr["ms"] > 0 and pr["busbw_GBps"] > 0


def test_bench_self_spawn_native_host_backend_cpu():
    p = _run(["bench.py", "--gpus", "3", "--device", "cpu", "--image-size", "32", "--steps", "1", "--warmup", "1",
              "--backend", "host"])
    assert p.returncode == 0, p.stderr
    (r,) = _json_lines(p.stdout)
    assert r["n_gpus"] == 3 and r["config"]["reducer"] == "native"


def test_bench_spawn_failure_propagates_cpu():
    # --shared-device refuses a non-gloo backend inside every rank: the parent must fail, not hang
    p = _run(["bench.py", "--gpus", "2", "--device", "cpu", "--image-size", "32", "--steps", "1", "--warmup", "0",
              "--backend", "host", "--shared-device"], timeout=200)
    assert p.returncode != 0
    (r,) = _json_lines(p.stdout)  # one failure record, no measurement
    assert r["status"] == "failed" and r["value"] is None and "shared-device" in r["error"]


def test_bench_allreduce_cpu_rehearsal():
    """tools/bench_allreduce.py end to end on 2 gloo ranks (tiny sizes): the all-reduce sweep
    and the fc-gradient exchange paths it times on the 8-GPU node."""
    p = _run(["tools/bench_allreduce.py", "--gpus", "2", "--device", "cpu", "--backend", "gloo", "--max-bytes", "4096",
              "--iters", "2", "--warmup", "1", "--no-ddp-sizes", "--exchanges", "--rows", "2", "--in-features", "4096"])
    assert p.returncode == 0, p.stderr[-2000:]
    rec = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["world"] == 2 and len(rec["rows"]) == 6
    assert [r["path"].split()[0] for r in rec["exchanges"]] == ["activations", "sharded", "chunked", "allreduce"]


# ---- W=8 rehearsal and bounded failure handling (bench.py's first real multi-GPU run must
# succeed or explain itself inside the driver's lease)

@pytest.mark.parametrize("backend", ["gloo", "host"])
def test_bench_w8_cpu(backend):
    """The 8-rank path end to end: self-spawn, rendezvous, the W=8 fc-gradient choice (sharded
    exchange by the byte model) and the one JSON line."""
    # 256^2: the fc weight (10 x 131072) is big enough to be an exchange candidate
    p = _run(["bench.py", "--gpus", "8", "--device", "cpu", "--image-size", "256", "--steps", "1", "--warmup", "1",
              "--backend", backend, "--no-allreduce-probe"], timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    (r,) = _json_lines(p.stdout)
    assert r["n_gpus"] == 8 and r["config"]["global_batch"] == 40 and r["config"]["parallelism"] == "dp8"
    assert r["config"]["fc_grad"] == "sharded-exchange(zs)"  # zero-suppressed X shards (parallel/zs.py)
    assert r["config"]["reducer"] == ("native" if backend == "host" else "python")
    assert r["config"]["store"] == "native"


def test_bench_rank_that_never_joins_reports_json():
    """A rank that never reaches the rendezvous: the job ends within the bounded waits and the
    parent prints ONE failure record naming the failing rank."""
    import time

    t0 = time.time()
    p = _run(["bench.py", "--gpus", "2", "--device", "cpu", "--image-size", "32", "--steps", "1", "--warmup", "1",
              "--backend", "gloo", "--pg-timeout", "8", "--deadline", "60", "--spawn-timeout", "90"],
             env={"TDS_BENCH_FAULT": "1:init:hang"}, timeout=200)
    assert time.time() - t0 < 150
    assert p.returncode != 0
    (r,) = _json_lines(p.stdout)
    assert r["status"] == "failed" and r["value"] is None and r["n_gpus"] == 2
    assert r["failed_rank"] in (0, 1) and r["error"] and r["rc"] != 0


def test_bench_rank_deadline_reports_json_under_torchrun_env():
    """Run as one rank of an externally launched job (WORLD_SIZE set, the driver's torchrun
    form) that cannot finish: rank 0 itself prints the failure record at its deadline."""
    p = _run(["bench.py", "--gpus", "1", "--device", "cpu", "--image-size", "32", "--steps", "1", "--warmup", "2",
              "--deadline", "20"],
             env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0", "TDS_BENCH_FAULT": "0:step:hang"}, timeout=200)
    assert p.returncode == 124
    (r,) = _json_lines(p.stdout)
    assert r["status"] == "failed" and "still running" in r["error"]


def test_bench_falls_back_after_a_failed_attempt_cpu():
    """Attempt 0 (the native host backend) fails on rank 1 mid-warmup; every rank votes through
    the rendezvous store, tears the group down and the plain stack (gloo, bucket all-reduce)
    produces the measurement, labelled with the reason."""
    p = _run(["bench.py", "--gpus", "2", "--device", "cpu", "--image-size", "32", "--steps", "1", "--warmup", "1",
              "--backend", "host", "--fallback", "--pg-timeout", "15", "--no-allreduce-probe"],
             env={"TDS_BENCH_FAULT": "1:step:raise:1"}, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    (r,) = _json_lines(p.stdout)
    assert r["value"] > 0 and r["config"]["attempt"] == 1
    assert r["config"]["backend"].startswith("gloo (fallback: rank 1")
    assert "InjectedFault" in r["config"]["backend"]
    assert r["config"]["store"] == "native"  # the vote and both attempts' rendezvous went through it


def test_trainer_and_bench_pick_the_same_stack(monkeypatch):
    """mnist_distributed.py (trainer) and bench.py default to the same multi-GPU stack on a GPU:
    rccl-native (this package's communicator, so the C++ reducer) with the CU split."""
    import argparse

    sys.path.insert(0, ROOT)
    import bench
    from torch_distributed_sandbox_amd.parallel import distributed as tdist
    from torch_distributed_sandbox_amd.trainer import add_common_args, resolve_backend

    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    targs = add_common_args(argparse.ArgumentParser()).parse_args([])
    targs.backend = "auto"
    bargs = bench._parser().parse_args([])
    assert bargs.backend is None and bargs.device == "cuda"
    assert resolve_backend(targs) == tdist.default_backend(bargs.device == "cuda") == "rccl-native"
    assert tdist._normalise_backend("auto") == "rccl-native"
    assert tdist.is_device_backend("rccl-native") and tdist.is_device_backend("nccl")
    assert not tdist.is_device_backend("gloo")
    targs.backend = "rccl"
    assert resolve_backend(targs) == "rccl"  # torch's ProcessGroupNCCL stays selectable


def _torchrun(n, args, env=None, timeout=300):
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    return _run(["-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr", "127.0.0.1",
                 "--master-port", str(port)] + args, env=env, timeout=timeout)


def test_bench_under_torchrun_cpu():
    """The driver's multi-GPU form: torchrun starts the ranks, bench.py runs as each of them
    (WORLD_SIZE set), rank 0 prints the one JSON line."""
    p = _torchrun(2, ["bench.py", "--gpus", "2", "--device", "cpu", "--image-size", "32", "--steps", "2",
                      "--warmup", "1", "--no-allreduce-probe"])
    assert p.returncode == 0, p.stderr[-3000:]
    (r,) = _json_lines(p.stdout)
    assert r["n_gpus"] == 2 and r["steps"] == 2 and r["value"] > 0 and r["config"]["parallelism"] == "dp2"
    assert r["config"]["store"] == "native"  # located through torchrun's agent store


def test_bench_under_torchrun_falls_back_cpu():
    """Under torchrun there is no spawning parent: the ranks themselves vote through the store
    and re-run on the plain stack in the same processes."""
    p = _torchrun(2, ["bench.py", "--gpus", "2", "--device", "cpu", "--image-size", "32", "--steps", "1",
                      "--warmup", "1", "--backend", "host", "--fallback", "--pg-timeout", "15",
                      "--no-allreduce-probe"], env={"TDS_BENCH_FAULT": "1:step:raise:1"})
    assert p.returncode == 0, p.stderr[-3000:]
    (r,) = _json_lines(p.stdout)
    assert r["value"] > 0 and r["config"]["backend"].startswith("gloo (fallback: rank 1")


@pytest.mark.parametrize("world,phase", [(2, "preflight"), (2, "step"), (8, "preflight"), (8, "step")])
def test_bench_fallback_tiers_keep_the_exchange_cpu(world, phase):
    """A fault on rank 1 in the collective preflight or mid-warmup of tier 1 (the native host
    ring standing in for rccl-native): the ranks vote, tear down and run tier 2 -- torch's own
    process group (gloo standing in for ProcessGroupNCCL) with the SAME zero-suppressed fc
    exchange, not the dense all-reduce.  The JSON names the tier, the reason and the preflight
    of the tier that ran."""
    p = _run(["bench.py", "--gpus", str(world), "--device", "cpu", "--image-size", "232", "--steps", "1",
              "--warmup", "1", "--backend", "host", "--fallback", "--pg-timeout", "30", "--no-allreduce-probe"],
             env={"TDS_BENCH_FAULT": f"1:{phase}:raise:1"}, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    (r,) = _json_lines(p.stdout)
    c = r["config"]
    assert r["value"] > 0 and c["attempt"] == 1 and c["tier"] == "2/3"
    assert c["backend"].startswith("gloo (fallback: rank 1") and f"phase {phase}" in c["backend"]
    assert c["store"] == "native"
    want = "activation-exchange(zs)" if world == 2 else "sharded-exchange(zs)"
    assert c["fc_grad"] == want
    pf = c["preflight"]
    assert pf["fc_path"] == ("activations" if world == 2 else "sharded")
    ops = [x["op"] for x in pf["collectives"]]
    assert "BN buffer broadcast (coalesced)" in ops and ops[-1] == "barrier"
    if world == 2:
        assert any(o.startswith("zs values all-gather") and o.endswith("(first-step capacity)") for o in ops)
    else:
        assert "X column-shard exchange (per peer)" in ops and "updated W shard exchange (per peer)" in ops
    assert all(x["ms"] >= 0 for x in pf["collectives"])


def test_bench_last_tier_is_the_bucket_allreduce_cpu():
    """Tiers 1 and 2 both fail in the preflight: tier 3, the plain bucket all-reduce, runs."""
    p = _run(["bench.py", "--gpus", "2", "--device", "cpu", "--image-size", "232", "--steps", "1",
              "--warmup", "1", "--backend", "host", "--fallback", "--pg-timeout", "30", "--no-allreduce-probe"],
             env={"TDS_BENCH_FAULT": "1:preflight:raise:2"}, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    (r,) = _json_lines(p.stdout)
    c = r["config"]
    assert r["value"] > 0 and c["attempt"] == 2 and c["tier"] == "3/3"
    assert c["fc_grad"] == "allreduce" and c["preflight"]["fc_path"] == "allreduce"
    assert any(x["op"].startswith("bucket 0 all-reduce") for x in c["preflight"]["collectives"])
