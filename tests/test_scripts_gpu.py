"""Entry points on the MI355X: the toy on this package's RCCL communicator and a one-GPU
rehearsal of the OOM demo's DDP half (the whole story needs an 8-GPU node)."""
import json
import os
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=240):
    return subprocess.run([sys.executable, "-u"] + args, cwd=ROOT, capture_output=True, text=True, timeout=timeout)


def test_allreduce_toy_rccl_native_device_tensor(gpu):
    """Reference: allreduce_toy.py:30-31 all-reduces an int32 tensor on cuda:{rank}; here on the
    rccl-native communicator (one rank: the box has one GPU)."""
    p = _run(["allreduce_toy.py", "-s", "1", "--backend", "rccl-native", "--steps", "3"])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = re.findall(r"rank: 0, step: (\d+), value: (\d+), reduced sum: (\d+)\.", p.stdout)
    assert [s for s, _, _ in lines] == ["1", "2", "3"]
    assert all(v == t for _, v, t in lines)  # one rank: the sum is its own value


def test_oom_demo_ddp_half_shared_device_rehearsal(gpu):
    """tools/oom_demo.py --gpus 2 starts its own ranks (no torchrun); rank 0 runs the
    single-GPU half first, then both ranks run the DDP half (gloo ranks sharing cuda:0 at a
    small image edge: plumbing, not an OOM result)."""
    p = _run(["tools/oom_demo.py", "--gpus", "2", "--shared-device", "--image-size", "512", "--calib-size", "256",
              "--steps", "2", "--timeout", "200"])
    assert p.returncode == 0, p.stderr[-3000:]
    (rec,) = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert rec["world_size"] == 2 and rec["effective_batch"] == 10 and rec["shared_device"]
    assert rec["bs_fail_result"]["oom"] is False  # 512^2 fits: the rehearsal checks the path only
    assert rec["bs_fit_result"]["batch_per_rank"] == 5 and rec["bs_fit_result"]["ms_per_step"] > 0


def test_mnist_onegpu_runs_the_tuned_plan(gpu):
    """mnist_onegpu.py on the GPU runs the plan bench.py measures (DDP wrapper at world size 1:
    flat buffers, the fc SGD step fused into the head backward, overlapped optimizer) with the
    device-resident loader, and still prints the reference's log lines."""
    import json

    p = subprocess.run([sys.executable, "mnist_onegpu.py", "--image-size", "512", "--epochs", "1", "--max-steps", "6",
                        "--log-interval", "3", "--dataset-size", "200", "--json"], cwd=ROOT, capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    assert "Epoch [1/1], Step [3/6], Loss:" in p.stdout and "Training complete in:" in p.stdout
    r = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert r["steps"] == 6 and r["plan"].startswith("DDP wrapper (native reducer, fc grad local")
    assert "overlap_optimizer=True" in r["plan"] and r["ms_per_step"] > 0
