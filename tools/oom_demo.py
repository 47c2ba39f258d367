"""The reference's "OOM workaround" story (README.md:9-15),
re-sized for 288 GB of HBM3E per MI355X.

The reference: at 3000x3000 a per-GPU batch of 10 does not fit one 24 GB A5000,
a batch of 5 does, so DDP with 5 per rank x N ranks gives an effective batch
of 5N.  Our fused ConvNet plan needs far less memory per image (no y1, no p2,
1-byte argmax, NHWC bf16 hi|lo activations), so the edge where batch 10 stops
fitting 288 GB is much larger.  This script:

1. prints the memory model of the fused plan and the predicted OOM edge,
2. tries ONE training step at batch 10 on this GPU at --image-size and reports
   the out-of-memory error (expected),
3. runs --steps steps at batch 5 on the same image size (fits) and reports
   peak memory and images/sec,
4. with --gpus N (ranks started here, one per GPU, like bench.py and the reference's
   mp.spawn) or under torchrun with N ranks: step 2 runs on rank 0 alone, step 3 is the
   DDP run over all ranks, effective batch 5N.

    python tools/oom_demo.py                                     # 1 GPU, just past the batch-10 edge
    python tools/oom_demo.py --gpus 8                            # the DDP half: 8 ranks

Round 4 re-measured the plan at HEAD (uint8 level input, fp16 p1): at 18000^2 a batch of 10
now fits (275 GB peak, profiles/r4_oom_demo_18000.json).  With the conv2 output stored as y2h
(64 B per pixel instead of 128) the edge moved again: at 23000^2 batch 10 runs out of memory and
batch 5 trains at 224.9 GB peak (profiles/r4_oom_demo_23000.json), so the default edge is 23000.
    python tools/oom_demo.py --gpus 2 --shared-device --image-size 1024 --calib-size 512
                                                                 # rehearsal: 2 gloo ranks on cuda:0
"""
import argparse
import gc
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

# Memory model of the fused plan at HEAD, peak(H, B) = (act * B + fixed) * H^2 bytes, calibrated on
# this GPU by two short runs at --calib-size (batch 1 and 2): act = bytes per input pixel per image
# (x levels, p1, argmax codes, y2h, ya, g2m, dp1h, ...), fixed = per-pixel bytes that do not scale
# with the batch: the fc weight, 10 * 32 * (H/4)^2 * 4 B = 80 B/px, held once in DDP's flat parameter
# buffer.  Its GRADIENT is not a fixed cost of this plan: the runs below train as bench.py and the
# trainer do (DistributedDataParallel(overlap_optimizer=True), plain SGD), so at world size 1 the fc
# weight steps inside the head backward kernel and its 80 B/px gradient slot is never allocated
# (parallel/ddp.py _lazy_from; round 4's record still carried it: 39.4 GiB at 23000^2).  The DDP
# constructor holds the flat buffer and one original parameter at a time (2 x 80 B/px, before any
# activation exists): its peak is modelled apart, peak(H, B) = max((act * B + fixed), ctor) * H^2.


def calibrate(H, device):
    """(act, fixed, ctor) bytes per input pixel: the training step's peak is (B * act + fixed) * H^2,
    the DDP constructor's (before any activation exists) ctor * H^2.  The two peaks are measured
    apart (r6: at 3000^2 the constructor's 2 x 80 B/px was above the batch-1 step, and fitting
    the overall peaks at batch 1 and 2 made act far too small -- the auto size then OOMed at batch 5)."""
    ra, rb = run(H, 1, 1, device, 1, 0), run(H, 2, 1, device, 1, 0)
    a, b = ra["step_peak_gb"] * 1e9, rb["step_peak_gb"] * 1e9
    act = (b - a) / (H * H)
    fixed = a / (H * H) - act
    ctor = max(ra["ctor_peak_gb"], rb["ctor_peak_gb"]) * 1e9 / (H * H)
    return act, fixed, ctor, [ra, rb]


def predicted_bytes(H, B, act, fixed, ctor=0.0):
    return max(B * act + fixed, ctor) * H * H


def run(H, B, steps, device, world, rank):
    from torch_distributed_sandbox_amd.data import synthetic_batch
    from torch_distributed_sandbox_amd.models import ConvNet
    from torch_distributed_sandbox_amd.ops import SGD, CrossEntropyLoss
    from torch_distributed_sandbox_amd.ops import functional as TF
    from torch_distributed_sandbox_amd.parallel import DistributedDataParallel

    gc.collect()
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(device)
    base = torch.cuda.memory_allocated(device)  # anything a previous run left (should be ~0)
    torch.manual_seed(0)
    model = ConvNet(image_shape=(H, H), device=device)
    opt = SGD(model.parameters(), 1e-4)
    ddp = DistributedDataParallel(model, device_ids=[device.index], overlap_optimizer=True)
    ddp.attach_optimizer(opt)
    ctor_peak = torch.cuda.max_memory_allocated(device)
    torch.cuda.reset_peak_memory_stats(device)
    crit = CrossEntropyLoss()
    src, lab = synthetic_batch(B, (H, H), device, seed=7 + rank)
    t0 = None
    for i in range(steps):
        images = TF.upsample_bilinear_u8(src, H, H, levels=True)  # the bench / trainer default input
        loss = crit(ddp(images), lab)
        opt.zero_grad()
        TF.backward(loss)
        opt.step()
        ddp.wait_pending_updates()
        if i == 0:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / max(1, steps - 1) if steps > 1 else None
    step_peak = torch.cuda.max_memory_allocated(device)
    peak = max(ctor_peak, step_peak)
    grad_gb = ddp.grad_storage_bytes() / 1e9
    del ddp, model, opt, images, loss
    gc.collect()
    torch.cuda.empty_cache()
    return {"batch_per_rank": B, "peak_gb": round((peak - base) / 1e9, 3), "base_gb": round(base / 1e9, 3),
            "ctor_peak_gb": round((ctor_peak - base) / 1e9, 3), "step_peak_gb": round((step_peak - base) / 1e9, 3),
            "flat_grad_gb": round(grad_gb, 4),
            "ms_per_step": round(dt * 1e3, 2) if dt else None,
            "images_per_sec_node": round(world * B / dt, 2) if dt else None}


def _parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--image-size", type=int, default=0,
                    help="0 (default): just past the calibrated model's batch-10 edge (batch 10 predicted at "
                         ">= 106 %% of the GPU's memory), rounded up to a multiple of 500")
    ap.add_argument("--bs-fail", type=int, default=10)
    ap.add_argument("--bs-fit", type=int, default=5)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--calib-size", type=int, default=3000)
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU) started by this script")
    ap.add_argument("--backend", default=None, help="process group for --gpus > 1 (default: rccl-native)")
    ap.add_argument("--shared-device", action="store_true",
                    help="rehearsal: every rank on cuda:0 over gloo (plumbing only, not an OOM result)")
    ap.add_argument("--timeout", type=float, default=1800.0, help="--gpus > 1: terminate the ranks after this (s)")
    ap.add_argument("--single-gpu-half", action="store_true",
                    help="internal: run the calibration and the batch-%(default)s attempt, print their JSON, exit")
    return ap


def single_gpu_half(args, device):
    """Calibrate the memory model, pick the image size and try the failing batch on ONE GPU.
    Runs in a process of its own (main() starts it before touching the GPU): a training step that
    dies of out-of-memory part-way through the forward can leave tensors referenced from the
    half-built autograd graph and the DDP hooks, and the batch-5 run must start on an empty GPU."""
    total = torch.cuda.get_device_properties(device).total_memory
    act, fixed, ctor, calib_runs = calibrate(args.calib_size, device)
    gc.collect()
    torch.cuda.empty_cache()
    H = args.image_size
    if H <= 0:
        edge = (1.06 * total / max(args.bs_fail * act + fixed, ctor)) ** 0.5
        H = int(-(-edge // 500) * 500)
    rec = {"image_size": H, "gpu_total_gb": round(total / 1e9, 1),
           "model": {"calibrated_at": args.calib_size, "calibration_runs": calib_runs,
                     "act_bytes_per_px_per_image": round(act, 1),
                     "fixed_bytes_per_px": round(fixed, 1),
                     "ddp_constructor_bytes_per_px": round(ctor, 1),
                     "predicted_gb": {str(b): round(predicted_bytes(H, b, act, fixed, ctor) / 1e9, 1)
                                      for b in (args.bs_fit, args.bs_fail)},
                     "predicted_oom_edge_bs%d" % args.bs_fail:
                         int((total / max(args.bs_fail * act + fixed, ctor)) ** 0.5)}}
    try:
        r = run(H, args.bs_fail, 1, device, 1, 0)
        rec["bs_fail_result"] = {"oom": False, **r}
    except torch.cuda.OutOfMemoryError as e:
        msg = str(e).split("\n")[0]
        rec["bs_fail_result"] = {"oom": True, "error": msg[:300]}
    return rec


def _run_single_gpu_half(argv, local):
    """The single-GPU half in a child process (this process has not touched the GPU yet)."""
    import subprocess

    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["LOCAL_RANK"] = str(local)
    p = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), *argv, "--gpus", "1", "--single-gpu-half"],
                       env=env, stdout=subprocess.PIPE, text=True)
    if p.returncode != 0:
        raise SystemExit(f"oom_demo: the single-GPU half failed (exit {p.returncode})")
    return json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])


def _rank_entry(i, argv, world, addr, port):
    os.environ.update({"RANK": str(i), "LOCAL_RANK": str(i), "WORLD_SIZE": str(world), "LOCAL_WORLD_SIZE": str(world),
                       "MASTER_ADDR": addr, "MASTER_PORT": port})
    main(argv)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = _parser().parse_args(argv)
    from torch_distributed_sandbox_amd.parallel import distributed as tdist
    from torch_distributed_sandbox_amd.parallel import launch

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # the parent starts one rank per GPU and never touches the GPU itself
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        launch.spawn(_rank_entry, args=(argv, args.gpus, addr, launch.find_free_port(addr)), nprocs=args.gpus,
                     timeout=args.timeout)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.shared_device else int(os.environ.get("LOCAL_RANK", "0"))
    if args.single_gpu_half:
        torch.cuda.set_device(local)
        print(json.dumps(single_gpu_half(args, torch.device("cuda", local))), flush=True)
        return
    H = args.image_size
    rec = None
    if H <= 0 and world > 1:
        raise SystemExit("oom_demo: --image-size 0 (auto) is for one process; give the size for --gpus > 1")
    if rank == 0:
        # 1) calibration + batch 10 on ONE GPU, in a child process, BEFORE this rank touches the GPU
        # or the process group exists; the other ranks wait in the rendezvous meanwhile
        rec = _run_single_gpu_half(argv, local)
        H = rec["image_size"]
        rec["world_size"] = world
        if args.shared_device:
            rec["shared_device"] = True  # rehearsal: all ranks on one GPU
    elif H <= 0:
        raise SystemExit("oom_demo: the ranks need --image-size")
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        import datetime

        backend = "gloo" if args.shared_device else (args.backend or tdist.default_backend(True))
        tdist.init_process_group(backend, rank=rank, world_size=world, timeout=datetime.timedelta(hours=1),
                                 device_id=None if backend == "gloo" else local)
    # 2) batch 5 per rank: DDP over all ranks
    try:
        fit = run(H, args.bs_fit, args.steps, device, world, rank)
    except torch.cuda.OutOfMemoryError as e:
        if world > 1:
            raise
        fit = {"oom": True, "error": str(e).split("\n")[0][:300]}
    if rank == 0:
        rec["bs_fit_result"] = fit
        rec["effective_batch"] = args.bs_fit * world
        print(json.dumps(rec), flush=True)
    if world > 1:
        tdist.barrier()
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
