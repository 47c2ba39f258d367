"""Training loops behind ``mnist_onegpu.py`` and ``mnist_distributed.py``.

Reference loops: mnist_onegpu.py:34-84 (single GPU) and
mnist_distributed.py:48-109 (DDP); SURVEY.md §3.3-§3.4.  Kept: seed 0 before
model construction, ConvNet topology, bs=5, SGD(lr=1e-4), CE loss,
``zero_grad -> backward -> step`` order, the log lines (every 100 steps on
local GPU 0, rank-local loss) and ``Training complete in: ...``.  Added:
images/sec, peak memory, ``--max-steps``, synthetic on-device data, optional
global-average loss (the reference's commented-out ``all_reduce(AVG)``,
mnist_distributed.py:102), checkpoint/resume, fault injection.
"""
from __future__ import annotations

import argparse
import json
import os
import time
from datetime import datetime

import torch

from . import _ext
from .data import DeviceUpsampleLoader, SyntheticMNIST
from .models import ConvNet, convnet_fused
from .ops import CrossEntropyLoss, SGD
from .ops import functional as TF
from .parallel import DistributedDataParallel, DistributedSampler
from .parallel import distributed as tdist
from .utils import checkpoint, fault
from .utils.timing import StepTimer


def add_common_args(p: argparse.ArgumentParser) -> argparse.ArgumentParser:
    p.add_argument("--epochs", default=2, type=int, metavar="N", help="number of total epochs to run")
    p.add_argument("--image-size", default=3000, type=int, help="square image edge (reference: 3000)")
    p.add_argument("--batch-size", default=5, type=int, help="per-GPU batch size (reference: 5)")
    p.add_argument("--lr", default=1e-4, type=float)
    p.add_argument("--max-steps", default=0, type=int, help="stop after this many steps per epoch (0 = full epoch)")
    p.add_argument("--dataset-size", default=60000, type=int, help="synthetic MNIST size (reference: 60000)")
    p.add_argument("--log-interval", default=100, type=int)
    p.add_argument("--mode", default="auto", choices=["auto", "fused", "layers"], help="ConvNet execution plan")
    p.add_argument("--input", default="levels", choices=["levels", "fp32"],
                   help="batches as the resized images' uint8 levels (ToTensor's 1/255 folded into conv1) or as "
                        "the materialised fp32 ToTensor image")
    p.add_argument("--device", default="auto", choices=["auto", "cuda", "cpu"])
    p.add_argument("--checkpoint", default="", help="save a checkpoint here at the end (rank 0)")
    p.add_argument("--resume", default="", help="resume from this checkpoint")
    p.add_argument("--json", action="store_true", help="print a JSON summary line at the end")
    p.add_argument("--grad-exchange", default="auto", choices=["auto", "allreduce", "activations", "sharded", "chunked"],
                   help="DDP gradient path of the big fc layer (parallel/factored.py)")
    p.add_argument("--phase-times", action="store_true",
                   help="time forward / backward / optimizer per step with HIP events (utils/timing.StepTimer; "
                        "adds them to the summary; roctx ranges with TDS_ROCTX=1)")
    p.add_argument("--overlap-optimizer", action=argparse.BooleanOptionalAction, default=True,
                   help="finish the fc bucket (collective + SGD) on a side stream under the next forward")
    p.add_argument("--bucket-mb", default=None, type=float, help="DDP bucket cap (MB, default 25 like torch)")
    p.add_argument("--reserve-cus", default=None, type=int,
                   help="rccl-native: CUs split off for the collectives (multiple of 32; default 32 at world > 1)")
    return p


def resolve_backend(args) -> str:
    """--backend, or the tuned default (parallel.distributed.default_backend): rccl-native on
    the GPU -- the stack bench.py measures -- and gloo on the CPU."""
    b = getattr(args, "backend", None)
    if b in (None, "auto"):
        on_gpu = args.device != "cpu" and torch.cuda.is_available()
        return tdist.default_backend(on_gpu)
    return tdist._normalise_backend(b)


def _device(args, gpu: int) -> torch.device:
    want = args.device
    if want == "auto":
        want = "cuda" if torch.cuda.is_available() else "cpu"
    if want == "cuda":
        torch.cuda.set_device(gpu)
        _ext.ops()  # fail loudly if the native extension is missing on a GPU box
        return torch.device("cuda", gpu)
    return torch.device("cpu")


def train(gpu: int, args, distributed: bool = False) -> dict:
    rank = 0
    world = 1
    if distributed:
        rank = args.nr * args.gpus + gpu
        world = args.world_size
        backend = resolve_backend(args)
        dev_backend = tdist.is_device_backend(backend)
        # the same stack bench.py measures: rccl-native + C++ reducer + the compute/comm CU split
        tdist.init_process_group(backend=backend, world_size=world, rank=rank,
                                 device_id=gpu if dev_backend else None,
                                 comm_cus=getattr(args, "reserve_cus", None) if backend == "rccl-native" else None)
    device = _device(args, gpu)
    torch.manual_seed(0)
    H = W = args.image_size
    model = ConvNet(image_shape=(H, W), device=device, mode=args.mode)
    batch_size = args.batch_size
    criterion = CrossEntropyLoss()
    optimizer = SGD(model.parameters(), args.lr)
    if distributed or device.type == "cuda":
        # the tuned plan bench.py measures, also for the single-GPU script: at world size 1 the
        # wrapper owns the flat parameter / gradient buffers (one SGD sweep over the small
        # parameters), fuses the fc weight's SGD step into the head backward kernel
        # (ops/fused_update.py) and finishes the rest under the next forward (overlap_optimizer)
        # -- the reference's mnist_onegpu.py has no wrapper and steps all 180 M parameters in a
        # separate pass
        model = DistributedDataParallel(model, device_ids=[gpu] if device.type == "cuda" else None,
                                        bucket_cap_mb=getattr(args, "bucket_mb", None),
                                        grad_exchange=getattr(args, "grad_exchange", "auto"),
                                        overlap_optimizer=getattr(args, "overlap_optimizer", True))
        model.attach_optimizer(optimizer)
    start_epoch = 0
    if args.resume:
        _, start_epoch, _ = checkpoint.load(args.resume, model, optimizer, map_location=device)
    dataset = SyntheticMNIST(size=args.dataset_size)
    levels = getattr(args, "input", "levels") == "levels"
    fused_plan = getattr(args, "mode", "auto") != "layers"
    moments = levels and fused_plan  # the fused plan reads them
    if distributed:
        sampler = DistributedSampler(len(dataset), num_replicas=world, rank=rank)
        loader = DeviceUpsampleLoader(dataset, batch_size, (H, W), device, sampler=sampler, levels=levels,
                                      moments=moments)
    else:
        loader = DeviceUpsampleLoader(dataset, batch_size, (H, W), device, shuffle=True, levels=levels,
                                      moments=moments)

    start = datetime.now()
    total_step = len(loader)
    if args.max_steps:
        total_step = min(total_step, args.max_steps)
    steps_done = 0
    t_first = None
    loss = None
    timer = StepTimer(enabled=getattr(args, "phase_times", False) and device.type == "cuda")
    for epoch in range(start_epoch, args.epochs):
        loader.set_epoch(epoch)
        for i, (images, labels) in enumerate(loader):
            if args.max_steps and i >= args.max_steps:
                break
            fault.maybe_inject(rank, steps_done)
            with timer.phase("forward"):
                if fused_plan and images.is_cuda:
                    # (fused plan: the loss and dlogits formed by the head forward with the logits)
                    convnet_fused.attach_labels(images, labels)
                outputs = model(images)
                loss = criterion(outputs, labels)
            optimizer.zero_grad()
            with timer.phase("backward"):
                TF.backward(loss)
            with timer.phase("optimizer"):
                optimizer.step()
            if distributed:
                # the reference builds a group every step (mnist_distributed.py:99-100); cached here
                tdist.new_group(ranks=list(range(args.gpus)) if args.nodes == 1 else None)
            steps_done += 1
            if steps_done == 1 and device.type == "cuda":
                torch.cuda.synchronize()
                t_first = time.perf_counter()
            if (i + 1) % args.log_interval == 0:
                shown = loss.detach()
                if distributed and getattr(args, "avg_loss", False):
                    # collective: every rank joins, rank 0 prints
                    shown = shown.clone()
                    tdist.all_reduce(shown, tdist.ReduceOp.AVG)
                if gpu != 0:
                    pass
                elif distributed:
                    print("Rank [{}], Epoch [{}/{}], Step [{}/{}], Loss: {:.4f}".format(
                        rank, epoch + 1, args.epochs, i + 1, total_step, shown.item()), flush=True)
                else:
                    print("Epoch [{}/{}], Step [{}/{}], Loss: {:.4f}".format(
                        epoch + 1, args.epochs, i + 1, total_step, shown.item()), flush=True)
    if hasattr(model, "wait_pending_updates"):
        model.wait_pending_updates()  # the last step's deferred fc update (ops/param_fence.py)
    if device.type == "cuda":
        torch.cuda.synchronize()
    t_end = time.perf_counter()
    summary = {"rank": rank, "world_size": world, "steps": steps_done, "batch_size": batch_size,
               "image_size": H, "final_loss": float(loss.item()) if loss is not None else None,
               "plan": (f"DDP wrapper ({getattr(model, 'reducer_kind', '?')} reducer, fc grad "
                        f"{model.fc_grad_path()}, overlap_optimizer={model.overlap_optimizer})"
                        if isinstance(model, DistributedDataParallel) else "plain module"),
               "store": tdist.store_kind() if distributed else None}
    if t_first is not None and steps_done > 1:
        dt = t_end - t_first
        summary["images_per_sec_per_rank"] = (steps_done - 1) * batch_size / dt
        summary["images_per_sec_global"] = summary["images_per_sec_per_rank"] * world
        summary["ms_per_step"] = 1e3 * dt / (steps_done - 1)
    if device.type == "cuda":
        summary["peak_mem_gb"] = torch.cuda.max_memory_allocated(device) / 1e9
    if getattr(args, "phase_times", False):
        summary["phases"] = timer.summary()
    if gpu == 0:
        print("Training complete in: " + str(datetime.now() - start), flush=True)
        if args.json:
            print(json.dumps(summary), flush=True)
    if args.checkpoint:
        checkpoint.save(args.checkpoint, model, optimizer, step=steps_done, epoch=args.epochs, rank=rank)
    if distributed:
        tdist.barrier()
        tdist.destroy_process_group()
    return summary
