"""Headline benchmark: images/sec (whole node) of the 3000x3000 MNIST ConvNet under DDP.

BASELINE.json metric/config: ConvNet (mnist_onegpu.py:11-31), 3000x3000 inputs,
per-rank batch 5, SGD(lr=1e-4), CrossEntropy, one process per MI355X over
RCCL/xGMI, synthetic data + random init (no network for MNIST), fp32.

    python bench.py                                  # 1 GPU, default steps
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A timed step is the full training step: on-device data generation (28x28
uint8 -> 3000x3000 bilinear upsample), forward, loss, zero_grad, backward
(with the bucketed gradient all-reduce), optimizer step.  W untimed warmup
steps, then exactly K steps bracketed by barrier + synchronize; the elapsed
time is the MAX over ranks.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

METRIC = "images/sec (whole node), 3000x3000 MNIST ConvNet DDP at 1/2/4/8 MI355X"


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--image-size", type=int, default=3000)
    ap.add_argument("--batch-size", type=int, default=5, help="per-rank batch (reference: 5)")
    ap.add_argument("--mode", default="auto", choices=["auto", "fused", "layers"])
    ap.add_argument("--bucket-mb", type=float, default=None)
    ap.add_argument("--backend", default=os.environ.get("TDS_BENCH_BACKEND", "rccl"),
                    help="rccl (torch ProcessGroupNCCL = RCCL) | rccl-native (this package's C++ communicator)")
    ap.add_argument("--grad-exchange", default="auto", choices=["auto", "allreduce", "activations"],
                    help="fc gradient path under DDP: auto picks the activation exchange when it moves fewer "
                         "bytes per rank than the ring all-reduce (parallel/factored.py)")
    ap.add_argument("--overlap-optimizer", action=argparse.BooleanOptionalAction, default=True,
                    help="finish the fc bucket (collective + SGD) on a side stream under the next forward's convs")
    ap.add_argument("--profile-phases", action="store_true", help="also report per-phase GPU times (adds events)")
    args = ap.parse_args(argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal only (tools/steps_multirank_rehearsal.txt): several ranks on one GPU with a
    # host-side backend (gloo), to exercise the multi-rank code path where RCCL refuses a
    # shared device.  Never set by the driver.
    if os.environ.get("TDS_BENCH_SHARED_DEVICE") is not None:
        local_rank = int(os.environ["TDS_BENCH_SHARED_DEVICE"])
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus={args.gpus}; launch N>1 with torch.distributed.run",
              file=sys.stderr)
        if world == 1 and args.gpus > 1:
            sys.exit(2)

    import torch_distributed_sandbox_amd as tds
    from torch_distributed_sandbox_amd.data import synthetic_batch
    from torch_distributed_sandbox_amd.models import ConvNet
    from torch_distributed_sandbox_amd.ops import SGD, CrossEntropyLoss
    from torch_distributed_sandbox_amd.ops import functional as TF
    from torch_distributed_sandbox_amd.parallel import DistributedDataParallel
    from torch_distributed_sandbox_amd.parallel import distributed as tdist

    assert torch.cuda.is_available(), "bench.py needs a GPU"
    torch.cuda.set_device(local_rank)
    tds._ext.ops()  # native extension must be loaded (fails loudly otherwise)
    device = torch.device("cuda", local_rank)
    if world > 1 or args.grad_exchange == "activations":
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
        tdist.init_process_group(args.backend, rank=rank, world_size=world, device_id=local_rank)

    H = W = args.image_size
    B = args.batch_size
    torch.manual_seed(0)
    model = ConvNet(image_shape=(H, W), device=device, mode=args.mode)
    criterion = CrossEntropyLoss()
    optimizer = SGD(model.parameters(), 1e-4)
    ddp = DistributedDataParallel(model, device_ids=[local_rank], bucket_cap_mb=args.bucket_mb,
                                  grad_exchange=args.grad_exchange, overlap_optimizer=args.overlap_optimizer)
    ddp.attach_optimizer(optimizer)

    # a pool of synthetic 28x28 sources; each step upsamples a different slice on device
    pool = 16
    src_pool, lab_pool = synthetic_batch(B * pool, (H, W), device, seed=1234 + rank)
    src_pool = src_pool.view(pool, B, 28, 28)
    lab_pool = lab_pool.view(pool, B)

    def step(i):
        j = i % pool
        images = TF.upsample_bilinear_u8(src_pool[j], H, W)
        out = ddp(images)
        loss = criterion(out, lab_pool[j])
        optimizer.zero_grad()
        loss.backward()
        optimizer.step()
        return loss

    def sync_all():
        if world > 1:
            tdist.barrier()
        torch.cuda.synchronize()

    loss = None
    for i in range(args.warmup):
        loss = step(i)
    sync_all()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(args.warmup + i)
    sync_all()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        tdist.all_reduce(t, tdist.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(loss.item()) if loss is not None else None
    ms = 1e3 * elapsed / max(1, args.steps)
    imgs_per_sec = world * B * args.steps / elapsed
    if rank == 0:
        rec = {
            "metric": METRIC,
            "value": round(imgs_per_sec, 3),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (seeded 28x28 uint8 sources upsampled on device to HxW; random labels; random init)",
            "config": {
                "model": "ConvNet(conv5x5 1->16+BN+ReLU+pool2, conv5x5 16->32+BN+ReLU+pool2, fc 32*(H/4)^2->10)",
                "global_batch": world * B,
                "per_rank_batch": B,
                "seq_len": None,
                "image_size": [H, W],
                "parallelism": f"dp{world}",
                "mode": args.mode,
                "backend": args.backend if world > 1 else None,
                "reducer": ddp.reducer_kind,
                "overlap_optimizer": ddp.overlap_optimizer,
                "fc_grad": ("activation-exchange" if any(e.steps_exchanged for e in ddp.exchanges)
                            else "allreduce" if world > 1 else "local"),
                "optimizer": "SGD(lr=1e-4)",
                "peak_mem_gb": round(torch.cuda.max_memory_allocated(device) / 1e9, 3),
                "final_loss": final_loss,
            },
        }
        print(json.dumps(rec), flush=True)
    if tdist.is_initialized():
        tdist.barrier()
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
