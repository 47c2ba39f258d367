"""Annotated process-group init smoke test (reference: test_init.py).

``test_setup`` spawns 4 ranks that each run ``init_process_group``; the
backend switches from gloo to the device backend (RCCL) when enough GPUs are
visible.  pytest-collectable, and runnable as a script.

Deviation: the reference switches to NCCL whenever *any* GPU is present; with
4 ranks on fewer than 4 GPUs RCCL would refuse (two ranks on one device), so
we switch only when ``torch.cuda.device_count() >= world_size``.  Each rank
also tears its group down (the reference defines ``cleanup`` but never calls it).
"""
from typing import Tuple

import torch
from torch import Tensor

import torch_distributed_sandbox_amd.parallel.distributed as dist
from torch_distributed_sandbox_amd.parallel import launch


def set_sharing_strategy(new_strategy=None):
    """torch.multiprocessing sharing strategy: 'file_system' on macOS, else 'file_descriptor'."""
    import torch.multiprocessing as tmp
    from sys import platform

    if new_strategy is not None:
        tmp.set_sharing_strategy(new_strategy=new_strategy)
    elif platform == "darwin":
        tmp.set_sharing_strategy("file_system")
    else:
        tmp.set_sharing_strategy("file_descriptor")


def use_file_system_sharing_strategy():
    """Use when 'too many open files' errors appear with tensor sharing."""
    import torch.multiprocessing as tmp

    tmp.set_sharing_strategy("file_system")


find_free_port = launch.find_free_port


def setup_process(rank, world_size, port, backend="gloo", master_addr="127.0.0.1"):
    """Initialise the default process group for this rank (-1 = serial, skip)."""
    import os

    if rank != -1:
        print(f"setting up rank={rank} (with world_size={world_size})", flush=True)
        os.environ["MASTER_ADDR"] = master_addr
        print(f"{master_addr=}", flush=True)
        os.environ["MASTER_PORT"] = str(port)
        print(f"{port=}", flush=True)
        if torch.cuda.is_available() and torch.cuda.device_count() >= world_size:
            backend = "rccl"
        print(f"{backend=}", flush=True)
        dist.init_process_group(backend, rank=rank, world_size=world_size)
        print(f"--> done setting up rank={rank}", flush=True)


def cleanup(rank):
    """Destroy the default process group (skipped for serial code, rank -1)."""
    if rank != -1:
        dist.destroy_process_group()


def get_batch(batch: Tuple[Tensor, Tensor], rank) -> Tuple[Tensor, Tensor]:
    x, y = batch
    if torch.cuda.is_available():
        x, y = x.to(rank), y.to(rank)
    return x, y


def _setup_and_cleanup(rank, world_size, port):
    setup_process(rank, world_size, port)
    dist.barrier()
    cleanup(rank)


def test_setup():
    print("test_setup")
    port = find_free_port()
    world_size = 4
    launch.spawn(_setup_and_cleanup, args=(world_size, port), nprocs=4, timeout=300)
    print("successful test_setup!")


if __name__ == "__main__":
    test_setup()
