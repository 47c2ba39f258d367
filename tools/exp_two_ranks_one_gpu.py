"""Experiment: can two ranks share one GPU with the native RCCL communicator?
(Used to rehearse multi-rank device collectives on a one-GPU box.)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from torch_distributed_sandbox_amd.parallel import distributed as dist  # noqa: E402
from torch_distributed_sandbox_amd.parallel import launch  # noqa: E402


def w(rank, backend):
    dist.init_process_group(backend, rank=rank, world_size=2, device_id=0)
    t = torch.full((1 << 20,), float(rank + 1), device="cuda:0")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    print(f"rank {rank} {backend} allreduce -> {t[0].item()}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    launch.setup_rendezvous_env()
    launch.spawn(w, args=(sys.argv[1] if len(sys.argv) > 1 else "rccl-native",), nprocs=2, timeout=90)
