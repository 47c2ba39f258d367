"""All-reduce toy: every rank contributes a random int per step; ranks 0 and 1 print the sum.

Reference: allreduce_toy.py (spawn N ranks; per step new_group + int32 all_reduce(SUM)
+ barrier; ranks 0/1 print 'rank: R, step: S, value: V, reduced sum: X.').
Fixes: --backend, --steps, --init-method and --rank are honoured (the
reference parses and ignores them); groups are cached, not re-created per step.

Usage:
  python allreduce_toy.py -s 2 --backend gloo            # CPU, no GPU needed
  python allreduce_toy.py -s 8 --backend rccl-native     # one rank per MI355X, native RCCL communicator
  python allreduce_toy.py -s 8 --backend rccl            # torch's ProcessGroupNCCL (RCCL)
  python allreduce_toy.py -s 2 -r 0 -i tcp://HOST:PORT   # run one rank by hand (multi-node)
"""
import argparse
import os
from random import randint

import torch

from torch_distributed_sandbox_amd.parallel import distributed as dist
from torch_distributed_sandbox_amd.parallel import launch

find_free_port = launch.find_free_port


def _device_for(backend, rank):
    # the device backends (torch's RCCL process group and this package's rccl-native
    # communicator) all-reduce a tensor on cuda:{rank}, as the reference does (allreduce_toy.py:30)
    if dist.is_device_backend(backend):
        return torch.device("cuda", rank % torch.cuda.device_count())
    return torch.device("cpu")


def run(world_size, rank, steps, backend="rccl"):
    device = _device_for(backend, rank)
    for step in range(1, steps + 1):
        value = randint(0, 10)
        group = dist.new_group(ranks=list(range(world_size)))
        tensor = torch.tensor(value, dtype=torch.int).to(device)
        dist.all_reduce(tensor, op=dist.ReduceOp.SUM, group=group)
        dist.barrier()
        if rank in (0, 1):
            print("rank: {}, step: {}, value: {}, reduced sum: {}.".format(rank, step, value, tensor.item()),
                  flush=True)


def setup(rank, world_size, backend="rccl", steps=20, init_method=None):
    if rank != -1:  # -1 rank indicates serial code
        dist.init_process_group(backend, init_method=init_method, rank=rank, world_size=world_size)
        print(f"--> done setting up rank={rank}", flush=True)
        run(world_size, rank, steps, backend)
        dist.barrier()
        dist.destroy_process_group()


def main(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument("--backend", type=str, default="auto",
                        help="rccl-native (this package's RCCL communicator; auto on GPU) | rccl/nccl (torch "
                             "ProcessGroupNCCL) | gloo (auto on CPU) | host (this package's TCP ring)")
    parser.add_argument("-i", "--init-method", type=str, default=None,
                        help="URL specifying how to initialize the package (default: env:// with a free port)")
    parser.add_argument("-s", "--world_size", type=int, default=2, help="Number of processes participating in the job.")
    parser.add_argument("-r", "--rank", type=int, default=None,
                        help="Run only this rank in this process (needs -i or MASTER_ADDR/MASTER_PORT)")
    parser.add_argument("--steps", type=int, default=20)
    args = parser.parse_args(argv)
    if args.rank is not None:
        if args.init_method is None and "MASTER_PORT" not in os.environ:
            parser.error("--rank needs --init-method or MASTER_ADDR/MASTER_PORT shared by all ranks")
        setup(args.rank, args.world_size, args.backend, args.steps, args.init_method)
        return
    if args.init_method is None:
        launch.setup_rendezvous_env("127.0.0.1", find_free_port())
    launch.spawn(setup, args=(args.world_size, args.backend, args.steps, args.init_method), nprocs=args.world_size)


if __name__ == "__main__":
    main()
