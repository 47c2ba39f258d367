"""DDP ConvNet trainer on 3000x3000 (synthetic) MNIST — one process per MI355X over RCCL/xGMI.

Reference: mnist_distributed.py (mp.spawn one rank per GPU, rank = nr*gpus + gpu,
DDP(model, device_ids=[gpu]), DistributedSampler, per-rank bs=5).

Usage:
  python mnist_distributed.py -n 1 -g 8 --epochs 2                  # spawn 8 ranks on this node
  torchrun --nproc-per-node 8 mnist_distributed.py -g 8             # or let torchrun launch them
  python mnist_distributed.py -n 2 -g 8 -nr 0 --master-addr HOST    # node 0 of 2 (multi-node)
  python mnist_distributed.py -g 2 --device cpu --backend gloo --image-size 64   # CPU rehearsal
"""
import argparse
import os

from torch_distributed_sandbox_amd.parallel import launch
from torch_distributed_sandbox_amd.trainer import add_common_args, train


def _train_entry(gpu, args):
    train(gpu, args, distributed=True)


def main(argv=None):
    parser = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    parser.add_argument("-n", "--nodes", default=1, type=int, metavar="N", help="number of nodes")
    parser.add_argument("-g", "--gpus", default=1, type=int, help="number of gpus (ranks) per node")
    parser.add_argument("-nr", "--nr", default=0, type=int, help="ranking within the nodes")
    parser.add_argument("--backend", default="auto",
                        help="rccl-native (auto on GPU: this package's RCCL communicator + C++ reducer, the stack "
                             "bench.py measures) | rccl/nccl (torch ProcessGroupNCCL) | gloo (auto on CPU) | host")
    parser.add_argument("--master-addr", default=None)
    parser.add_argument("--master-port", default=None)
    parser.add_argument("--avg-loss", action="store_true", help="log the global-average loss (all_reduce AVG)")
    add_common_args(parser)
    args = parser.parse_args(argv)
    args.world_size = args.gpus * args.nodes
    if "LOCAL_RANK" in os.environ and "WORLD_SIZE" in os.environ:
        # launched by torchrun: one process already per GPU
        args.world_size = int(os.environ["WORLD_SIZE"])
        local = int(os.environ["LOCAL_RANK"])
        args.nr = (int(os.environ["RANK"]) - local) // max(1, args.gpus)
        return train(local, args, distributed=True)
    if args.nodes > 1 and args.master_addr is None and "MASTER_ADDR" not in os.environ:
        parser.error("multi-node runs need --master-addr (or MASTER_ADDR) reachable from every node")
    if args.nodes > 1 and args.master_port is None and "MASTER_PORT" not in os.environ:
        parser.error("multi-node runs need the same --master-port on every node")
    launch.setup_rendezvous_env(args.master_addr, args.master_port)
    launch.spawn(_train_entry, args=(args,), nprocs=args.gpus)


if __name__ == "__main__":
    main()
