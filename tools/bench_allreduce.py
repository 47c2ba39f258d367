"""All-reduce bandwidth sweep over RCCL/xGMI.

Measures algorithm and bus bandwidth of a float32 all-reduce from 4 B to 1 GiB
(busbw = algbw * 2(W-1)/W, the per-link figure to compare with the ≈153 GB/s of
one xGMI link), for torch's ProcessGroupNCCL ("rccl") and this package's native
communicator ("rccl-native").  Also reports the DDP-relevant sizes: the 720 MB
fc bucket and the 53 KB conv/BN bucket of the 3000² ConvNet.

  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_allreduce.py --backend rccl-native
  python tools/bench_allreduce.py --gpus 2          # spawn ranks itself
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from torch_distributed_sandbox_amd.parallel import distributed as dist  # noqa: E402
from torch_distributed_sandbox_amd.parallel import launch  # noqa: E402

DDP_SIZES = {"fc_bucket_720MB": 180_000_010 * 4, "conv_bucket_53KB": 13_344 * 4}


def _sizes(max_bytes):
    s, out = 4, []
    while s <= max_bytes:
        out.append(s)
        s *= 4
    return out


def _worker(local, args):
    rank = int(os.environ.get("RANK", local))
    world = int(os.environ.get("WORLD_SIZE", args.gpus))
    dist.init_process_group(args.backend, rank=rank, world_size=world, device_id=local)
    dev = torch.device("cuda", local)
    rows = []
    sizes = _sizes(args.max_bytes) + sorted(DDP_SIZES.values())
    for nbytes in sizes:
        n = max(1, nbytes // 4)
        t = torch.ones(n, device=dev)
        iters = args.iters if nbytes < (64 << 20) else max(3, args.iters // 5)
        for _ in range(args.warmup):
            dist.all_reduce(t, dist.ReduceOp.AVG)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            dist.all_reduce(t, dist.ReduceOp.AVG)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / iters
        algbw = n * 4 / dt / 1e9
        busbw = algbw * (2 * (world - 1) / world if world > 1 else 1.0)
        name = [k for k, v in DDP_SIZES.items() if v == nbytes]
        rows.append({"bytes": n * 4, "us": dt * 1e6, "algbw_GBps": algbw, "busbw_GBps": busbw,
                     "tag": name[0] if name else ""})
    if rank == 0:
        print(f"# all-reduce AVG fp32, backend={args.backend}, world={world}")
        print(f"{'bytes':>12} {'time_us':>10} {'algbw GB/s':>11} {'busbw GB/s':>11}")
        for r in rows:
            print(f"{r['bytes']:>12} {r['us']:>10.1f} {r['algbw_GBps']:>11.2f} {r['busbw_GBps']:>11.2f} {r['tag']}")
        print(json.dumps({"backend": args.backend, "world": world, "rows": rows}))
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="rccl", help="rccl | rccl-native")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--max-bytes", type=int, default=1 << 30)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()
    if "LOCAL_RANK" in os.environ:
        _worker(int(os.environ["LOCAL_RANK"]), args)
    else:
        launch.setup_rendezvous_env()
        launch.spawn(_worker, args=(args,), nprocs=args.gpus)


if __name__ == "__main__":
    main()
