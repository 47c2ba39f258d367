"""All-reduce bandwidth sweep over RCCL/xGMI.

Measures algorithm and bus bandwidth of a float32 all-reduce from 4 B to 1 GiB
(busbw = algbw * 2(W-1)/W, the per-link figure to compare with the ≈153 GB/s of
one xGMI link), for torch's ProcessGroupNCCL ("rccl") and this package's native
communicator ("rccl-native").  Also reports the DDP-relevant sizes: the 720 MB
fc bucket and the 53 KB conv/BN bucket of the 3000² ConvNet.

With ``--exchanges`` it also times the fc-gradient paths of parallel/factored.py at the bench
shape (B=5, N=10, K=18e6): the activation all-gather of X, the sharded exchange's grouped
point-to-point phases, and the 4-chunk row-segment all-reduce -- the inputs of the byte/time
model in docs/DISTRIBUTED.md.

  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_allreduce.py --backend rccl-native --exchanges
  python tools/bench_allreduce.py --gpus 2          # spawn ranks itself
  python tools/bench_allreduce.py --gpus 2 --device cpu --backend gloo --max-bytes 65536 --no-ddp-sizes  # rehearsal
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


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize()


def _time(fn, dev, iters, warmup):
    for _ in range(warmup):
        fn()
    _sync(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    _sync(dev)
    return (time.perf_counter() - t0) / iters


def _exchange_rows(dev, world, rank, args):
    """The fc-gradient paths of parallel/factored.py at B x K (per-rank bytes on the busiest link)."""
    from torch_distributed_sandbox_amd.parallel import factored

    B, N, K = args.rows, 10, args.in_features
    out = []
    x = torch.ones(B, K, device=dev)
    xg = torch.empty(world * B, K, device=dev)
    t = _time(lambda: dist.all_gather_into_tensor(xg, x), dev, args.iters, args.warmup)
    out.append({"path": "activations (all-gather X)", "us": t * 1e6,
                "link_MB": factored.link_bytes("activations", B, N, K, world) / 1e6})
    bounds = factored.shard_bounds(K, world)
    k0, k1 = bounds[rank]
    xs = torch.empty(world, B, k1 - k0, device=dev)
    sends = [(x[b, a:e], s) for s, (a, e) in enumerate(bounds) if e > a for b in range(B)]
    recvs = [(xs[s, b], s) for s in range(world) for b in range(B)]
    dw = torch.ones(N, K, device=dev)
    gs = [(dw[c, k0:k1], s) for s in range(world) if s != rank for c in range(N)]
    gr = [(dw[c, a:e], s) for s, (a, e) in enumerate(bounds) if s != rank and e > a for c in range(N)]

    def sharded():
        dist.sendrecv(sends, recvs, async_op=False)
        if gs:
            dist.sendrecv(gs, gr, async_op=False)

    t = _time(sharded, dev, args.iters, args.warmup)
    out.append({"path": "sharded (all-to-all X shards + all-gather dW shards)", "us": t * 1e6,
                "link_MB": factored.link_bytes("sharded", B, N, K, world) / 1e6})
    chunks = [(a, e) for a, e in factored.shard_bounds(K, 4) if e > a]

    def chunked():
        ws = [dist.all_reduce(dw[j, a:e], dist.ReduceOp.AVG, async_op=True) for a, e in chunks for j in range(N)]
        for w in ws:
            w.wait()

    t = _time(chunked, dev, args.iters, args.warmup)
    out.append({"path": "chunked (4 K-chunks x 10 row all-reduces)", "us": t * 1e6,
                "link_MB": factored.link_bytes("allreduce", B, N, K, world) / 1e6})
    t = _time(lambda: dist.all_reduce(dw, dist.ReduceOp.AVG), dev, args.iters, args.warmup)
    out.append({"path": "allreduce (one 720 MB bucket)", "us": t * 1e6,
                "link_MB": factored.link_bytes("allreduce", B, N, K, world) / 1e6})
    return out


def _worker(local, args):
    rank = int(os.environ.get("RANK", local))
    world = int(os.environ.get("WORLD_SIZE", args.gpus))
    on_gpu = args.device == "cuda"
    dist.init_process_group(args.backend, rank=rank, world_size=world, device_id=local if on_gpu else None,
                            comm_cus=args.comm_cus)
    dev = torch.device("cuda", local) if on_gpu else torch.device("cpu")
    rows = []
    sizes = _sizes(args.max_bytes) + ([] if args.no_ddp_sizes else sorted(DDP_SIZES.values()))
    for nbytes in sizes:
        n = max(1, nbytes // 4)
        t = torch.ones(n, device=dev)
        iters = args.iters if nbytes < (64 << 20) else max(3, args.iters // 5)
        dt = _time(lambda: dist.all_reduce(t, dist.ReduceOp.AVG), dev, iters, args.warmup)
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
    ex = _exchange_rows(dev, world, rank, args) if args.exchanges else []
    if rank == 0:
        for r in ex:
            bw = r["link_MB"] / r["us"] * 1e3 if r["us"] > 0 else 0.0
            print(f"{r['path']:<55} {r['us']:>10.1f} us  {r['link_MB']:>8.1f} MB/link  {bw:>7.2f} GB/s/link")
        rec = {"backend": args.backend, "world": world, "device": args.device, "comm_cus": dist.comm_cus(),
               "rows": rows, "exchanges": ex}
        print(json.dumps(rec))
        if args.out:
            with open(args.out, "w") as f:
                json.dump(rec, f, indent=1)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="rccl", help="rccl | rccl-native | gloo | host")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--comm-cus", type=int, default=None,
                    help="rccl-native: CUs the communicator's stream is confined to (default 32 at world > 1, "
                         "as in training; 0 = unconfined)")
    ap.add_argument("--no-ddp-sizes", action="store_true", help="skip the 720 MB / 53 KB DDP bucket sizes")
    ap.add_argument("--exchanges", action="store_true", help="also time the fc-gradient paths (factored.py)")
    ap.add_argument("--rows", type=int, default=5, help="per-rank fc rows for --exchanges (bench: 5)")
    ap.add_argument("--in-features", type=int, default=32 * 750 * 750, help="fc K for --exchanges")
    ap.add_argument("--out", default=None, help="also write the JSON record here")
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
