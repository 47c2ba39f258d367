"""Headline benchmark: images/sec (whole node) of the 3000x3000 MNIST ConvNet under DDP.

BASELINE.json metric/config: ConvNet (mnist_onegpu.py:11-31), 3000x3000 inputs,
per-rank batch 5, SGD(lr=1e-4), CrossEntropy, one process per MI355X over
RCCL/xGMI, synthetic data + random init (no network for MNIST).

    python bench.py                                  # 1 GPU, default steps
    python bench.py --gpus 8 --steps 20 --warmup 5   # spawns 8 ranks itself
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P bench.py --gpus N --steps K --warmup W

Launch: like the reference (``mp.spawn(train, nprocs=args.gpus)``,
mnist_distributed.py:123-127) ``--gpus N`` with no ``WORLD_SIZE`` in the
environment starts N rank processes itself (spawn start method) before the
parent touches the GPU, and exits with the first failing rank's status.  Under
torchrun (``WORLD_SIZE`` set) it runs as that rank.

A timed step is the full training step: on-device data generation (28x28
uint8 -> 3000x3000 bilinear upsample), forward, loss, zero_grad, backward
(with the gradient exchange), optimizer step.  W untimed warmup steps, then
exactly K steps bracketed by barrier + synchronize; the elapsed time is the
MAX over ranks.  Rank 0 prints one JSON line.

Default multi-GPU stack: this package's RCCL communicator (``rccl-native``:
own comm stream, non-blocking init with a bounded wait, watchdog) and the C++
gradient reducer; ``--backend rccl`` selects torch's ProcessGroupNCCL instead.

Failure handling (a multi-GPU run must succeed or explain itself inside the
driver's 600 s lease):

* every wait is bounded below the lease: rendezvous / communicator init /
  collectives by ``--pg-timeout`` (default 120 s), the whole rank by
  ``--deadline`` (default 540 s from process start), the self-spawned job by
  ``--spawn-timeout`` (default 570 s);
* on any failure exactly one JSON line still comes out, with ``"value": null``,
  ``"status": "failed"``, the failing rank, its error and the exit status;
* preflight (world > 1): before the warmup, every collective the step will use
  (buffer broadcast, bucket all-reduces, the fc path's all-gathers / grouped
  point-to-point exchanges at their real sizes) runs once on the live
  communicator with a bounded wait; times and bus bandwidths are reported in
  ``config.preflight`` -- a broken link fails the attempt there, named;
* fallback tiers (``--fallback``, default on when no ``--backend`` was given):
  if an attempt fails on any rank, all ranks agree through the rendezvous store,
  tear it down and run again inside the same processes (nothing is re-exec'd):
  1. ``rccl-native`` + CU split + the fc exchange picked by ``auto``;
  2. torch's ProcessGroupNCCL (RCCL), no CU split, the SAME fc exchange;
  3. torch's ProcessGroupNCCL with the plain 720 MB bucket all-reduce;
  labelled ``"backend": "rccl (fallback: <reason>)"`` and ``"tier": "k/n"``.  A
  self-spawned job whose rank crashed is re-spawned once from tier 2, with fresh
  child processes, by the parent (which never touched the GPU).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

_T_START = time.time()  # process start (the --deadline clock)

METRIC = "images/sec (whole node), 3000x3000 MNIST ConvNet DDP at 1/2/4/8 MI355X"
MODEL = "ConvNet(conv5x5 1->16+BN+ReLU+pool2, conv5x5 16->32+BN+ReLU+pool2, fc 32*(H/4)^2->10)"
DATA = ("synthetic (seeded 28x28 uint8 sources upsampled on device to HxW, a fresh batch every step -- no batch "
        "repeats within the run; random labels; random init)")
DTYPE_TF32 = ("fp32 (conv2 fwd+dgrad+wgrad: TF32-class -- one fp16 MFMA per product, both operands rounded to 11 "
              "significant bits = TF32's significand, exact power-of-two range scaling, fp32 accumulate: the arithmetic "
              "of the reference's default cuDNN TF32 convolutions; conv1 fwd+wgrad: bf16x3 split MFMA (~2^-16); BN, fc, "
              "CE, SGD: fp32; stored in fp16 at exact power-of-two scales (11 significant bits): the conv2 output the "
              "backward re-reads (y2h; BN2 statistics and argmax from fp32) and its value at each pooling window's argmax "
              "that the head reads (ya, the same fp16 value), the pooled gradient "
              "entering the BN2 backward (g2m; its statistics from fp32) and the conv2 data gradient (dp1h) -- "
              "docs/KERNELS.md 'y2h', 'ya', 'g2m', 'dp1h')")


def _dtype(on_gpu: bool = True) -> str:
    """The compute precision of the GPU plan (csrc/kernels/conv2_common.h)."""
    if not on_gpu:
        return "fp32 (CPU rehearsal: torch ops)"
    try:
        import torch_distributed_sandbox_amd as tds

        tds._ext.ops()
        return DTYPE_TF32
    except Exception:  # noqa: BLE001 -- CPU rehearsal without the extension: the torch-ops plan
        return "fp32 (CPU rehearsal: torch ops)"


def _parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--image-size", type=int, default=3000)
    ap.add_argument("--batch-size", type=int, default=5, help="per-rank batch (reference: 5)")
    ap.add_argument("--mode", default="auto", choices=["auto", "fused", "layers"])
    ap.add_argument("--bucket-mb", type=float, default=None)
    ap.add_argument("--backend", default=os.environ.get("TDS_BENCH_BACKEND"),
                    help="rccl-native (default on GPU: this package's C++ RCCL communicator + C++ reducer) | "
                         "rccl (torch ProcessGroupNCCL = RCCL) | gloo | host")
    ap.add_argument("--grad-exchange", default="auto",
                    choices=["auto", "allreduce", "activations", "sharded", "chunked"],
                    help="fc gradient path under DDP (parallel/factored.py); auto picks by the xGMI byte model")
    ap.add_argument("--exchange-compress", action=argparse.BooleanOptionalAction, default=True,
                    help="send the activation exchange's fc input rows zero-suppressed (lossless, parallel/zs.py)")
    ap.add_argument("--exchange-source", choices=["pooled", "rows"], default="pooled",
                    help="what the activation exchange gathers: the fused head's pooled input ya (fp16) and "
                         "128 head constants per rank (pooled), or the fc input rows X (rows, zero-suppressed)")
    ap.add_argument("--exchange-groups", type=int, default=None,
                    help="column groups of the zero-suppressed activation exchange (one head launch, encode and "
                         "gather pair each; default 4 at world > 1, 1 at world 1)")
    ap.add_argument("--allreduce-chunks", type=int, default=None,
                    help="K-chunks of the fc weight gradient in the all-reduce regime (default 4 on GPU)")
    ap.add_argument("--reserve-cus", type=int, default=None,
                    help="keep N CUs (a multiple of 32) out of the compute stream and confine the native "
                         "communicator's stream to them (utils/streams.py); default 32 at world > 1 on "
                         "rccl-native, else 0")
    ap.add_argument("--rccl-max-ctas", type=int, default=0,
                    help="bound RCCL's workgroups per collective (ncclConfig maxCTAs; TDS_RCCL_MAX_CTAS); "
                         "default: the reserved CU count on rccl-native")
    ap.add_argument("--overlap-optimizer", action=argparse.BooleanOptionalAction, default=True,
                    help="finish the fc bucket (collective + SGD) on a side stream under the next forward's convs")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: rehearsal of the launch/exchange path on the torch-ops plan (small --image-size)")
    ap.add_argument("--shared-device", action="store_true",
                    help="rehearsal only: every rank uses cuda:0 (needs --backend gloo); recorded in the JSON")
    ap.add_argument("--input", default="levels", choices=["levels", "fp32"],
                    help="how each step's batch reaches the model: 'levels' = the resized images' uint8 levels "
                         "(ToTensor's 1/255 folded into conv1 by the fused plan, models/convnet.py to_image), "
                         "'fp32' = the ToTensor image materialised by the upsample kernel")
    ap.add_argument("--fused-input-moments", action=argparse.BooleanOptionalAction, default=True,
                    help="levels input, fused plan: the upsample kernel also forms the batch's x autocorrelation "
                         "partials behind BN1's statistics (ops.functional.upsample_levels_moments); off: the "
                         "layer-1 forward forms them from the written image")
    ap.add_argument("--fused-ce", action=argparse.BooleanOptionalAction, default=True,
                    help="fused plan: the batch's labels go with it, and the head forward's finalizing workgroup "
                         "forms the cross-entropy loss and dlogits with the logits (no separate CE launch)")
    ap.add_argument("--prefetch", action=argparse.BooleanOptionalAction, default=False,
                    help="produce the next batch (upsample + BN1 input moments) on a side stream beside the "
                         "current step's head kernels (--prefetch-at)")
    ap.add_argument("--prefetch-at", choices=["head", "conv2_bwd"], default="head",
                    help="where --prefetch queues the next batch: beside the head forward / backward (memory-"
                         "bound, room for the pipeline's workgroups) or beside the conv2 backward (round 2: no room)")
    ap.add_argument("--allreduce-probe", action=argparse.BooleanOptionalAction, default=True,
                    help="world > 1: after the timed steps, time a few all-reduces over the same communicator "
                         "and report their bus bandwidth in config.allreduce_probe (outside the timed region)")
    ap.add_argument("--sim-comm-us", type=int, default=0,
                    help="1-GPU rehearsal of a collective's CU footprint: after each forward, hold "
                         "--sim-comm-ctas workgroups of RCCL's size (256 threads, 19.7 KB LDS) for this many "
                         "microseconds on a side stream (recorded in the JSON; not a training number)")
    ap.add_argument("--sim-comm-ctas", type=int, default=16)
    ap.add_argument("--sim-sdma-mb", type=float, default=0.0,
                    help="rehearsal on one GPU: after each forward, copy this many MB device-to-device on a side "
                         "stream beside the backward (the fc exchange's bulk payload), joined at the step's end")
    ap.add_argument("--sim-sdma-engine", default="nocu", choices=["nocu", "blit"],
                    help="--sim-sdma-mb copy by the copy engines (hipMemcpyDeviceToDeviceNoCU) or the blit kernel")
    ap.add_argument("--spawn-timeout", type=float, default=570.0,
                    help="self-spawn: terminate all ranks if the job runs longer than this (s)")
    ap.add_argument("--pg-timeout", type=float, default=120.0,
                    help="rendezvous, communicator init and per-collective timeout (s)")
    ap.add_argument("--deadline", type=float, default=540.0,
                    help="a rank still running this long after its start prints the failure record and exits (s)")
    ap.add_argument("--preflight", action=argparse.BooleanOptionalAction, default=True,
                    help="world > 1: before the warmup, run every collective the step uses once on the live "
                         "communicator, each with a bounded wait (--preflight-timeout); the times and bus "
                         "bandwidths go to config.preflight")
    ap.add_argument("--preflight-timeout", type=float, default=60.0)
    ap.add_argument("--step-times", action="store_true",
                    help="record each timed step's GPU time with events (config.step_ms; diagnostics)")
    ap.add_argument("--lr", type=float, default=1e-4, help="SGD learning rate (reference: 1e-4)")
    ap.add_argument("--transport-tune", action=argparse.BooleanOptionalAction, default=None,
                    help="before the model is built, time the fc exchange's collectives at each candidate "
                         "(reserve-cus, rccl-max-ctas) on the live node and take the one with the lowest predicted "
                         "step time (parallel/transport_tune.py; config.preflight.transport).  Off by default: "
                         "its communicator re-creation crashed a one-GPU run (r6_s4), see docs/DISTRIBUTED.md")
    ap.add_argument("--store", default="native", choices=["native", "c10d"],
                    help="rendezvous store (world > 1 or a forced exchange): this package's C++ TCP store, located "
                         "through c10d's at MASTER_ADDR:MASTER_PORT (the agreed fallback), or c10d's only; "
                         "TDS_STORE overrides.  The torch-RCCL fallback tiers always use c10d's")
    ap.add_argument("--fallback", action=argparse.BooleanOptionalAction, default=None,
                    help="after a failed rccl-native attempt, run once more on torch's RCCL process group with "
                         "the plain bucket all-reduce (default: on unless --backend is given)")
    return ap


def _rank_entry(i: int, argv, world: int, master_addr: str, master_port: str, fallback_reason):
    os.environ.update({"RANK": str(i), "LOCAL_RANK": str(i), "WORLD_SIZE": str(world),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": master_addr, "MASTER_PORT": master_port,
                       "TDS_BENCH_CHILD": "1"})  # the spawning parent prints any failure record
    if fallback_reason:
        os.environ["TDS_BENCH_FALLBACK_REASON"] = fallback_reason
    rc = run_rank(argv)
    if rc:
        sys.exit(rc)


def _short(err: str, n: int = 400) -> str:
    """The last meaningful line(s) of an error / traceback, bounded."""
    lines = [ln.strip() for ln in str(err).strip().splitlines() if ln.strip()]
    tail = " | ".join(lines[-2:]) if lines else str(err)
    return tail[-n:]


def _fail_record(args, world: int, failed_rank, error: str, rc: int, extra=None) -> dict:
    cfg = {"model": MODEL, "global_batch": world * args.batch_size, "per_rank_batch": args.batch_size,
           "seq_len": None, "image_size": [args.image_size, args.image_size], "parallelism": f"dp{world}"}
    cfg.update(extra or {})
    return {"metric": METRIC, "value": None, "unit": "images/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": _dtype(args.device == "cuda"), "data": DATA, "status": "failed", "failed_rank": failed_rank,
            "error": error, "rc": rc, "elapsed_s": round(time.time() - _T_START, 1), "config": cfg}


def _spawn_ranks(args, argv) -> int:
    """One process per GPU, started here (no GPU call happens in this parent).  If the job
    fails (a rank raised, crashed or timed out) and no --backend was forced, it is re-spawned
    ONCE with fresh rank processes on torch's RCCL process group with the plain bucket
    all-reduce; if that fails too (or there is no time left) one failure record is printed."""
    import tempfile

    from torch_distributed_sandbox_amd.parallel import launch

    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    fallback = args.fallback if args.fallback is not None else args.backend is None
    plans = [(list(argv), None)]
    if fallback and args.device == "cuda":
        # torch's RCCL process group, no CU split, same fc path; its own in-process fallback is
        # the plain bucket all-reduce
        plans.append((list(argv) + ["--backend", "rccl", "--reserve-cus", "0", "--fallback"], "retry"))
    fail = None
    port_retried = False
    for k, (av, label) in enumerate(plans):
        remaining = args.spawn_timeout - (time.time() - _T_START)
        if k > 0 and remaining < 90:
            break
        port = (os.environ.get("MASTER_PORT") if k == 0 else None) or launch.find_free_port(addr)
        reason = None if label is None else f"rank {fail[0]} of the first spawn: {fail[1]}"
        with tempfile.TemporaryDirectory(prefix="tds_bench_") as td:
            os.environ["TDS_BENCH_RESULT_FILE"] = os.path.join(td, "result.json")
            try:
                launch.spawn(_rank_entry, args=(av, args.gpus, addr, str(port), reason), nprocs=args.gpus,
                             timeout=max(30.0, remaining))
                return 0
            except launch.ProcessRaisedException as e:
                fail = (e.error_index, _short(str(e)), 1)
            except launch.ProcessExitedException as e:
                fail = (e.error_index, str(e), e.exit_code if e.exit_code and e.exit_code > 0 else 1)
            except TimeoutError as e:
                fail = (None, str(e), 124)
            finally:
                printed = os.path.exists(os.environ.pop("TDS_BENCH_RESULT_FILE"))
            print(f"bench.py: spawn attempt {k} failed: rank {fail[0]}: {fail[1]}", file=sys.stderr, flush=True)
            if printed:  # rank 0 already printed the measurement; the failure came after it (teardown)
                return 0
            if "address already in use" in str(fail[1]).lower() and not port_retried:
                # the rendezvous port was taken between its probe and the store's bind: the same
                # plan once more on a fresh port
                port_retried = True
                plans.insert(k + 1, (av, label))
                os.environ.pop("MASTER_PORT", None)
    print(json.dumps(_fail_record(args, args.gpus, fail[0], fail[1], fail[2],
                                  {"spawn_attempts": len(plans) if fallback and args.device == "cuda" else 1})),
          flush=True)
    return fail[2]


def _allreduce_probe(tdist, device, world, on_gpu):
    """All-reduce (SUM) bus bandwidth over the bench's own communicator, after the timed steps:
    the xGMI numbers behind the step time (busbw = 2 (W-1)/W x bytes / time, the ring volume per
    link).  Sizes: a conv/BN-sized bucket, a mid bucket, and the 720 MB fc gradient on GPU."""
    sizes = [4 << 20, 64 << 20, 720_000_040] if on_gpu else [1 << 20]
    out = []
    for nbytes in sizes:
        t = torch.ones(nbytes // 4, device=device, dtype=torch.float32)
        iters = 5 if on_gpu else 2
        for _ in range(2):
            tdist.all_reduce(t)
        if on_gpu:
            torch.cuda.synchronize(device)
        tdist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            tdist.all_reduce(t)
        if on_gpu:
            torch.cuda.synchronize(device)
        dt = (time.perf_counter() - t0) / iters
        g = torch.tensor([dt], device=device, dtype=torch.float64)
        tdist.all_reduce(g, tdist.ReduceOp.MAX)
        dt = float(g.item())
        out.append({"MB": round(nbytes / 1e6, 3), "ms": round(dt * 1e3, 3),
                    "busbw_GBps": round(2 * (world - 1) / world * nbytes / dt / 1e9, 2)})
        del t
    return out


_BUS = {  # bytes on the busiest link per byte counted (nccl-tests "busbw" conventions)
    "all_reduce": lambda w: 2.0 * (w - 1) / w,   # nbytes = the buffer
    "all_gather": lambda w: (w - 1) / w,         # nbytes = the gathered output
    "broadcast": lambda w: 1.0,
    "sendrecv": lambda w: 1.0,                   # nbytes = what one peer link carries
}


def _preflight(ddp, tdist, device, world: int, rank: int, rows: int, timeout_s: float):
    """Run every collective the step will use once (``DistributedDataParallel.preflight``: the
    buffer broadcast, the reducer's bucket all-reduces, the fc path's gathers / point-to-point
    exchanges at their real sizes) on the live communicator and its streams, before any model
    work.  Each gets a bounded wait: its completion event is polled on the host and a collective
    still running after ``timeout_s`` raises, so a broken link, a missing peer or a collective
    the backend cannot run fails the attempt here -- named -- instead of mid-warmup.  Returns
    [{"op", "MB", "ms", "busbw_GBps"}] (the second of two runs of each; the first pays RCCL's
    lazy channel setup) and the fc path."""
    from torch_distributed_sandbox_amd.utils import fault

    on_gpu = device.type == "cuda"
    out = []

    def wait_bounded(name, work, t0):
        if work is not None:
            work.wait()  # RCCL: the current stream waits on the device; gloo/host: on the host
        if not on_gpu:
            return
        ev = torch.cuda.Event()
        ev.record()
        while not ev.query():
            if time.perf_counter() - t0 > timeout_s:
                raise TimeoutError(f"preflight: {name} did not complete within {timeout_s:.0f} s on rank {rank}")
            time.sleep(2e-4)

    def timed(name, nbytes, kind, issue):
        best = None
        for _ in range(2):
            fault.maybe_inject_bench(rank, "preflight")
            t0 = time.perf_counter()
            wait_bounded(name, issue(), t0)
            best = time.perf_counter() - t0
        out.append({"op": name, "MB": round(nbytes / 1e6, 3), "ms": round(best * 1e3, 3),
                    "busbw_GBps": round(_BUS[kind](world) * nbytes / best / 1e9, 2)})

    info = ddp.preflight(rows, timed)
    t0 = time.perf_counter()
    tdist.barrier()
    out.append({"op": "barrier", "MB": 0.0, "ms": round((time.perf_counter() - t0) * 1e3, 3), "busbw_GBps": None})
    return out, info["fc_path"]


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else list(argv)
    args = _parser().parse_args(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return _spawn_ranks(args, argv)
    return run_rank(argv)


def run_rank(argv) -> int:
    """One rank: the attempts (rccl-native, then the torch-RCCL fallback), bounded by the
    --deadline watchdog.  Rank 0 prints exactly one JSON line -- the measurement or, unless a
    spawning parent reports for it, the failure record."""
    import threading

    args = _parser().parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    child = os.environ.get("TDS_BENCH_CHILD") == "1"
    phase = ["start"]
    done = threading.Event()

    def watchdog():
        left = args.deadline - (time.time() - _T_START)
        if done.wait(max(0.0, left)):
            return
        msg = f"rank {rank} still running {args.deadline:.0f} s after its start (phase: {phase[0]})"
        print(f"bench.py: {msg}; exiting", file=sys.stderr, flush=True)
        if rank == 0 and not child:
            print(json.dumps(_fail_record(args, world, rank, msg, 124)), flush=True)
        os._exit(124)

    threading.Thread(target=watchdog, daemon=True, name="bench-deadline").start()
    try:
        rec = _run_attempts(args, world, rank, phase)
    except BaseException as e:  # noqa: BLE001 -- reported, then re-raised for the exit status
        msg = f"{type(e).__name__}: {_short(str(e))}"
        print(f"bench.py: rank {rank} failed in phase {phase[0]}: {msg}", file=sys.stderr, flush=True)
        if rank == 0 and not child:
            print(json.dumps(_fail_record(args, world, rank, msg, 1, {"phase": phase[0]})), flush=True)
        done.set()
        if child:
            raise
        return 1
    done.set()
    if rank == 0 and rec is not None:
        line = json.dumps(rec)
        path = os.environ.get("TDS_BENCH_RESULT_FILE")
        if path:
            with open(path, "w") as f:
                f.write(line + "\n")
        print(line, flush=True)
    return 0


def _make_store(args, rank: int, world: int):
    """The rendezvous store every attempt shares (each attempt under its own prefix), so the
    ranks can agree on a fallback even when a communicator could not be created: this package's
    C++ store (parallel/store.py ``rendezvous``; c10d's TCPStore at MASTER_ADDR:MASTER_PORT only
    locates it, and replaces it on every rank if some rank cannot use it).  Returns (store, kind,
    c10d store): the last one carries the rendezvous of the torch-RCCL fallback tiers, which run
    torch's stack top to bottom."""
    import datetime

    from torch_distributed_sandbox_amd.parallel.store import rendezvous

    from torch_distributed_sandbox_amd.parallel import launch

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    own_port = "MASTER_PORT" not in os.environ and world == 1
    if "MASTER_PORT" not in os.environ:
        # one process (a forced exchange at world 1): nobody else needs to agree on the port, so a
        # free one -- a fixed default collided with the previous run's socket (EADDRINUSE, r6_s4)
        os.environ["MASTER_PORT"] = launch.find_free_port(os.environ["MASTER_ADDR"]) if world == 1 else "29533"
    for attempt in range(3):
        try:
            store, kind = rendezvous(rank, world, timeout=datetime.timedelta(seconds=args.pg_timeout),
                                     prefer=os.environ.get("TDS_STORE") or args.store)
            break
        except Exception as e:  # noqa: BLE001 -- only a lost race for our own free port is retried
            # the port found free was taken before the locator bound it (r6_s27: the native store's
            # own ephemeral listener can draw the port just released): a world-1 run picks another
            if not (own_port and attempt < 2 and "address already in use" in str(e).lower()):
                raise
            os.environ["MASTER_PORT"] = launch.find_free_port(os.environ["MASTER_ADDR"])
    return store, kind, getattr(store, "_locator", store)


def _run_attempts(args, world: int, rank: int, phase):
    import datetime
    import gc

    import torch.distributed as dist

    on_gpu = args.device == "cuda"
    from torch_distributed_sandbox_amd.parallel.distributed import default_backend

    backend = args.backend or default_backend(on_gpu)
    fallback = args.fallback if args.fallback is not None else (args.backend is None and on_gpu)
    label = None
    if os.environ.get("TDS_BENCH_FALLBACK_REASON"):
        label = f"{backend} (fallback: {os.environ['TDS_BENCH_FALLBACK_REASON']})"
    attempts = [(backend, args.grad_exchange, args.reserve_cus, label)]
    # fallback tiers: torch's own process group (RCCL on the GPU, gloo on a CPU rehearsal)
    # with no CU split, first keeping the fc gradient path (the zero-suppressed exchange runs on
    # ProcessGroupNCCL's all_gather_into_tensor / batch_isend_irecv too), then -- last resort --
    # the plain 720 MB bucket all-reduce
    plain = "rccl" if on_gpu else "gloo"
    if fallback and world > 1:
        for tier in ((plain, args.grad_exchange, 0, None), (plain, "allreduce", 0, None)):
            if all((a[0], a[1]) != tier[:2] for a in attempts):
                attempts.append(tier)
    dist_needed = world > 1 or args.grad_exchange in ("activations", "sharded", "chunked")
    store, store_kind, c10d_store = _make_store(args, rank, world) if dist_needed else (None, None, None)
    # a collective that stalls raises (after --pg-timeout) instead of killing the rank, so the
    # ranks can still agree on the fallback and report
    os.environ.setdefault("TDS_RCCL_ERROR_HANDLING", "raise")
    os.environ.setdefault("TDS_RCCL_INIT_TIMEOUT_MS", str(int(args.pg_timeout * 1000)))
    tune = bool(args.transport_tune)
    transport = None
    if tune and backend == "rccl-native" and on_gpu and store is not None:
        phase[0] = "transport tune"
        transport = _tune_transport(args, store, rank, world)
        ch = transport.get("chosen")
        if ch is not None:
            attempts[0] = (attempts[0][0], attempts[0][1], ch["reserve_cus"], attempts[0][3])
            if ch["max_ctas"] > 0:
                os.environ["TDS_RCCL_MAX_CTAS"] = str(ch["max_ctas"])
            else:
                os.environ.pop("TDS_RCCL_MAX_CTAS", None)
    reason = None
    for k, (be, gx, reserve, lab) in enumerate(attempts):
        if reason is not None:
            lab = f"{be} (fallback: {reason})"
        last = k == len(attempts) - 1
        ok, err, rec = True, None, None
        try:
            # torch's own process group (the fallback tiers) rendezvouses on c10d's store
            st, st_kind = (c10d_store, "c10d") if be == "rccl" and store is not None else (store, store_kind)
            rec = _attempt(args, world, rank, be, gx, reserve, lab, st, k, phase)
            if rec is not None:
                rec["config"]["store"] = st_kind
                if transport is not None:
                    rec["config"].setdefault("preflight", {})["transport"] = transport
        except Exception as e:  # noqa: BLE001
            ok, err = False, f"{type(e).__name__}: {_short(str(e))}"
            if last:
                raise
            del e
        if rec is not None:
            rec["config"]["tier"] = f"{k + 1}/{len(attempts)}"
        if store is None or len(attempts) == 1:
            if store is not None:
                # the communicator goes down here, not in the static destructors at exit (under
                # rocprofv3 those ran after the runtime's own teardown and crashed the process)
                _teardown(abort=False)
            return rec
        # every rank reports its attempt; all take the same decision
        phase[0] = f"vote after attempt {k}"
        store.set_timeout(datetime.timedelta(seconds=2 * args.pg_timeout + 30))
        store.set(f"bench/vote{k}/{rank}", "ok" if ok else ("fail " + err)[:600])
        votes = [store.get(f"bench/vote{k}/{r}").decode(errors="replace") for r in range(world)]
        bad = [(r, v[5:]) for r, v in enumerate(votes) if v != "ok"]
        # name the root cause: a rank that failed by itself before one that timed out waiting for it
        bad.sort(key=lambda rv: ("timed out" in rv[1] or "timeout" in rv[1].lower(), rv[0]))
        if not bad:
            _teardown(abort=False)
            return rec
        if last:
            raise RuntimeError(f"rank {bad[0][0]} failed: {bad[0][1]}")
        reason = f"rank {bad[0][0]}: {bad[0][1]}"[:300]
        print(f"bench.py: rank {rank}: attempt {k} ({be}) failed ({reason}); falling back", file=sys.stderr,
              flush=True)
        rec = None
        _teardown(abort=True)
        gc.collect()
        if on_gpu:
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
    return None


def _tune_transport(args, store, rank: int, world: int) -> dict:
    """parallel/transport_tune.py on the live node: for each candidate (reserve_cus, max_ctas), a
    process group on this package's communicator with that split, the collectives the step's fc
    exchange will issue at their real sizes (the path ``auto`` picks, zero-suppressed at the
    expected ratio) timed -- max over ranks -- then torn down.  Rank 0's choice is everyone's."""
    import datetime

    import torch.distributed as dist

    from torch_distributed_sandbox_amd.parallel import distributed as tdist
    from torch_distributed_sandbox_amd.parallel import transport_tune as TT

    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local_rank)
    K = 32 * (args.image_size // 4) ** 2
    # (the pooled exchange moves ya in fp16: half the dense rows; the zero-suppressed rows ~0.6)
    path, colls = TT.step_collectives(max(2, world), args.batch_size, 10, K,
                                      x_ratio=0.5 if args.exchange_source == "pooled" else 0.6)
    n_probe = [0]

    def measure(cfg):
        i = n_probe[0]
        n_probe[0] += 1
        saved = os.environ.get("TDS_RCCL_MAX_CTAS")
        if cfg.max_ctas > 0:
            os.environ["TDS_RCCL_MAX_CTAS"] = str(cfg.max_ctas)
        else:
            os.environ.pop("TDS_RCCL_MAX_CTAS", None)
        try:
            tdist.init_process_group("rccl-native", rank=rank, world_size=world,
                                     store=dist.PrefixStore(f"tune{i}", store),
                                     timeout=datetime.timedelta(seconds=args.pg_timeout), device_id=local_rank,
                                     comm_cus=cfg.reserve_cus)
            issue = []
            try:
                for kind, nbytes in colls:
                    n = max(1, nbytes // 4)
                    if kind == "all_gather":
                        inp = torch.ones(n, device=dev)
                        out = torch.empty(world * n, device=dev)
                        issue.append(lambda out=out, inp=inp: tdist.all_gather_into_tensor(out, inp))
                    elif kind == "sendrecv":
                        sb = [torch.ones(n, device=dev) for _ in range(world)]
                        rb = [torch.empty(n, device=dev) for _ in range(world)]
                        peers = [r for r in range(world) if r != rank]
                        issue.append(lambda sb=sb, rb=rb, peers=peers: tdist.sendrecv(
                            [(sb[r], r) for r in peers], [(rb[r], r) for r in peers]).wait())
                    else:
                        t = torch.ones(n, device=dev)
                        issue.append(lambda t=t: tdist.all_reduce(t, tdist.ReduceOp.AVG))
                best = None
                for _ in range(3):  # the first pays RCCL's lazy channel setup
                    tdist.barrier()
                    torch.cuda.synchronize(dev)
                    t0 = time.perf_counter()
                    for f in issue:
                        f()
                    torch.cuda.synchronize(dev)
                    dt = time.perf_counter() - t0
                    best = dt if best is None else min(best, dt)
                g = torch.tensor([best], device=dev, dtype=torch.float64)
                tdist.all_reduce(g, tdist.ReduceOp.MAX)
                res_ms = float(g.item()) * 1e3
                del g
                return res_ms
            finally:
                # the probe's buffers were used on the communicator's CU-masked stream: free them
                # (the caching allocator records an event on every stream a block was used on)
                # while that stream exists -- after the teardown releases it, that free is a
                # use-after-free of the stream (r6_s4: a segfault in the second candidate)
                issue.clear()
                # (the loop's last buffers, and the last issued lambda's defaults: r6_s5's faulthandler
                # trace put the crash at measure()'s return, where those locals are freed)
                inp = out = sb = rb = t = f = None  # noqa: F841
                torch.cuda.synchronize(dev)
                import gc

                gc.collect()
                torch.cuda.empty_cache()
                _teardown(abort=False)
        finally:
            if saved is None:
                os.environ.pop("TDS_RCCL_MAX_CTAS", None)
            else:
                os.environ["TDS_RCCL_MAX_CTAS"] = saved
            torch.cuda.empty_cache()

    res = TT.choose(measure)
    res["path"] = path
    res["bytes_per_rank"] = [b for _, b in colls]
    # one decision for all ranks (a candidate may fail on one rank only)
    if rank == 0:
        store.set("bench/transport", json.dumps(res))
    else:
        res = json.loads(store.get("bench/transport").decode())
    return res


def _teardown(abort: bool) -> None:
    from torch_distributed_sandbox_amd.parallel import distributed as tdist
    from torch_distributed_sandbox_amd.parallel.rccl_backend import native_comm_of

    if not tdist.is_initialized():
        return
    split = tdist.comm_cus() > 0
    if abort:
        comm, kind = native_comm_of(None)
        if kind == "rccl":
            comm.abort("bench fallback")
    else:
        tdist.barrier()
    tdist.destroy_process_group()
    if split:
        # the communicator's CU-masked streams end with it, not at process exit (utils/streams.py).
        # The DDP wrapper's reference cycles still hold the native communicator (through its C++
        # reducer) until a collection: free it first -- its tensors were used on the comm stream,
        # and freeing them after that stream is destroyed fails (hipErrorInvalidHandle at exit)
        import gc

        from torch_distributed_sandbox_amd.utils.streams import release_streams

        gc.collect()
        release_streams()


def _attempt(args, world, rank, backend, grad_exchange, reserve, backend_label, store, k, phase):
    """One full benchmark run (init, model, warmup, timed steps) on ``backend``; returns rank 0's
    record (None elsewhere).  The process group is left up for the caller's vote/teardown."""
    import datetime

    import torch.distributed as dist

    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    on_gpu = args.device == "cuda"
    if args.shared_device:
        if backend != "gloo":
            raise SystemExit("bench.py: --shared-device is a rehearsal mode and needs --backend gloo")
        local_rank = 0

    import torch_distributed_sandbox_amd as tds
    from torch_distributed_sandbox_amd.data import synthetic_batch
    from torch_distributed_sandbox_amd.models import ConvNet
    from torch_distributed_sandbox_amd.ops import SGD, CrossEntropyLoss
    from torch_distributed_sandbox_amd.ops import functional as TF
    from torch_distributed_sandbox_amd.parallel import DistributedDataParallel
    from torch_distributed_sandbox_amd.parallel import distributed as tdist
    from torch_distributed_sandbox_amd.parallel.rccl_backend import native_comm_of
    from torch_distributed_sandbox_amd.utils import fault

    phase[0] = f"attempt {k} ({backend}): init"
    fault.maybe_inject_bench(rank, "init")
    if on_gpu:
        assert torch.cuda.is_available(), "bench.py needs a GPU (use --device cpu for a CPU rehearsal)"
        torch.cuda.set_device(local_rank)
        tds._ext.ops()  # native extension must be loaded (fails loudly otherwise)
        device = torch.device("cuda", local_rank)
    else:
        device = torch.device("cpu")
    # CU split for overlapped collectives (parallel/distributed.py init_process_group comm_cus,
    # utils/streams.py, docs/DISTRIBUTED.md): on rccl-native the process group sets it up
    # (default 32 CUs at world > 1); otherwise --reserve-cus masks the compute side only
    if args.rccl_max_ctas > 0:
        os.environ["TDS_RCCL_MAX_CTAS"] = str(args.rccl_max_ctas)
    if store is not None:
        tdist.init_process_group(backend, rank=rank, world_size=world, store=dist.PrefixStore(f"attempt{k}", store),
                                 timeout=datetime.timedelta(seconds=args.pg_timeout),
                                 device_id=local_rank if on_gpu and backend != "gloo" else None,
                                 comm_cus=reserve if backend == "rccl-native" else None)
    if backend == "rccl-native" and tdist.is_initialized():
        reserve = tdist.comm_cus()
    own_split = False
    if backend == "rccl-native" and tdist.is_initialized():
        pass
    elif on_gpu and reserve:
        from torch_distributed_sandbox_amd.utils.streams import reserve_cus_for_comm

        torch.cuda.set_stream(reserve_cus_for_comm(reserve, device))
        own_split = True
    reserve = reserve or 0
    rccl_max_ctas = int(os.environ.get("TDS_RCCL_MAX_CTAS", "0") or 0) if backend == "rccl-native" else 0
    rccl_ranks = None
    if tdist.is_initialized():
        comm, kind = native_comm_of(None)
        if kind == "rccl":
            rccl_ranks = int(comm.comm_count())
        # sanity: one collective over the live communicator before anything is timed
        t = torch.full((1,), float(rank + 1), device=device)
        tdist.all_reduce(t)
        want = world * (world + 1) / 2
        if float(t.item()) != want:
            raise RuntimeError(f"{backend} sanity all-reduce gave {float(t.item())}, expected {want}")

    H = W = args.image_size
    B = args.batch_size
    torch.manual_seed(0)
    phase[0] = f"attempt {k} ({backend}): model"
    model = ConvNet(image_shape=(H, W), device=device, mode=args.mode)
    criterion = CrossEntropyLoss()
    optimizer = SGD(model.parameters(), args.lr)
    ddp = DistributedDataParallel(model, device_ids=[local_rank] if on_gpu else None, bucket_cap_mb=args.bucket_mb,
                                  grad_exchange=grad_exchange, overlap_optimizer=args.overlap_optimizer,
                                  allreduce_chunks=args.allreduce_chunks, exchange_compress=args.exchange_compress,
                                  exchange_groups=args.exchange_groups, exchange_source=args.exchange_source)

    ddp.attach_optimizer(optimizer)

    preflight = None
    if args.preflight and tdist.is_initialized():  # world > 1, or a forced exchange at world 1
        phase[0] = f"attempt {k} ({backend}): preflight"
        preflight, planned = _preflight(ddp, tdist, device, world, rank, B, args.preflight_timeout)
        preflight = {"fc_path": planned, "collectives": preflight}

    # synthetic 28x28 sources + labels, a FRESH batch for every warmup and timed step (as an epoch
    # over the reference's 60 000 MNIST images gives it): with a small pool of repeated batches the
    # 18 M-input fc layer memorises the random labels within ~10 steps at lr 1e-4, the loss reaches
    # 0 and every later backward runs on all-zero gradients -- which the chip executes ~15 % faster
    # (lower MFMA power, higher clock: profiles/r4_data_dependence.md), a number no real epoch has
    pool = max(1, args.warmup + args.steps)
    src_pool, lab_pool = synthetic_batch(B * pool, (H, W), device, seed=1234 + rank)
    src_pool = src_pool.view(pool, B, 28, 28)
    lab_pool = lab_pool.view(pool, B)

    # input pipeline (the role of the reference's DataLoader prefetch): batch i+1 -- the 28x28 ->
    # HxW upsample and, for the fused plan, the batch's x moments behind BN1's statistics
    # (convnet_fused.input_stats: weight-independent) -- is produced on a side stream that starts
    # when step i's head forward is enqueued (--prefetch-at head), so its kernels run beside the
    # memory-bound head forward / backward, whose workgroups leave registers and LDS free, instead
    # of on the step's critical path (beside the conv2 backward, round 2, they got no CU until it
    # ended).  Step i+1's compute stream waits on it; the tensors are
    # recorded on the compute stream so the caching allocator cannot recycle them early.  A step
    # whose hook did not fire (no fused plan, first step) produces its batch inline.  The work per
    # timed step is unchanged: each step produces exactly one batch.
    from torch_distributed_sandbox_amd.models import convnet_fused

    data_stream = torch.cuda.Stream(device) if on_gpu and args.prefetch else None
    with_stats = data_stream is not None and args.mode != "layers"

    fused_moments = on_gpu and args.fused_input_moments and args.input == "levels" and args.mode != "layers"
    fused_ce = on_gpu and args.fused_ce and args.mode != "layers"

    def produce(i):
        if fused_moments:
            # the step's input op with the x moments formed from its levels in the same pass: the layer-1
            # forward then reduces them (no second read of the image); the batch's 45 M pixels and 41
            # products per pixel are computed every step exactly as before
            x, part = TF.upsample_levels_moments(src_pool[i % pool], H, W)
            if part is not None:
                convnet_fused.attach_input_stats(x, (part, None))
            return x
        return TF.upsample_bilinear_u8(src_pool[i % pool], H, W, levels=args.input == "levels")

    pending = {}
    sim_stream = None
    if on_gpu and args.sim_comm_us > 0:
        # on the communication side of the CU split when there is one, as RCCL's kernels would be
        h = tds._ext.ops().cu_comm_stream(device.index) if reserve > 0 else 0
        sim_stream = torch.cuda.ExternalStream(h, device=device) if h else torch.cuda.Stream(device, priority=-1)

    def prefetch(i):
        cur = torch.cuda.current_stream(device)
        data_stream.wait_stream(cur)
        with torch.cuda.stream(data_stream):
            x = produce(i)
            stats = convnet_fused.input_stats(x) if with_stats and not fused_moments else None
        x.record_stream(cur)
        if stats is not None:
            convnet_fused.attach_input_stats(x, stats)
        for t in convnet_fused._take_input_stats(x):
            if t is not None:
                t.record_stream(cur)
        pending[i] = x

    sdma = None
    if on_gpu and args.sim_sdma_mb > 0:
        n = int(args.sim_sdma_mb * 1e6) // 4
        sdma = (torch.cuda.Stream(device), torch.empty(n, device=device), torch.zeros(n, device=device))

    def step(i):
        j = i % pool
        if i in pending:
            images = pending.pop(i)
            torch.cuda.current_stream(device).wait_stream(data_stream)
        else:
            images = produce(i)
        if data_stream is not None:
            hook = (convnet_fused.before_head_forward if args.prefetch_at == "head"
                    else convnet_fused.before_conv2_backward)
            hook(lambda: prefetch(i + 1))
        labels = lab_pool[j]
        if fused_ce:
            # the loss and dlogits formed by the head forward's finalizing workgroup with the logits
            convnet_fused.attach_labels(images, labels)
        out = ddp(images)
        if sim_stream is not None:
            sim_stream.wait_stream(torch.cuda.current_stream(device))
            with torch.cuda.stream(sim_stream):
                tds._ext.ops().comm_spin(out, args.sim_comm_us, args.sim_comm_ctas, 19744)
        if sdma is not None:  # the copy starts when the forward is done and runs beside the backward
            sdma[0].wait_stream(torch.cuda.current_stream(device))
            with torch.cuda.stream(sdma[0]):
                tds._ext.ops().copy_engine(sdma[1], sdma[2], args.sim_sdma_engine == "nocu")
        loss = criterion(out, labels)
        optimizer.zero_grad()
        TF.backward(loss)
        optimizer.step()
        if sdma is not None:
            torch.cuda.current_stream(device).wait_stream(sdma[0])
        if data_stream is not None:
            convnet_fused._before_conv2_backward.clear()  # (a plan without the hook)
            convnet_fused._before_head_forward.clear()
        return loss

    def sync_all():
        # a deferred parameter update (ops/param_fence.py: the exchange's fc step, queued by the
        # next forward) is queued here, so the timed region holds exactly K updates
        if hasattr(ddp, "wait_pending_updates"):
            ddp.wait_pending_updates()
        if world > 1:
            tdist.barrier()
        if on_gpu:
            torch.cuda.synchronize()

    loss = None
    phase[0] = f"attempt {k} ({backend}): warmup"
    for i in range(args.warmup):
        fault.maybe_inject_bench(rank, "step")
        loss = step(i)
    sync_all()
    phase[0] = f"attempt {k} ({backend}): timed steps"
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)] if on_gpu and args.step_times else None
    t0 = time.perf_counter()
    for i in range(args.steps):
        if evs is not None:
            evs[i].record()
        loss = step(args.warmup + i)
    if evs is not None:
        evs[-1].record()
    sync_all()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        tdist.all_reduce(t, tdist.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(loss.item()) if loss is not None else None
    if own_split:
        # the masked streams end with the run, not at process exit (utils/streams.py)
        from torch_distributed_sandbox_amd.utils.streams import release_streams

        release_streams()
    phase[0] = f"attempt {k} ({backend}): report"
    probe = _allreduce_probe(tdist, device, world, on_gpu) if world > 1 and args.allreduce_probe else None
    ms = 1e3 * elapsed / max(1, args.steps)
    imgs_per_sec = world * B * args.steps / elapsed
    if rank == 0:
        config = {
            "model": MODEL,
            "global_batch": world * B,
            "per_rank_batch": B,
            "seq_len": None,
            "image_size": [H, W],
            "parallelism": f"dp{world}",
            "mode": args.mode,
            "device": args.device,
            "backend": (backend_label or backend) if world > 1 else None,
            "attempt": k,
            "rccl_ranks": rccl_ranks,
            "reducer": ddp.reducer_kind,
            "overlap_optimizer": ddp.overlap_optimizer,
            "fc_grad": ddp.fc_grad_path(),
            "allreduce_chunks": ddp.allreduce_chunks,
            "x_exchange": [{"source": ex.source, "last_path": ex.last_path, "ratio": round(ex.x_ratio, 4),
                            **ex.zs_stats} for ex in ddp.exchanges if ex.steps_exchanged] or None,
            "reserve_cus": reserve,
            "prefetch": data_stream is not None,
            # where the batch's x moments (BN1's weight-independent half) are formed: in the upsample's pass
            # over the levels, by the prefetch stream's own kernel, or in the layer-1 forward
            "input_moments": ("upsample" if fused_moments else "prefetch" if with_stats else "layer1_forward"),
            "loss_in_head": fused_ce,
            "prefetch_at": args.prefetch_at if data_stream is not None else None,
            "input": ("uint8 levels (ToTensor's 1/255 folded into conv1)" if args.input == "levels"
                      else "fp32 image"),
            "rccl_max_ctas": rccl_max_ctas or None,
            "optimizer": f"SGD(lr={args.lr:g})",
            "peak_mem_gb": round(torch.cuda.max_memory_allocated(device) / 1e9, 3) if on_gpu else None,
            "final_loss": final_loss,
        }
        if evs is not None:
            config["step_ms"] = [round(evs[i].elapsed_time(evs[i + 1]), 4) for i in range(args.steps)]
        if preflight is not None:
            config["preflight"] = preflight
        if probe is not None:
            config["allreduce_probe"] = probe
        if sdma is not None:
            config["sim_sdma"] = {"MB": args.sim_sdma_mb, "engine": args.sim_sdma_engine}
        if sim_stream is not None:
            config["sim_comm"] = {"us": args.sim_comm_us, "ctas": args.sim_comm_ctas,
                                  "cu_mask_layout": os.environ.get("TDS_CU_MASK_LAYOUT", "striped")}
        if args.shared_device:
            config["shared_device"] = True  # rehearsal: all ranks on one GPU, not a multi-GPU number
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
            "dtype": _dtype(on_gpu),
            "data": DATA,
            "config": config,
        }
        return rec
    return None


if __name__ == "__main__":
    sys.exit(main())
