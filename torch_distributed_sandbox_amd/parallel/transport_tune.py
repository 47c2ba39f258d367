"""Self-tuning of the world > 1 transport configuration on first contact.

The reference's DDP (mnist_distributed.py:67) leaves every transport choice to NCCL.  Here two
knobs decide how the fc exchange's collectives (parallel/factored.py) share the chip with this
package's persistent compute kernels (docs/DISTRIBUTED.md "CU split"):

* ``reserve_cus`` -- CUs split off the compute stream for the communicator's stream
  (utils/streams.py; a multiple of 32, one CU per shader engine);
* ``max_ctas`` -- RCCL's workgroups per collective (``ncclConfig_t.maxCTAs``).

More reserved CUs / CTAs move bytes faster over the 7 xGMI links but leave fewer CUs to the
compute-bound convolutions; none at all lets RCCL's workgroups collide with the persistent
kernels.  Which is best depends on the link bandwidth RCCL reaches on THIS node, which no
one-GPU measurement can give.  So the launcher (bench.py ``--transport-tune``) times the
step's real collectives at each candidate configuration on the live node before the model is
built, and this module predicts the step time of each from those link times and one-GPU
measured compute costs, and picks the fastest:

    step(cfg) = local + exchange + split[reserve] + max(0, link(cfg) - window)
                + interference * link(cfg)           (reserve == 0 only)

``local``: the local step; ``exchange``: what the exchanged step adds on one GPU with the
exchange forced (X encode, update sweep, small collectives); ``split[n]``: the compute cost
of reserving n CUs; ``window``: the part of the step the exchange's gathers overlap;
``interference``: the fraction of an unsplit collective's time the persistent kernels lose to
its workgroups (round 2's spin-kernel rehearsal: a 3 ms collective added 1.44 ms).  Their
values and provenance are in ``DEFAULT_MODEL``; the choice, the measured link times and the
predictions go to bench.py's ``config.preflight.transport``.
"""
from __future__ import annotations

import dataclasses
from typing import Callable, Dict, Iterable, List, Optional


@dataclasses.dataclass(frozen=True)
class TransportConfig:
    reserve_cus: int
    max_ctas: int

    def as_dict(self):
        return {"reserve_cus": self.reserve_cus, "max_ctas": self.max_ctas}


CANDIDATES = (TransportConfig(32, 32), TransportConfig(64, 64), TransportConfig(0, 0))


@dataclasses.dataclass(frozen=True)
class StepModel:
    local_ms: float
    exchange_ms: float
    split_ms: Dict[int, float]
    window_ms: float
    interference: float

    def as_dict(self):
        return {"local_ms": self.local_ms, "exchange_ms": self.exchange_ms,
                "split_ms": {str(k): v for k, v in sorted(self.split_ms.items())},
                "window_ms": self.window_ms, "interference": self.interference}


# One-MI355X measurements at the bench shape (3000^2, batch 5), ms (docs/DISTRIBUTED.md "The pooled
# source"), for the default activation exchange (the pooled input, round 6 end):
#  local 1.93: the driver's command at round-6 HEAD (r6_s25 1.916-1.929, r6_s27 / r6_s28 1.927-1.949);
#  exchange 0.35: the forced pooled exchange with no CU split minus local, same box (r6_s27 +0.30,
#    r6_s28 +0.39, r6_s29 +0.36, r6_s31 +0.33);
#  split[32] 0.14: the forced exchange at --reserve-cus 32 minus 0 (r6_s27 0.19, r6_s28 0.10,
#    r6_s29 0.12, r6_s31 0.15); split[64] 0.30: the zero-suppressed rows' r6s2 fx_64 - fx_0 (not
#    re-measured for the pooled source);
#  window 2.4: the gathers leave ~0.70 ms into the ~2.4 ms step and must land before the next step's
#    update at ~0.69 ms: about one step (profiles/r6_s29_forced_pooled_exchange_kernel_stats.md);
#  interference 0.48: a 3 ms collective of 32 RCCL-sized workgroups beside the unsplit step
#    added 1.44 ms (profiles/r2_cu_split.md).
DEFAULT_MODEL = StepModel(local_ms=1.93, exchange_ms=0.35, split_ms={0: 0.0, 32: 0.14, 64: 0.30},
                          window_ms=2.4, interference=0.48)


def predict_ms(cfg: TransportConfig, link_ms: float, model: StepModel = DEFAULT_MODEL) -> float:
    """Predicted step time (ms) of ``cfg`` whose collectives took ``link_ms`` per step."""
    if cfg.reserve_cus not in model.split_ms:
        # linear in the reserved CUs between the measured points (an unmeasured split)
        pts = sorted(model.split_ms.items())
        lo = max((p for p in pts if p[0] <= cfg.reserve_cus), default=pts[0])
        hi = min((p for p in pts if p[0] >= cfg.reserve_cus), default=pts[-1])
        split = lo[1] if hi[0] == lo[0] else lo[1] + (hi[1] - lo[1]) * (cfg.reserve_cus - lo[0]) / (hi[0] - lo[0])
    else:
        split = model.split_ms[cfg.reserve_cus]
    t = model.local_ms + model.exchange_ms + split + max(0.0, link_ms - model.window_ms)
    if cfg.reserve_cus == 0:
        t += model.interference * link_ms
    return t


def choose(measure: Callable[[TransportConfig], float], model: StepModel = DEFAULT_MODEL,
           candidates: Iterable[TransportConfig] = CANDIDATES) -> dict:
    """Time each candidate with ``measure(cfg) -> link ms per step`` (it may raise: that
    candidate is skipped and its error recorded) and pick the lowest predicted step time (ties:
    the earlier candidate).  Returns {"chosen": cfg dict or None, "candidates": [...],
    "model": ...}; "chosen" is None when no candidate could be measured."""
    rows: List[dict] = []
    best: Optional[TransportConfig] = None
    best_t = float("inf")
    for cfg in candidates:
        row = cfg.as_dict()
        try:
            link = float(measure(cfg))
        except Exception as e:  # noqa: BLE001 -- a configuration this node cannot run
            row["error"] = f"{type(e).__name__}: {str(e)[:200]}"
            rows.append(row)
            continue
        t = predict_ms(cfg, link, model)
        row.update(link_ms=round(link, 4), predicted_step_ms=round(t, 4))
        rows.append(row)
        if t < best_t:
            best, best_t = cfg, t
    return {"chosen": best.as_dict() if best is not None else None,
            "predicted_step_ms": round(best_t, 4) if best is not None else None,
            "candidates": rows, "model": model.as_dict()}


def step_collectives(world: int, rows: int, out_f: int, in_f: int, x_ratio: float = 0.6):
    """(path, [(kind, bytes per rank)]) of the fc exchange ``auto`` picks at this shape
    (parallel/factored.py choose_path): what the probe must move per step."""
    from .factored import choose_path

    path = choose_path(rows, out_f, in_f, world, x_ratio=x_ratio)
    if path == "activations":
        return path, [("all_gather", int(rows * in_f * 4 * x_ratio)), ("all_gather", rows * out_f * 4)]
    if path == "sharded":
        shard = -(-in_f // world)
        return path, [("sendrecv", int(rows * shard * 4 * x_ratio)), ("sendrecv", out_f * shard * 4)]
    return path, [("all_reduce", out_f * in_f * 4)]
