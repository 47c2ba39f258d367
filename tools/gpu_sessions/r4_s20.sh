#!/bin/bash
# round 4 session 20: same-box A/B of the layer-1 conv change (l1prev = HEAD's layer-1 kernels,
# default = wave-uniform fast/slow epilogue + unconditional prefetch), isolated layer-1 ops,
# 3 alternating rounds
set -u
O=gpurun_out/r4s20
mkdir -p $O
for r in 1 2 3; do
  for v in l1prev default; do
    V=$v; [ $v = default ] && V=""
    timeout -k 10 120 env TDS_SO_VARIANT=$V python3 -u tools/micro/step_ops_timing.py --iters 20 --only l1_fwd,l1_bwd > $O/${v}_$r.log 2>&1 || { echo "$v rc=$?"; tail -3 $O/${v}_$r.log; exit 1; }
    echo "$v $r $(tail -n 1 $O/${v}_$r.log)"
  done
done
