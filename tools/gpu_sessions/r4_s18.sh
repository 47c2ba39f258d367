#!/bin/bash
# round 4 session 18: A/B of the conv2 forward epilogue (isolated ops, 3 alternating rounds):
# prev = HEAD before the packed statistics, nob = packed statistics without the tie ballot,
# default = packed statistics + ballot-gated argmax nudge
set -u
O=gpurun_out/r4s18
mkdir -p $O
for r in 1 2 3; do
  for v in prev nob default; do
    V=$v; [ $v = default ] && V=""
    timeout -k 10 120 env TDS_SO_VARIANT=$V python3 -u tools/micro/step_ops_timing.py --iters 20 --only conv2_fwd > $O/${v}_$r.log 2>&1 || { echo "$v rc=$?"; tail -3 $O/${v}_$r.log; exit 1; }
    echo "$v $r $(tail -n 1 $O/${v}_$r.log)"
  done
done
