#!/bin/bash
# per-op times of the step on CU-masked streams (reserve 0 / 16 / 32, striped mask)
set -u
O=gpurun_out/cuprobe2
mkdir -p $O
for r in 0 16 32; do
  timeout -k 10 150 python -u tools/micro/step_ops_timing.py --iters 10 --reserve-cus $r > $O/ops_r$r.log 2>&1 || { echo "r$r rc=$?"; tail -20 $O/ops_r$r.log; exit 1; }
  echo "== reserve $r"; cat $O/ops_r$r.log | tail -25
done
