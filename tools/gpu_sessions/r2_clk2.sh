#!/bin/bash
# conv2 backward per-role barrier-wait clocks (diag build, DIAG 13) + diag timings
set -u
O=gpurun_out/clk2
mkdir -p $O
for d in 0 13; do
  TDS_SO_VARIANT=diag TDS_CONV2_DIAG=$d timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 10 --only conv2_bwd \
    > $O/d$d.log 2>&1 || { echo "diag $d rc=$?"; tail -5 $O/d$d.log; exit 1; }
  grep -v amdgpu.ids $O/d$d.log
done
