#!/bin/bash
# round 3 session 9: fp16x2 conv2 backward / forward timing-only variants (diag build) --
# 0 full, 1 no MFMA, 3 no global loads, 5 no staging, 7 no y2 loads, 9 no BN2/pool math,
# 13 per-role barrier-wait clocks; forward 4 = no y2 stores; plus all ops of the step in isolation
set -u
O=gpurun_out/r3s9
mkdir -p $O
timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 > $O/ops.log 2>&1 || { echo "ops rc=$?"; tail -5 $O/ops.log; exit 1; }
grep " ms" $O/ops.log
for d in 0 1 3 5 7 9 13; do
  TDS_SO_VARIANT=diag TDS_CONV2_DIAG=$d timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 --only conv2_bwd \
    > $O/d$d.log 2>&1 || { echo "diag $d rc=$?"; tail -5 $O/d$d.log; exit 1; }
  echo "bwd diag $d: $(grep -E 'conv2_bwd|clock' $O/d$d.log | tr '\n' ' ')"
done
for d in 0 1 3 4; do
  TDS_SO_VARIANT=diag TDS_CONV2_DIAG=$d timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 --only conv2_fwd \
    > $O/f$d.log 2>&1 || { echo "fdiag $d rc=$?"; tail -5 $O/f$d.log; exit 1; }
  echo "fwd diag $d: $(grep conv2_fwd $O/f$d.log | head -1)"
done
