#!/bin/bash
# round 4 session 10: where the TF32-class conv2 kernels' time goes -- timing-only DIAG variants of the
# isolated ops at the bench shape (diag build: -DTDS_DIAG), incl. the per-role barrier waits (13)
set -u
O=gpurun_out/r4s10
mkdir -p $O
for d in 0 1 3 5 9 4 13; do
  timeout -k 10 240 env TDS_SO_VARIANT=diag TDS_CONV2_DIAG=$d python3 -u tools/micro/step_ops_timing.py --iters 10 \
    --only conv2_fwd,conv2_bwd > $O/diag_$d.log 2>&1 || { echo "diag $d rc=$?"; tail -5 $O/diag_$d.log; exit 1; }
  echo "diag $d: $(tail -3 $O/diag_$d.log | tr '\n' ' ' | cut -c1-400)"
done
