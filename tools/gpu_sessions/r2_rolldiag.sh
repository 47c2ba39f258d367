#!/bin/bash
# timing-only variants of the rolling conv2 backward (diag build): 0 full, 1 no MFMA, 3 no
# global loads, 5 no staging, 7 no y2 loads, 9 no BN2/pool math
set -u
mkdir -p gpurun_out/rolldiag
for d in 0 1 3 5 7 9; do
  TDS_SO_VARIANT=diag TDS_CONV2_DIAG=$d timeout -k 10 90 python -u tools/micro/step_ops_timing.py --iters 20 --only conv2_bwd \
    > gpurun_out/rolldiag/d$d.log 2>&1 || { echo "diag $d rc=$?"; tail -5 gpurun_out/rolldiag/d$d.log; exit 1; }
  echo "diag $d: $(grep conv2_bwd gpurun_out/rolldiag/d$d.log | head -1)"
done
