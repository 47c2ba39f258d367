#!/bin/bash
# round 4 session 39: conv2 backward timing-only variants at the round-4 final (diag build):
# 0 full, 1 no MFMAs, 3 no global tile loads, 5 no staging (MFMA waves alone), 9 no BN2/pool
# math in the staging, 13 per-role barrier-wait clocks
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4s39
mkdir -p $O
cd $R
for d in 0 1 3 5 9 13; do
  timeout -k 10 240 env TDS_SO_VARIANT=diag TDS_CONV2_DIAG=$d python3 -u tools/micro/step_ops_timing.py --iters 10 \
    --only conv2_bwd > $O/diag_$d.log 2>&1 || { echo "diag $d rc=$?"; tail -5 $O/diag_$d.log; exit 1; }
  echo "diag $d: $(tail -n 4 $O/diag_$d.log | grep -v amdgpu.ids | tr '\n' ' ' | cut -c1-300)"
done
