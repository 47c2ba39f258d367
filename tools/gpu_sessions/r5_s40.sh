#!/bin/bash
# round 5 session 40: conv2 backward knobs re-swept after the g2m runs (GB): MFMA-wave priority 0 / 1
# (default) / 2, dgrad operand depth 3, staging-load priority 1; isolated op, alternating x2
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s40
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
for r in 1 2; do
  OP_ONLY=conv2_bwd op base_$r TDS_SO_VARIANT=
  OP_ONLY=conv2_bwd op mp0_$r TDS_SO_VARIANT=mp0
  OP_ONLY=conv2_bwd op mp2_$r TDS_SO_VARIANT=mp2
  OP_ONLY=conv2_bwd op dg3_$r TDS_SO_VARIANT=dg3
  OP_ONLY=conv2_bwd op lp1_$r TDS_SO_VARIANT=lp1
done
echo done
