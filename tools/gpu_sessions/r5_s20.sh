#!/bin/bash
# round 5 session 20: conv2 backward staging with g2m by runs through an LDS tile (GB, default
# build) vs per-item g2m loads (gb0): numerics (fused, plan, big-image), isolated op, driver's
# command alternating
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s20
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t tests 900 tests/test_fused_gpu.py tests/test_fullscale_plan_gpu.py tests/test_bigimage_gpu.py tests/test_model_gpu.py
OP_ONLY=conv2_bwd op gb TDS_SO_VARIANT=
OP_ONLY=conv2_bwd op gb0 TDS_SO_VARIANT=gb0
for i in 1 2 3; do
  b gb_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  b gb0_$i 200 env TDS_SO_VARIANT=gb0 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
