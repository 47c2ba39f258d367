#!/bin/bash
# round 5 session 16: conv2 backward staging with 8-channel items (cw8 build: 16-B y2h loads and
# dy2 stores, 160 items per tile) vs 4-channel items (default build): numerics of both, isolated
# op and the driver's command alternating; then the full GPU suite on the default build
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s16
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
export TDS_SO_VARIANT=cw8
t fused_cw8 300 tests/test_fused_gpu.py -k "conv2_backward or fused_model"
unset TDS_SO_VARIANT
OP_ONLY=conv2_bwd op base TDS_SO_VARIANT=
OP_ONLY=conv2_bwd op cw8 TDS_SO_VARIANT=cw8
for i in 1 2 3; do
  b base_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  b cw8_$i 200 env TDS_SO_VARIANT=cw8 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
t gpu_all 900 tests -m gpu
