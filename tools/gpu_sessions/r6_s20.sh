#!/bin/bash
# round 6 session 20: g2m stored in fp16 at a per-channel power-of-two scale (bounded by the head
# forward's max |W| per channel and class; k2, k3 from the stored values' sums): head backward
# backward's staging loads half; GPU tests of the new build, then a same-box A/B against the previous
# HEAD (_C_prev.so, built from git HEAD): isolated head / conv2 backward and the driver's command
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s20
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t g2h 600 tests/test_fused_gpu.py tests/test_model_gpu.py tests/test_fullscale_plan_gpu.py tests/test_determinism_gpu.py tests/test_bigimage_gpu.py tests/test_comm_gpu.py -m gpu
for v in new prev new prev; do
  if [ $v = new ]; then V=; else V=$v; fi
  OP_ONLY=head_bwd,conv2_bwd op ab_$v TDS_SO_VARIANT=$V
done
for v in new prev new prev; do
  if [ $v = new ]; then V=; else V=$v; fi
  b drv_$v 200 env TDS_SO_VARIANT=$V python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
echo done
