#!/bin/bash
# round 6 session 11: layer-1 conv epilogue A/B -- pool the accumulators (weights sign-folded by
# BN1's scale) and run the affine once per pooled value (default build) against the per-pixel
# affine (side build _C_l1old.so, -D TDS_L1_OLD); the layer-1 / model GPU tests on the new build
# first
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s11
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t l1 400 tests/test_fused_gpu.py tests/test_model_gpu.py tests/test_fullscale_plan_gpu.py tests/test_ups_moments_gpu.py -m gpu
for v in new old new old; do
  if [ $v = old ]; then V=l1old; else V=; fi
  OP_ONLY=l1_fwd op l1_$v TDS_SO_VARIANT=$V
done
for v in new old new old; do
  if [ $v = old ]; then V=l1old; else V=; fi
  b drv_$v 200 env TDS_SO_VARIANT=$V python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
echo done
