#!/bin/bash
# round 5 session 42: the fused upsample's vertical taps precomputed one per lane (v_readlane per row)
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s42
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t tests 600 tests/test_ups_moments_gpu.py tests/test_kernels_gpu.py -k "upsample or moments or partials or loader"
for r in 1 2 3; do
  OP_ONLY=ups_mom op um_$r TDS_SO_VARIANT=
done
echo done
