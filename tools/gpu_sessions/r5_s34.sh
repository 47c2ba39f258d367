#!/bin/bash
# round 5 session 34: border strips as exact u64 atomic sums over the batch, the Gram body's corner
# table formed by the column workgroups before the hand-off; numerics, the reducer in an isolated
# trace, the driver's command
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s34
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t tests 900 tests/test_ups_moments_gpu.py tests/test_fused_gpu.py tests/test_fullscale_plan_gpu.py tests/test_bigimage_gpu.py tests/test_fullscale_gpu.py tests/test_head_ce_gpu.py
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/op -o run -- python3 -u tools/micro/step_ops_timing.py --iters 10 --only ups_mom,l1_fwd_u8 > $O/op.log 2>&1 || { echo "op failed"; tail -5 $O/op.log; exit 1; }
echo "op: $(grep -v amdgpu $O/op.log | grep ms | tr '\n' ' ')"
for i in 1 2; do
  b drv_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
echo done
