#!/bin/bash
# round 6 session 25: ya (the pooled conv2 output the head streams) stored in fp16 as the y2h value
# at each window's argmax (half of its 357 MB at the bench shape).  GPU tests of the changed kernels
# and the plan, the driver's command three times, isolated ops, and a kernel trace.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s25
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t fused 400 tests/test_fused_gpu.py
t plan 400 tests/test_fullscale_plan_gpu.py tests/test_fullscale_gpu.py tests/test_model_gpu.py
for i in 1 2 3; do
  b drv_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
OP_ONLY=conv2_fwd,head_fwd,head_bwd op ops TDS_SO_VARIANT=
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o ya16 -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo "prof: $(grep '^{' $O/prof.log | cut -c1-120)"
echo done
