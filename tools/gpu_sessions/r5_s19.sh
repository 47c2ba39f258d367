#!/bin/bash
# round 5 session 19: the layer-1 backward reduction + finalize on 54 workgroups (8 columns each): numerics,
# driver's command, trace
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s19
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t tests 600 tests/test_fused_gpu.py tests/test_model_gpu.py tests/test_fullscale_plan_gpu.py tests/test_determinism_gpu.py
for i in 1 2 3; do b drv_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5; done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_drv -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace_drv.log 2>&1
echo "trace_drv rc=$?"
