#!/bin/bash
# round 5 session 30: the Gram build with a corner-product table and pipelined strip sums; kernel trace of the layer-1 forward on
# the fused op's partials for the default build, g1 (no Gram body) and g2 (no border workgroups)
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s30
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t tests 900 tests/test_ups_moments_gpu.py tests/test_fused_gpu.py tests/test_fullscale_plan_gpu.py tests/test_bigimage_gpu.py tests/test_fullscale_gpu.py
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base g1 g3 g4; do
  vv=$v; [ $v = base ] && vv=
  TDS_SO_VARIANT=$vv timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 -u tools/micro/step_ops_timing.py --iters 10 --only ups_mom,l1_fwd_u8 > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; exit 1; }
  echo "$v: $(grep -h 'l1_reduce_gram\|ups_moments' $O/$v/run_kernel_stats.csv | cut -d, -f1-5 | tr '\n' ' ' | cut -c1-400)"
done
echo done
