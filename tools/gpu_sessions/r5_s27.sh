#!/bin/bash
# round 5 session 27: the Gram body's inputs staged by every workgroup of the reducer's launch at its
# start, column sums with 16 loads in flight; numerics (layer-1, fused, plan, big image), driver's
# command, kernel trace
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s27
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t new 900 tests/test_ups_moments_gpu.py tests/test_fused_gpu.py tests/test_fullscale_plan_gpu.py tests/test_bigimage_gpu.py tests/test_model_gpu.py
for i in 1 2; do
  b fm_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo "prof: $(grep '^{' $O/prof.log | cut -c1-120)"
echo done
