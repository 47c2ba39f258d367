#!/bin/bash
# round 5 session 23: the upsample fused with the x moments' partials (ups_moments.hip) and the
# border strips inside the layer-1 reducer's launch (xmom_u8.h): numerics, isolated ops, the
# driver's command with and without the fused input moments, a kernel trace
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s23
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t new 300 tests/test_ups_moments_gpu.py tests/test_kernels_gpu.py -k "upsample or moments or partials"
t fused 600 tests/test_fused_gpu.py tests/test_fullscale_plan_gpu.py tests/test_bench_gpu.py
OP_ONLY=ups,moments,ups_mom,l1_fwd_u8,l1_fwd_u8_self op um
for i in 1 2; do
  b fm_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  b nofm_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-fused-input-moments
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo "prof: $(tail -1 $O/prof.log | cut -c1-200)"
echo done
