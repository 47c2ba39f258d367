#!/bin/bash
# round 5 session 26: border chunk sums loaded 16 at a time in the Gram body;
# numerics, isolated ops, driver's command, kernel trace
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s26
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t new 600 tests/test_ups_moments_gpu.py tests/test_kernels_gpu.py tests/test_fused_gpu.py -k "upsample or moments or partials or loader or input_stats or levels"
OP_ONLY=ups,moments,ups_mom,l1_fwd_u8 op um
for i in 1 2; do
  b fm_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo "prof: $(grep '^{' $O/prof.log | cut -c1-120)"
echo done
