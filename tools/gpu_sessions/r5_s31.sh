#!/bin/bash
# round 5 session 31: the cross-entropy loss formed by the head forward's finalizing workgroup
# (labels attached to the batch); numerics, bench / scripts, the driver's command A/B, kernel trace
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s31
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t tests 900 tests/test_head_ce_gpu.py tests/test_bench_gpu.py tests/test_scripts_gpu.py tests/test_fused_gpu.py tests/test_ups_moments_gpu.py
for i in 1 2; do
  b ce_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  b noce_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-fused-ce
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo "prof: $(grep '^{' $O/prof.log | cut -c1-120)"
echo done
