#!/bin/bash
# round 6 session 24: next-batch prefetch beside the layer-1 backward (--prefetch --prefetch-at
# l1_bwd: the 28^2 -> 3000^2 upsample with the x moments of batch i+1 on a side stream, queued when
# step i's layer-1 backward is, so it starts when the conv2 backward ends) against the inline input
# op; the driver's command shape, interleaved, and a kernel trace of the prefetch run
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s24
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
for i in 1 2 3; do
  b base_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  b pf_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --prefetch --prefetch-at l1_bwd
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o pf -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --prefetch --prefetch-at l1_bwd > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo "prof: $(grep '^{' $O/prof.log | cut -c1-120)"
echo done
