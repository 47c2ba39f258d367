#!/bin/bash
# round 5 session 15: next-batch prefetch beside the head kernels (bench --prefetch, --prefetch-at
# head) vs none, alternating 3 + 3; a trace of the prefetching step
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s15
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
for i in 1 2 3; do
  b base_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  b pf_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --prefetch
done
b pf100 300 python3 -u bench.py --gpus 1 --steps 100 --warmup 5 --prefetch
b base100 300 python3 -u bench.py --gpus 1 --steps 100 --warmup 5
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_pf -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --prefetch > $O/trace_pf.log 2>&1
echo "trace_pf rc=$?"
