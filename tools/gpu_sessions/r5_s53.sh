#!/bin/bash
# round 5 session 53: end-of-round HEAD kernel trace of the driver's command and the 100-step bench
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s53
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo "prof: $(grep '^{' $O/prof.log | cut -c1-100)"
b drv 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
b b100 300 python3 -u bench.py --gpus 1 --steps 100 --warmup 5
echo done
