#!/bin/bash
# round 6 session 16: the deferred-update runner keeps its owner visible (__self__) under the weak
# reference -- test_comm_gpu.py again, the driver's command x3 and the end-of-round kernel trace
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s16
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t comm 400 tests/test_comm_gpu.py tests/test_multirank_gpu.py -m gpu
for i in 1 2 3; do
  b drv_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo "prof: $(grep '^{' $O/prof.log | cut -c1-120)"
echo done
