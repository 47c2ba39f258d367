#!/bin/bash
# round 5 session 41: the loss formed in the head forward on the activation exchange's path too;
# the comm / CE / bench tests, the forced exchange's step
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s41
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t tests 900 tests/test_comm_gpu.py tests/test_head_ce_gpu.py tests/test_bench_gpu.py tests/test_multirank_gpu.py
for i in 1 2; do
  b xa_$i 240 python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5
done
echo done
