#!/bin/bash
# round 6 session 30: the pooled exchange's deferred fc step folded into the head forward
# (TDS_FUSED_PULL, default on) -- kernel and exchange tests, then the forced exchange at W = 1 with
# the fused step vs the separate sweep (TDS_FUSED_PULL=0) and the local step, same box, and a trace
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s30
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t kern 300 tests/test_fused_gpu.py -k "pooled"
t comm 600 tests/test_comm_gpu.py
t multi 600 tests/test_multirank_gpu.py -k "activations"
for i in 1 2; do
  b drv_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  b xf32_$i 240 python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5
  b xs32_$i 240 env TDS_FUSED_PULL=0 python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5
  b xf0_$i 240 python3 -u bench.py --backend rccl-native --reserve-cus 0 --grad-exchange activations --steps 20 --warmup 5
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o xf -- python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5 > $O/prof.log 2>&1
echo "prof rc=$? (the exit abort under rocprofv3 is known; the csv is written before it)"
echo done
