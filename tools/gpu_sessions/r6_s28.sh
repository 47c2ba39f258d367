#!/bin/bash
# round 6 session 28: the pooled activation exchange -- the multi-rank test with the fixed
# expectation, the forced exchange at W = 1 against the local step (interleaved, same box), and a
# kernel trace of the forced pooled step with the 32-CU split (where the gathers start)
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s28
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t multi 600 tests/test_multirank_gpu.py -k "activations"
for i in 1 2; do
  b drv_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  b xp32_$i 240 python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5
  b xp0_$i 240 python3 -u bench.py --backend rccl-native --reserve-cus 0 --grad-exchange activations --steps 20 --warmup 5
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o xp -- python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5 > $O/prof.log 2>&1
echo "prof rc=$? (the exit abort under rocprofv3 is known; the csv is written before it)"
echo done
