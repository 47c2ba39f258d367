#!/bin/bash
# round 6 session 27: the activation exchange from the pooled input (ya fp16 + 128 head constants
# per rank, gathered right after the conv2 forward; the fc step from them by head_update_pooled).
# Tests, then the forced exchange at W = 1 (pooled vs the zero-suppressed rows, with and without the
# 32-CU split) against the local step, and a kernel trace of the forced pooled step.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s27
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t kern 300 tests/test_fused_gpu.py -k "head_update_pooled or head_forward_backward"
t comm 600 tests/test_comm_gpu.py
t multi 600 tests/test_multirank_gpu.py
b drv_1 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
b xp32_1 240 python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5
b xp0_1 240 python3 -u bench.py --backend rccl-native --reserve-cus 0 --grad-exchange activations --steps 20 --warmup 5
b xr32_1 240 python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --exchange-source rows --steps 20 --warmup 5
b drv_2 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
b xp32_2 240 python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5
b xp0_2 240 python3 -u bench.py --backend rccl-native --reserve-cus 0 --grad-exchange activations --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o xp -- python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5 > $O/prof.log 2>&1
echo "prof rc=$? (the exit abort under rocprofv3 is known; the csv is written before it)"
echo done
