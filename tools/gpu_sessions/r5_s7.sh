#!/bin/bash
# round 5 session 7: forced activation exchange at W = 1 vs the local step (verdict item 1):
# local step with / without the in-launch finalizers, the exchange with the 32-CU split, without it,
# and with the separate update sweep (TDS_FUSED_FIN=0); kernel traces of the local step and the
# forced exchange; the copy-engine rehearsal (200 MB beside the backward: SDMA vs blit kernel)
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s7
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t tests 300 tests/test_comm_gpu.py
b drv 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
b drv_nofin 200 env TDS_FUSED_FIN=0 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
b xa32 240 python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5
b xa0 240 python3 -u bench.py --backend rccl-native --reserve-cus 0 --grad-exchange activations --steps 20 --warmup 5
b xa32sep 240 env TDS_FUSED_FIN=0 python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5
b sdma_nocu 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --sim-sdma-mb 200 --sim-sdma-engine nocu
b sdma_blit 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --sim-sdma-mb 200 --sim-sdma-engine blit
b drv2 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_drv -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace_drv.log 2>&1 || { echo "trace drv rc=$?"; tail -5 $O/trace_drv.log; exit 1; }
echo "trace_drv ok"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_xa -o run -- \
  python3 $R/bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5 > $O/trace_xa.log 2>&1
echo "trace_xa rc=$?"
