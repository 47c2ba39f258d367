#!/bin/bash
# round 5 session 9: the activation exchange's pieces in isolation (step_ops_timing: head forward
# writing X, encode from X / from ya, the update sweep, the head forward applying the update), the
# forced exchange with the round-5 paths switched on / off, and a trace of the 200 MB copy-engine
# rehearsal (is hipMemcpyDeviceToDeviceNoCU a kernel?)
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s9
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t tests 300 tests/test_comm_gpu.py
OP_ONLY=head_fwd,head_fwd_x,zs_enc_x,zs_enc_ya,dw_zs,head_fwd_upd op xch TDS_SO_VARIANT=
b xa32_off 240 python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5
b xa32_ya 240 env TDS_ZS_FROM_YA=1 python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5
b xa0_off 240 python3 -u bench.py --backend rccl-native --reserve-cus 0 --grad-exchange activations --steps 20 --warmup 5
b drv 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_sdma -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --sim-sdma-mb 200 --sim-sdma-engine nocu > $O/trace_sdma.log 2>&1
echo "trace_sdma rc=$?"
