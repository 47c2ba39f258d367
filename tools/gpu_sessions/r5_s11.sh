#!/bin/bash
# round 5 session 11: ya encoder with 32-bit page geometry (no 64-bit divisions per piece)
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s11
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t tests 300 tests/test_comm_gpu.py -k "zs_encode or overlap"
OP_ONLY=head_fwd,head_fwd_x,zs_enc_x,zs_enc_ya,dw_zs,head_fwd_upd op xch TDS_SO_VARIANT=
b xa32_off 240 python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5
b xa32_ya 240 env TDS_ZS_FROM_YA=1 python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5
