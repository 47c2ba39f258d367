#!/bin/bash
# round 5 session 10: head forward X stores as 16-B / float2 pieces; the head-fused update with its
# rows' decode loads grouped (HP_MG); exchange pieces in isolation, forced exchange with each path
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s10
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t tests 300 tests/test_comm_gpu.py
OP_ONLY=head_fwd,head_fwd_x,zs_enc_x,zs_enc_ya,dw_zs,head_fwd_upd op xch TDS_SO_VARIANT=
b xa32_off 240 python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5
b xa32_upd 240 env TDS_HEAD_FUSED_UPDATE=1 python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5
b xa0_off 240 python3 -u bench.py --backend rccl-native --reserve-cus 0 --grad-exchange activations --steps 20 --warmup 5
b drv 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
b xa32_ya 240 env TDS_ZS_FROM_YA=1 python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5
b xa32_both 240 env TDS_ZS_FROM_YA=1 TDS_HEAD_FUSED_UPDATE=1 python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5
