#!/bin/bash
# round 5 session 8: (1) exchange tests (the head forward applying the exchange's update, the
# vectorised ya encoder at Q = 32 / 50 / 75); (2) the forced exchange at W = 1 with the update fused
# into the head forward (param_fence.take no longer refused by the side stream's event) and the
# 16-B ya loads in the encoder, + trace; (3) conv2 backward staging look-ahead: 3 register sets
# (default build) vs 2 sets (s2) vs 2 sets without the p1-piece rotation (s2r0, the round-4 kernel)
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s8
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t tests 300 tests/test_comm_gpu.py tests/test_fused_gpu.py
b xa32 240 python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5
op s3 TDS_SO_VARIANT=
op s2 TDS_SO_VARIANT=s2
op s2r0 TDS_SO_VARIANT=s2r0
op s3b TDS_SO_VARIANT=
b drv_s3 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
b drv_s2r0 200 env TDS_SO_VARIANT=s2r0 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
b drv_s3b 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
b drv_s2r0b 200 env TDS_SO_VARIANT=s2r0 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_xa -o run -- \
  python3 $R/bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5 > $O/trace_xa.log 2>&1
echo "trace_xa rc=$?"
