#!/bin/bash
# round 5 session 12: small-kernel latency fixes (l1_gram / l1_finalize inputs staged in LDS,
# reduce_partials loads in flight together); A/B of the in-launch finalizers on the driver's
# command (alternating, 3 each) and of the layer-1 in-launch finalize; kernel trace
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s12
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t tests 400 tests/test_fused_gpu.py tests/test_model_gpu.py
OP_ONLY=l1_fwd,l1_bwd op l1 TDS_SO_VARIANT=
OP_ONLY=l1_fwd,l1_bwd op l1fin TDS_FUSED_FIN_L1=1
for i in 1 2 3; do
  b drv_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  b nofin_$i 200 env TDS_FUSED_FIN=0 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_drv -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace_drv.log 2>&1
echo "trace_drv rc=$?"
