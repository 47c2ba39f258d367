#!/bin/bash
# round 6 session 36: the head kernels with ONE load set (loads right before their use, latency left
# to occupancy: forward 236 -> 140 VGPRs, backward 202 -> 149, 2 -> 3 waves per SIMD) against the
# double-buffered sets, chosen by temporary switches TDS_HEAD_PF_FWD / TDS_HEAD_PF_BWD (0: one set);
# head tests under the new variant, isolated ops and the driver's command, interleaved
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s36
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
timeout -k 10 300 env TDS_HEAD_PF_FWD=0 TDS_HEAD_PF_BWD=0 python -u -m pytest tests/test_fused_gpu.py -k "head" -x -q --timeout 120 --timeout-method thread > $O/kern.log 2>&1
rc=$?; echo "kern rc=$rc: $(tail -1 $O/kern.log)"; if crash_rc $rc; then exit 1; fi
for i in 1 2; do
  OP_ONLY=head_fwd,head_bwd op base_$i TDS_SO_VARIANT=
  OP_ONLY=head_fwd,head_bwd op one_$i TDS_HEAD_PF_FWD=0 TDS_HEAD_PF_BWD=0
done
for i in 1 2; do
  b drv_base_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  b drv_one_$i 200 env TDS_HEAD_PF_FWD=0 TDS_HEAD_PF_BWD=0 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  b drv_fwd1_$i 200 env TDS_HEAD_PF_FWD=0 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
echo done
