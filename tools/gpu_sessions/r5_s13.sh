#!/bin/bash
# round 5 session 13: A/B builds -- g2m stored with plain (temporal) stores so the conv2 backward
# may find it in the Infinity Cache (g2mt), the updated weight with plain stores (wupdt), the
# conv2 backward staging loads at priority 0 (prio0); the full-scale plan test's numbers (-s);
# the PMC counter list of the box
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s13
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
timeout -k 10 300 python -u -m pytest tests/test_fullscale_plan_gpu.py -x -q -s --timeout 240 --timeout-method thread > $O/plan.log 2>&1; echo "plan rc=$?"; grep -E "step [0-9]|benchmarked|passed|failed" $O/plan.log | head -20
OP_ONLY=head_bwd,conv2_bwd op base TDS_SO_VARIANT=
OP_ONLY=head_bwd,conv2_bwd op g2mt TDS_SO_VARIANT=g2mt
OP_ONLY=head_bwd,conv2_bwd op wupdt TDS_SO_VARIANT=wupdt
OP_ONLY=head_bwd,conv2_bwd op prio0 TDS_SO_VARIANT=prio0
for i in 1 2; do
  b base_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  b g2mt_$i 200 env TDS_SO_VARIANT=g2mt python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  b wupdt_$i 200 env TDS_SO_VARIANT=wupdt python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  b prio0_$i 200 env TDS_SO_VARIANT=prio0 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
timeout -k 10 60 rocprofv3 --list-avail > $O/counters.txt 2>&1; echo "list rc=$?"
