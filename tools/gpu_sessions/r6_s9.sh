#!/bin/bash
# round 6 session 9: head-kernel occupancy A/B (dynamic LDS only to cap workgroups per CU:
# TDS_HEAD_LDS_PAD=<fwd>,<bwd> bytes; 0 = as built, 40000 -> 3 WG/CU, 57344 -> 2, 98304 -> 1),
# isolated ops and the driver's command; the clock warm-up before the warmup steps (per-step times); then the OOM demo with its single-GPU half in a child
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s9
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
for pad in 0,0 40000,40000 57344,57344 98304,98304; do
  OP_ONLY=head_fwd,head_bwd op pad_$pad TDS_HEAD_LDS_PAD=$pad
done
for pad in 0,0 57344,57344 98304,98304 0,0 57344,57344 98304,98304; do
  b drv_$pad 200 env TDS_HEAD_LDS_PAD=$pad python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
for cw in 0 1000 0 1000; do
  b cw_$cw 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --step-times --clock-warmup-ms $cw
  echo "  steps: $(tail -1 $O/cw_$cw.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["config"]["step_ms"])')"
done
timeout -k 10 900 python3 -u tools/oom_demo.py > $O/oom.log 2>&1 || { echo "oom demo rc=$?"; tail -5 $O/oom.log; exit 1; }
echo "oom: $(tail -1 $O/oom.log | cut -c1-900)"
echo done
