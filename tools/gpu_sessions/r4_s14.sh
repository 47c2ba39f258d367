#!/bin/bash
# round 4 session 14: the OOM story at HEAD with y2h (the conv2 output now 64 B per pixel): calibrate,
# batch 10 at 23000^2 (expected OOM), batch 5 trains
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4s14
mkdir -p $O
timeout -k 10 900 python3 -u tools/oom_demo.py --image-size 23000 --steps 3 > $O/oom_23000.log 2>&1
rc=$?; tail -n 2 $O/oom_23000.log | cut -c1-1500; exit $rc
