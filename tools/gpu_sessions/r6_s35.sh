#!/bin/bash
# round 6 session 35: the OOM demo at HEAD (fp16 ya: fewer activation bytes per pixel) -- the
# calibration at 3000^2, the batch-10 edge it predicts, bs = 10 must OOM there and bs = 5 train
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s35
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u tools/oom_demo.py > $O/oom.log 2>&1 || { echo "oom demo rc=$?"; tail -5 $O/oom.log; exit 1; }
echo "oom: $(tail -1 $O/oom.log | cut -c1-1800)"
echo done
