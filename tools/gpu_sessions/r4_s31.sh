#!/bin/bash
# round 4 session 31: the forward stores each pooling window's argmax (a2, 2-bit codes) and the
# conv2 backward routes the pooled gradient by it (no y2h argmax nudge in the forward, no argmax
# recompute in the backward's staging) -- fused/model tests, the driver command x3, kernel trace
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4s31
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/tests.log | head -20; exit 1; }
for i in 1 2 3; do
  timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$i.log 2>&1 || { echo "rc=$?"; tail -5 $O/drv_$i.log; exit 1; }
  echo "drv_$i: $(tail -1 $O/drv_$i.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["value"])')"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
echo trace ok
