#!/bin/bash
# round 4 session 16: layer-1 backward prefetch without per-lane branches (its loads were each
# waited for right after issue) -- layer-1 / fused tests, two driver-command runs, kernel trace
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4s16
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "layer1 or fused_model" > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error|assert" $O/tests.log | head -30; exit 1; }
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$i.log 2>&1 || { echo "rc=$?"; exit 1; }
  echo "drv: $(tail -1 $O/drv_$i.log | cut -c80-200)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
echo trace ok
