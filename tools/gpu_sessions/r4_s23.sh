#!/bin/bash
# round 4 session 23: conv2 forward at 3 workgroups per CU by default; the level autocorrelation's
# row loop unrolled with branch-free row loads -- fused / model / big-image tests, two
# driver-command runs, kernel trace
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4s23
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_fused_gpu.py tests/test_model_gpu.py tests/test_bigimage_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error|assert" $O/tests.log | head -30; exit 1; }
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$i.log 2>&1 || { echo "rc=$?"; exit 1; }
  echo "drv: $(tail -1 $O/drv_$i.log | cut -c80-200)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
echo trace ok
