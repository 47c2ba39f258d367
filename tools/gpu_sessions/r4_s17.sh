#!/bin/bash
# round 4 session 17: conv2 forward epilogue in packed fp32 (statistics), max |y2 - b2| from the
# accumulator, the argmax nudge behind a wave ballot -- conv2 tests, isolated ops, two
# driver-command runs, kernel trace
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4s17
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv2 or fused_model or head" > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error|assert" $O/tests.log | head -30; exit 1; }
timeout -k 10 240 python3 -u tools/micro/step_ops_timing.py --iters 10 --only conv2_fwd,conv2_bwd > $O/ops.log 2>&1 || { echo "ops rc=$?"; exit 1; }
tail -n 1 $O/ops.log
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$i.log 2>&1 || { echo "rc=$?"; exit 1; }
  echo "drv: $(tail -1 $O/drv_$i.log | cut -c80-200)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
echo trace ok
