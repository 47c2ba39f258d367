#!/bin/bash
# rolling conv2 backward: numerics (fused / model / big-image tests), kernel timing, bench
set -u
mkdir -p gpurun_out/roll
O=gpurun_out/roll
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fused_gpu.py \
  tests/test_model_gpu.py tests/test_bigimage_gpu.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 > $O/ops.log 2>&1 || { echo "ops rc=$?"; tail -20 $O/ops.log; exit 1; }
cat $O/ops.log
timeout -k 10 180 python -u bench.py --steps 30 --warmup 5 > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
