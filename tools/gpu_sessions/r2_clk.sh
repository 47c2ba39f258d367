#!/bin/bash
# fork/join border strips: tests + bench; conv2 backward barrier-wait clocks (diag build, DIAG 13)
set -u
O=gpurun_out/clk
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_fused_gpu.py \
  tests/test_model_gpu.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 180 python -u bench.py --steps 30 --warmup 5 > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
TDS_SO_VARIANT=diag TDS_CONV2_DIAG=13 timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 1 --only conv2_bwd \
  > $O/clk.log 2>&1 || { echo "clk rc=$?"; tail -5 $O/clk.log; exit 1; }
grep -c BRCLK $O/clk.log
