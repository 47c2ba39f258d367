#!/bin/bash
# round 3 session 10: per-workgroup tile tables (conv2 fwd order, conv2 bwd walk) -- fused-plan
# tests, op timings, backward diag (5 = MFMA waves alone, 13 = barrier clocks), bench
set -u
O=gpurun_out/r3s10
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit 1; }
timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 > $O/ops.log 2>&1 || { echo "ops rc=$?"; tail -5 $O/ops.log; exit 1; }
grep " ms" $O/ops.log
for d in 0 5 13; do
  TDS_SO_VARIANT=diag TDS_CONV2_DIAG=$d timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 --only conv2_bwd \
    > $O/d$d.log 2>&1 || { echo "diag $d rc=$?"; tail -5 $O/d$d.log; exit 1; }
  echo "bwd diag $d: $(grep -E 'conv2_bwd |clock' $O/d$d.log | tr '\n' ' ')"
done
timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
