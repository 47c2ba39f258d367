#!/bin/bash
# round 4 session 22: conv2 forward at 3 workgroups per CU (fp16 staging of the finished tile, 168
# VGPRs; variant wg3) against the default 2 -- the variant's conv2 tests, then isolated conv2
# forward A/B in 3 alternating rounds, then the bench under each
set -u
O=gpurun_out/r4s22
mkdir -p $O
timeout -k 10 300 env TDS_SO_VARIANT=wg3 python -u -m pytest tests/test_fused_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv2 or fused_model" > $O/tests_wg3.log 2>&1
rc=$?; tail -1 $O/tests_wg3.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error|assert" $O/tests_wg3.log | head -30; exit 1; }
for r in 1 2 3; do
  for v in default wg3; do
    V=$v; [ $v = default ] && V=""
    timeout -k 10 120 env TDS_SO_VARIANT=$V python3 -u tools/micro/step_ops_timing.py --iters 20 --only conv2_fwd > $O/${v}_$r.log 2>&1 || { echo "$v rc=$?"; tail -3 $O/${v}_$r.log; exit 1; }
    echo "$v $r $(tail -n 1 $O/${v}_$r.log)"
  done
done
for v in default wg3; do
  V=$v; [ $v = default ] && V=""
  timeout -k 10 200 env TDS_SO_VARIANT=$V python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$v.log 2>&1 || { echo "rc=$?"; exit 1; }
  echo "drv $v: $(tail -1 $O/drv_$v.log | cut -c80-200)"
done
