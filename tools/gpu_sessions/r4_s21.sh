#!/bin/bash
# round 4 session 21: head kernels with two alternating load sets; dp1h (the conv2 data gradient stored as scaled fp16 in the dgrad MFMA's layout,
# read by the layer-1 backward) -- fused / model / big-image tests, isolated layer-1 backward at 4 and
# 5 workgroups per CU, two driver-command runs, kernel trace
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4s21
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_fused_gpu.py tests/test_model_gpu.py tests/test_bigimage_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error|assert" $O/tests.log | head -30; exit 1; }
for n in 4 5 4 5; do
  timeout -k 10 120 env TDS_L1B_PER_CU=$n python3 -u tools/micro/step_ops_timing.py --iters 20 --only conv2_bwd,l1_bwd > $O/ops_$n.log 2>&1 || { echo "ops rc=$?"; exit 1; }
  echo "per_cu $n $(tail -n 1 $O/ops_$n.log)"
done
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$i.log 2>&1 || { echo "rc=$?"; exit 1; }
  echo "drv: $(tail -1 $O/drv_$i.log | cut -c80-200)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
echo trace ok
