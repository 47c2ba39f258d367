#!/bin/bash
# A/B: layer-1 conv with unconditional buffer loads/stores (variant l1buf) vs HEAD
set -u
O=gpurun_out/l1ab
mkdir -p $O
for v in "" l1buf "" l1buf; do
  TDS_SO_VARIANT=$v timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 --only l1_fwd,l1_bwd,conv2_bwd \
    > $O/t_$v.log 2>&1 || { echo "variant $v rc=$?"; tail -5 $O/t_$v.log; exit 1; }
  echo "variant '$v': $(tail -1 $O/t_$v.log)"
done
TDS_SO_VARIANT=l1buf timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fused_gpu.py \
  tests/test_bigimage_gpu.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
