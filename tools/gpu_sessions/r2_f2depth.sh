#!/bin/bash
# conv2 forward A-fragment ring depth (3/4/5/6): isolated op timing, then bench for the best
set -u
O=gpurun_out/f2depth
mkdir -p $O
for v in "" fd3 fd5 fd6; do
  TDS_SO_VARIANT=$v timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 --only conv2_fwd > $O/t_$v.log 2>&1 || { echo "variant $v rc=$?"; tail -5 $O/t_$v.log; exit 1; }
  echo "variant '$v': $(grep conv2_fwd $O/t_$v.log | head -1)"
done
