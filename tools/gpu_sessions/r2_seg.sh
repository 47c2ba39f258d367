#!/bin/bash
# conv2 backward segment length A/B (variant builds seg48/96/200 vs default 24)
set -u
O=gpurun_out/seg
mkdir -p $O
for v in "" seg48 seg96 seg200 ""; do
  TDS_SO_VARIANT=$v timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 --only conv2_bwd \
    > $O/t_$v.log 2>&1 || { echo "variant $v rc=$?"; tail -5 $O/t_$v.log; exit 1; }
  echo "variant '$v': $(grep conv2_bwd $O/t_$v.log | head -1)"
done
