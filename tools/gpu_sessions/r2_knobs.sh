#!/bin/bash
# A/B knobs: staging load priority (lp3), conv2 forward A-operand ring depth 3 / 5 (fd3, fd5)
set -u
O=gpurun_out/knobs
mkdir -p $O
for v in "" lp3 fd3 fd5 "" lp3 fd3 fd5; do
  TDS_SO_VARIANT=$v timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 --only conv2_fwd,conv2_bwd \
    > $O/t_$v.log 2>&1 || { echo "variant $v rc=$?"; tail -5 $O/t_$v.log; exit 1; }
  echo "variant '$v': $(tail -1 $O/t_$v.log)"
done
for d in 1 3 4; do
  TDS_SO_VARIANT=diag TDS_CONV2_DIAG=$d timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 --only conv2_fwd \
    > $O/fd$d.log 2>&1 || { echo "fwd diag $d rc=$?"; tail -5 $O/fd$d.log; exit 1; }
  echo "fwd diag $d: $(grep conv2_fwd $O/fd$d.log | head -1)"
done
