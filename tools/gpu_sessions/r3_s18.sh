#!/bin/bash
# round 3 session 18: (a) staging's pooled gradient folded into the FMA constant (_C_fold.so) vs
# the default, same box, alternating; (b) the no-SLP conv2 kernels' timing-only variants
# (diag build: backward 0 full, 1 no MFMA, 3 no global loads, 5 no staging, 9 no BN2 math,
# 13 barrier clocks; forward 0, 1, 3, 4 no y2 stores)
set -u
O=gpurun_out/r3s18
mkdir -p $O
TDS_SO_VARIANT=fold timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py tests/test_fullscale_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests_fold.log 2>&1
rc=$?; tail -1 $O/tests_fold.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests_fold.log | head; exit 1; }
for i in 1 2; do
  for v in def fold; do
    vv=$v; [ $v = def ] && vv=
    TDS_SO_VARIANT=$vv timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 --only conv2_bwd > $O/ops_$v$i.log 2>&1 || { echo "ops rc=$?"; tail -5 $O/ops_$v$i.log; exit 1; }
    echo "$v: $(grep ' ms' $O/ops_$v$i.log | tr '\n' ' ')"
  done
done
for i in 1 2; do
  for v in def fold; do
    vv=$v; [ $v = def ] && vv=
    TDS_SO_VARIANT=$vv timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > $O/bench_$v$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_$v$i.log; exit 1; }
    echo "$v: $(tail -1 $O/bench_$v$i.log | cut -c90-190)"
  done
done
for d in 0 1 3 5 9 13; do
  TDS_SO_VARIANT=diag TDS_CONV2_DIAG=$d timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 --only conv2_bwd \
    > $O/d$d.log 2>&1 || { echo "diag $d rc=$?"; tail -5 $O/d$d.log; exit 1; }
  echo "bwd diag $d: $(grep -E 'conv2_bwd |clock' $O/d$d.log | tr '\n' ' ')"
done
for d in 0 1 3 4; do
  TDS_SO_VARIANT=diag TDS_CONV2_DIAG=$d timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 --only conv2_fwd \
    > $O/f$d.log 2>&1 || { echo "fdiag $d rc=$?"; tail -5 $O/f$d.log; exit 1; }
  echo "fwd diag $d: $(grep conv2_fwd $O/f$d.log | head -1)"
done
