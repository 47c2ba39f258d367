#!/bin/bash
# round 3 session 12: one code copy per role (conv2 bwd staging waves, conv2 fwd waves: kernel
# code 168 -> 56 KB and 38 -> 10 KB) -- tests, then same-box A/B against the previous build
# (_C_old.so, TDS_SO_VARIANT=old), alternating: op timings and the bench
set -u
O=gpurun_out/r3s12
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit 1; }
for i in 1 2; do
  for v in old new; do
    vv=$v; [ $v = new ] && vv=
    TDS_SO_VARIANT=$vv timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 --only conv2_fwd,conv2_bwd > $O/ops_$v$i.log 2>&1 || { echo "ops rc=$?"; tail -5 $O/ops_$v$i.log; exit 1; }
    echo "$v: $(grep ' ms' $O/ops_$v$i.log | tr '\n' ' ')"
  done
done
for i in 1 2; do
  for v in old new; do
    vv=$v; [ $v = new ] && vv=
    TDS_SO_VARIANT=$vv timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > $O/bench_$v$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_$v$i.log; exit 1; }
    echo "$v: $(tail -1 $O/bench_$v$i.log | cut -c90-190)"
  done
done
