#!/bin/bash
# border-strip workgroups merged behind the autocorrelation's in one launch (variant acm) vs two launches
set -u
O=gpurun_out/acmerge
mkdir -p $O
for v in "" acm; do
  TDS_SO_VARIANT=$v timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_fused_gpu.py -k "layer1" > $O/tests_$v.log 2>&1 || { echo "tests $v rc=$?"; tail -20 $O/tests_$v.log; exit 1; }
  TDS_SO_VARIANT=$v timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 --only l1_fwd > $O/t_$v.log 2>&1 || { echo "variant $v rc=$?"; tail -5 $O/t_$v.log; exit 1; }
  echo "variant '$v': $(tail -1 $O/tests_$v.log) $(grep l1_fwd $O/t_$v.log | head -1)"
done
b() {
  local name=$1; shift
  timeout -k 10 150 python -u bench.py "$@" > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -20 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
}
for k in 1 2; do
  b def_$k
  TDS_SO_VARIANT=acm b acm_$k
done
