#!/bin/bash
# layer-1 conv workgroups per CU (2/4/6/8): isolated op timing, then bench for the best
set -u
O=gpurun_out/l1wg
mkdir -p $O
for v in "" l1w2 l1w6 l1w8; do
  TDS_SO_VARIANT=$v timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 --only l1_fwd > $O/t_$v.log 2>&1 || { echo "variant $v rc=$?"; tail -5 $O/t_$v.log; exit 1; }
  echo "variant '$v': $(grep l1_fwd $O/t_$v.log | head -1)"
done
b() {
  local name=$1; shift
  timeout -k 10 150 python -u bench.py "$@" > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -20 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
}
for k in 1 2; do
  b def_$k
  TDS_SO_VARIANT=l1w6 b l1w6_$k
  TDS_SO_VARIANT=l1w8 b l1w8_$k
done
