#!/bin/bash
# head kernels: block rows per workgroup (2/4/8): isolated op timing, then bench
set -u
O=gpurun_out/hband
mkdir -p $O
for v in "" hb2 hb8; do
  TDS_SO_VARIANT=$v timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 --only head_fwd,head_bwd > $O/t_$v.log 2>&1 || { echo "variant $v rc=$?"; tail -5 $O/t_$v.log; exit 1; }
  echo "variant '$v': $(grep -E 'head_(fwd|bwd)' $O/t_$v.log | head -2 | tr '\n' ' ')"
done
b() {
  local name=$1; shift
  timeout -k 10 150 python -u bench.py "$@" > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -20 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
}
for k in 1 2; do
  b def_$k
  TDS_SO_VARIANT=hb2 b hb2_$k
  TDS_SO_VARIANT=hb8 b hb8_$k
done
