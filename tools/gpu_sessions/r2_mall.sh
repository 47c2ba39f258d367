#!/bin/bash
# MALL reuse: ya plain stores (+ fc weight loads non-temporal in the head kernels) vs default; bench A/B
set -u
O=gpurun_out/mall
mkdir -p $O
b() {
  local name=$1; shift
  timeout -k 10 150 python -u bench.py --steps 100 --warmup 10 "$@" > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -20 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
}
for k in 1 2 3; do
  b def_$k
  TDS_SO_VARIANT=mall b mall_$k
  TDS_SO_VARIANT=yaplain b yaplain_$k
done
