#!/bin/bash
# CU split with the comm stream confined to the reserved CUs: test, simulated collective beside the step
set -u
O=gpurun_out/cusplit
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_comm_gpu.py -k "cu_reserve" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
b() {
  local name=$1; shift
  timeout -k 10 150 python -u bench.py --steps 60 --warmup 8 "$@" > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -20 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
}
b base
b r32 --reserve-cus 32
for us in 1500 3000 4500; do
  b sim${us}_c32 --sim-comm-us $us --sim-comm-ctas 32
  b sim${us}_c32_r32 --sim-comm-us $us --sim-comm-ctas 32 --reserve-cus 32
done
b r64 --reserve-cus 64
b sim3000_c64_r64 --sim-comm-us 3000 --sim-comm-ctas 64 --reserve-cus 64
