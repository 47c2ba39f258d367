#!/bin/bash
# update-only fc exchange: comm + multirank tests, compute cost of each path at world 1
set -u
O=gpurun_out/updonly
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_comm_gpu.py tests/test_multirank_gpu.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
b() {
  local name=$1; shift
  timeout -k 10 150 python -u bench.py --steps 60 --warmup 8 --backend rccl-native "$@" > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -20 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); c=r["config"]; print(r["value"], r["ms_per_step"], c["fc_grad"], c["reserve_cus"])')"
}
b local_r32 --reserve-cus 32
for p in activations sharded; do
  b ${p}_r32 --grad-exchange $p --reserve-cus 32
done
