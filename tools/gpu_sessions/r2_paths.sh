#!/bin/bash
# compute-side cost of each fc-gradient path at world 1 (process group of one rank, 32 CUs split off)
set -u
O=gpurun_out/paths
mkdir -p $O
b() {
  local name=$1; shift
  timeout -k 10 150 python -u bench.py --steps 60 --warmup 8 --backend rccl-native "$@" > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -20 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); c=r["config"]; print(r["value"], r["ms_per_step"], c["fc_grad"], c["reserve_cus"])')"
}
b local_r0 --reserve-cus 0
b local_r32 --reserve-cus 32
for p in activations sharded chunked allreduce; do
  b ${p}_r32 --grad-exchange $p --reserve-cus 32
done
b sharded_r32_nooverlap --grad-exchange sharded --reserve-cus 32 --no-overlap-optimizer
