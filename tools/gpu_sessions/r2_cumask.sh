#!/bin/bash
# CU-mask layout (striped vs blocked) and a simulated collective's CU footprint beside the step
set -u
O=gpurun_out/cumask
mkdir -p $O
b() {
  local name=$1; shift
  timeout -k 10 150 python -u bench.py --steps 60 --warmup 8 "$@" > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -20 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
}
b base
TDS_CU_MASK_LAYOUT=blocked b r16_blocked --reserve-cus 16
TDS_CU_MASK_LAYOUT=striped b r16_striped --reserve-cus 16
b sim3000_c16 --sim-comm-us 3000 --sim-comm-ctas 16
TDS_CU_MASK_LAYOUT=striped b sim3000_c16_r16_striped --sim-comm-us 3000 --sim-comm-ctas 16 --reserve-cus 16
TDS_CU_MASK_LAYOUT=blocked b sim3000_c16_r16_blocked --sim-comm-us 3000 --sim-comm-ctas 16 --reserve-cus 16
TDS_CU_MASK_LAYOUT=striped b r32_striped --reserve-cus 32
TDS_CU_MASK_LAYOUT=striped b sim3000_c32_r32_striped --sim-comm-us 3000 --sim-comm-ctas 32 --reserve-cus 32
