#!/bin/bash
# round 5 session 54: HEAD validation after the conv2 packing max loads were clamped:
# whole GPU suite + smoke, the driver's command x2
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s54
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t gpu_all 900 tests -m gpu
timeout -k 10 300 python3 -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
echo "smoke: $(tail -1 $O/smoke.log)"
for i in 1 2; do
  b drv_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
echo done
