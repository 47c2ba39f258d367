#!/bin/bash
# round 6 session 22: whole GPU suite + smoke with g2m in fp16 (the big-image bias gradient now
# bounded by dy2's own rounding), the driver's command x2
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s22
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t gpu_all 900 tests -m gpu -s
grep -E "conv2 bias grad|fc tail" $O/gpu_all.log | head -3
timeout -k 10 300 python3 -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
echo "smoke: $(tail -1 $O/smoke.log)"
for i in 1 2; do
  b drv_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
echo done
