#!/bin/bash
# round 5 session 21: the s20 order again (fused + plan before the big image: the memory check now
# relative to what the process held at the test's start), then the whole GPU suite + smoke on the
# GB default build, and the driver's command
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s21
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t order 600 tests/test_fused_gpu.py tests/test_fullscale_plan_gpu.py tests/test_bigimage_gpu.py
t gpu_all 900 tests -m gpu
timeout -k 10 300 python3 -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
echo "smoke: $(tail -1 $O/smoke.log)"
for i in 1 2 3; do
  b drv_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
echo done
