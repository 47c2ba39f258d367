#!/bin/bash
# round 6 session 43: the rebuilt HEAD extension (after the band switches were removed): fused-kernel
# tests, the smoke and the driver's command
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s43
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t fused 600 tests/test_fused_gpu.py tests/test_fullscale_plan_gpu.py
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc: $(tail -1 $O/smoke.log)"; if crash_rc $rc; then exit 1; fi
b drv_1 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
b drv_2 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
echo done
