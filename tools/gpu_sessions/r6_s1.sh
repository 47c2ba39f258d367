#!/bin/bash
# round 6 session 1: lazy fc gradient slot (parallel/ddp.py _lazy_from), store fail-fast, CE label
# guard.  Whole GPU suite + smoke, the driver's command x2, the forced-exchange W=1 step, the OOM demo
# at the new edge.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s1
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t gpu_all 900 tests -m gpu
timeout -k 10 300 python3 -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
echo "smoke: $(tail -1 $O/smoke.log)"
for i in 1 2; do
  b drv_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
echo "peak: $(tail -1 $O/drv_1.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["config"]["peak_mem_gb"])')"
b fx 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --backend rccl-native --reserve-cus 32 --grad-exchange activations
timeout -k 10 600 python3 -u tools/oom_demo.py > $O/oom.log 2>&1 || { echo "oom demo rc=$?"; tail -5 $O/oom.log; exit 1; }
echo "oom: $(tail -1 $O/oom.log)"
echo done
