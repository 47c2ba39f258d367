#!/bin/bash
# round 6 session 17: the whole GPU suite + smoke at HEAD (r6_s15's run stopped at the deferred-
# runner failure fixed since), the driver's command x2, the OOM demo with the DDP lifetime fix
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s17
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t gpu_all 900 tests -m gpu
timeout -k 10 300 python3 -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
echo "smoke: $(tail -1 $O/smoke.log)"
for i in 1 2; do
  b drv_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
timeout -k 10 900 python3 -u tools/oom_demo.py > $O/oom.log 2>&1 || { echo "oom demo rc=$?"; tail -5 $O/oom.log; exit 1; }
echo "oom: $(tail -1 $O/oom.log | cut -c1-1500)"
echo done
