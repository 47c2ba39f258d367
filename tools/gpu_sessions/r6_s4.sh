#!/bin/bash
# round 6 session 4: the multi-GPU pieces measurable on one MI355X at HEAD -- the forced activation
# exchange at reserve 0 / 32 (the split costs parallel/transport_tune.py uses), the transport tune at
# W=1, and the OOM demo (bs 10 fails / bs 5 trains) with the lazy fc gradient slot.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s4
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
b drv 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
for r in 0 32; do
  b fx_$r 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --backend rccl-native --reserve-cus $r --grad-exchange activations
done
b tune 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --backend rccl-native --grad-exchange activations --transport-tune
echo "tune: $(tail -1 $O/tune.log | python3 -c 'import json,sys; c=json.loads(sys.stdin.read())["config"]; print(c.get("store"), json.dumps(c["preflight"].get("transport")))')"
timeout -k 10 600 python3 -u tools/oom_demo.py > $O/oom.log 2>&1 || { echo "oom demo rc=$?"; tail -5 $O/oom.log; exit 1; }
echo "oom: $(tail -1 $O/oom.log)"
echo done
