#!/bin/bash
# round 6 session 34: the transport tune on the pooled exchange (forced at W = 1: its probe, the
# refreshed step model and the choice), and the driver's command once more at HEAD
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s34
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
b drv 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
b tune 300 python3 -u bench.py --backend rccl-native --grad-exchange activations --transport-tune --steps 20 --warmup 5
python3 -c "import json; r=json.loads(open('$O/tune.log').read().strip().splitlines()[-1]); t=r['config']['preflight'].get('transport'); print('transport:', json.dumps(t)[:900])"
echo done
