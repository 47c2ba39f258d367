#!/bin/bash
# multi-rank rehearsal on one MI355X (gloo ranks sharing cuda:0): W=2 and W=4 with the default fc path
set -u
O=gpurun_out/rehearse4
mkdir -p $O
for w in 2 4; do
  timeout -k 10 300 python -u bench.py --gpus $w --backend gloo --shared-device --image-size 1024 --steps 5 --warmup 2 > $O/w$w.log 2>&1 || { echo "w$w rc=$?"; tail -30 $O/w$w.log; exit 1; }
  tail -1 $O/w$w.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); c=r["config"]; print(r["n_gpus"], r["value"], r["ms_per_step"], c["fc_grad"], c["final_loss"])'
done
