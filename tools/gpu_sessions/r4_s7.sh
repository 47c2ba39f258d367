#!/bin/bash
# round 4 session 7: fresh batch every step (no memorised pool) -- the driver's bench command x3 with
# per-step times, lr 0 for comparison, and the split (fp16x2) build A/B on the same box
set -u
O=gpurun_out/r4s7
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --step-times > $O/drv_$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/drv_$i.log; exit 1; }
  python3 -c "import json,sys; r=json.loads(open('$O/drv_$i.log').read().strip().splitlines()[-1]); s=r['config']['step_ms']; print('drv', r['ms_per_step'], r['value'], r['config']['final_loss'], s[:3], s[-3:])"
done
timeout -k 10 200 python -u bench.py --gpus 1 --steps 60 --warmup 5 --step-times > $O/s60.log 2>&1 || { echo "bench rc=$?"; exit 1; }
python3 -c "import json,sys; r=json.loads(open('$O/s60.log').read().strip().splitlines()[-1]); s=r['config']['step_ms']; print('s60', r['ms_per_step'], r['config']['final_loss'], [round(sum(s[i:i+10])/10,3) for i in range(0,60,10)])"
timeout -k 10 300 python -u bench.py > $O/def.log 2>&1 || { echo "bench rc=$?"; exit 1; }
echo "def: $(tail -1 $O/def.log | cut -c80-200)"
