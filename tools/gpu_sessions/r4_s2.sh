#!/bin/bash
# round 4 session 2: the clock ramp -- the driver's command with per-step GPU times, ramp 0 / 100 / 200 / 500 ms
set -u
O=gpurun_out/r4s2
mkdir -p $O
for r in 0 200 100 500 0 200; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --clock-ramp-ms $r --step-times > $O/ramp_$r.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/ramp_$r.log; exit 1; }
  python3 -c "import json,sys; r=json.loads(open('$O/ramp_$r.log').read().strip().splitlines()[-1]); print('ramp', $r, r['ms_per_step'], r['config']['clock_ramp_ms'], r['config']['step_ms'])"
done
