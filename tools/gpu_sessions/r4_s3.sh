#!/bin/bash
# round 4 session 3: is the step-time drift over a run data-dependent (DVFS on the training state)?
# lr 1e-4 (reference) vs lr 0 (stationary weights), 60 steps with per-step GPU times; plus the exchange GPU tests
set -u
O=gpurun_out/r4s3
mkdir -p $O
for lr in 1e-4 0 1e-4 0; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 60 --warmup 5 --lr $lr --step-times > $O/lr_$lr.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/lr_$lr.log; exit 1; }
  python3 -c "import json,sys; r=json.loads(open('$O/lr_$lr.log').read().strip().splitlines()[-1]); s=r['config']['step_ms']; print('lr', '$lr', r['ms_per_step'], r['config']['final_loss'], [round(sum(s[i:i+10])/10,3) for i in range(0,60,10)])"
done
timeout -k 10 600 python -u -m pytest tests/test_comm_gpu.py tests/test_multirank_gpu.py tests/test_bench_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; exit $rc
