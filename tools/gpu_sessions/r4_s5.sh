#!/bin/bash
# round 4 session 5: the fused-model numerics tests (incl. the range guards), then the whole GPU suite,
# smoke, the driver's bench command x2, the lr-0 drift check
set -u
O=gpurun_out/r4s5
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py -m gpu -x -v -s --timeout 120 --timeout-method thread -k "fused_model or conv2" > $O/fused_model.log 2>&1
rc=$?; tail -1 $O/fused_model.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/fused_model.log | head -20; exit 1; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -1 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/gpu_tests.log | head -20; exit 1; }
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
echo smoke ok
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/drv_$i.log; exit 1; }
  echo "drv: $(tail -1 $O/drv_$i.log | cut -c90-200)"
done
for lr in 1e-4 0; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 60 --warmup 5 --lr $lr --step-times > $O/lr_$lr.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/lr_$lr.log; exit 1; }
  python3 -c "import json,sys; r=json.loads(open('$O/lr_$lr.log').read().strip().splitlines()[-1]); s=r['config']['step_ms']; print('lr', '$lr', r['ms_per_step'], r['config']['final_loss'], [round(sum(s[i:i+10])/10,3) for i in range(0,60,10)])"
done
