#!/bin/bash
# round 4 session 19: layer-1 conv with a wave-uniform fast/slow epilogue and unconditional
# prefetch -- layer-1 / fused tests, two driver-command runs, kernel trace, then the conv2
# backward's timing-only DIAG variants after the staging-loop fix
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4s19
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "layer1 or fused_model or conv2" > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error|assert" $O/tests.log | head -30; exit 1; }
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$i.log 2>&1 || { echo "rc=$?"; exit 1; }
  echo "drv: $(tail -1 $O/drv_$i.log | cut -c80-200)"
done
for d in 0 1 3 5 7 9 13; do
  timeout -k 10 240 env TDS_SO_VARIANT=diag TDS_CONV2_DIAG=$d python3 -u tools/micro/step_ops_timing.py --iters 10 \
    --only conv2_bwd > $O/diag_$d.log 2>&1 || { echo "diag $d rc=$?"; tail -5 $O/diag_$d.log; exit 1; }
  echo "diag $d: $(tail -n 4 $O/diag_$d.log | grep -v amdgpu.ids | tr '\n' ' ' | cut -c1-300)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
echo trace ok
