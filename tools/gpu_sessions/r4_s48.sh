#!/bin/bash
# round 4 session 48: final validation at HEAD (layer-1 weight gradient at 5 workgroups per CU) -- the whole GPU suite, smoke, the
# driver's command x2, kernel trace of the driver's command, 4 PMC passes of the step,
# python bench.py (100 steps) and mnist_onegpu.py on the same box
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4s48
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -1 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/gpu_tests.log | head -20; exit 1; }
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
echo smoke ok
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$i.log 2>&1 || { echo "rc=$?"; exit 1; }
  echo "drv: $(tail -1 $O/drv_$i.log | cut -c80-200)"
done
timeout -k 10 300 python3 -u bench.py > $O/bench_default.log 2>&1 || { echo "bench rc=$?"; exit 1; }
echo "bench 100: $(tail -1 $O/bench_default.log | cut -c80-200)"
timeout -k 10 300 python3 -u mnist_onegpu.py --epochs 1 --max-steps 100 --json > $O/onegpu.log 2>&1 || { echo "onegpu rc=$?"; tail -5 $O/onegpu.log; exit 1; }
echo "onegpu: $(tail -1 $O/onegpu.log)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
echo "trace ok: $(tail -1 $O/trace.log | cut -c80-200)"
