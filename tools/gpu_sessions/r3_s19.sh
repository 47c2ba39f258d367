#!/bin/bash
# round 3 session 19 (re-entry after a container rebuild): rebuilt tree validated on MI355X --
# full GPU suite, smoke, then the 1-GPU bench twice
set -u
O=gpurun_out/r3s19
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gpu_tests.log | head; exit 1; }
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
echo smoke ok
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > $O/bench_$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_$i.log; exit 1; }
  echo "bench $i: $(tail -1 $O/bench_$i.log | cut -c90-200)"
done
