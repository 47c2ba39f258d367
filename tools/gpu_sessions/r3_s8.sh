#!/bin/bash
# round 3 session 8 (re-entry): full GPU suite at HEAD, smoke, 1-GPU bench x2
set -u
O=gpurun_out/r3s8
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -5 $O/tests.log
[ $rc -eq 0 ] || { echo "tests rc=$rc"; grep -E "FAILED|Error" $O/tests.log | head -20; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
echo smoke ok
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > $O/bench_$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_$i.log; exit 1; }
  tail -1 $O/bench_$i.log | cut -c1-200
done
