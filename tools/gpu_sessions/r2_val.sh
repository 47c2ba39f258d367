#!/bin/bash
# HEAD validation: full GPU suite, smoke, bench (default and long timed region)
set -u
O=gpurun_out/val
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 180 python -u bench.py > $O/bench_default.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
timeout -k 10 180 python -u bench.py --steps 200 --warmup 10 > $O/bench_long.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_long.log; exit 1; }
tail -1 $O/bench_long.log
